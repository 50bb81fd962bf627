"""Do speculative chunk starts converge for a huge object's AET?  Builds
tools/chunk_conv.c and runs it on FillEdgeTable's edges (the C oracle) of a
C3b-density soup as ONE object: 1024 x 512 px, 31,250 triangles of radius 16
(C3b's 1 M on 4096^2 per pixel; the list is a quarter of C3b's as long).
usage: python tools/chunk_conv.py [W H tris radius]"""
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cpu-renderer_amd"))
sys.path.insert(0, ROOT)
from oracle import oracle as O  # noqa: E402
from prk import scenes  # noqa: E402

W, H, T, rad = ([int(x) for x in sys.argv[1:5]] + [1024, 512, 31250, 16][len(sys.argv[1:5]):])
s = scenes.random_soup(T, W, H, radius=rad, seed=2024)
w = O.fill_edge_table_words(s, 0, s.tri_count)
f = w.view(np.float32)
i32 = w.view(np.int32)
rec = np.zeros(w.shape[0], dtype=[("X", "<f4"), ("G", "<f4"), ("Left", "<i4"), ("YMin", "<i4"), ("YMax", "<i4")])
rec["X"], rec["G"], rec["Left"], rec["YMin"], rec["YMax"] = f[:, 1], f[:, 4], i32[:, 12], i32[:, 7], i32[:, 0]
exe = "/tmp/chunk_conv"
subprocess.check_call(["gcc", "-O2", "-ffp-contract=off", "-o", exe, os.path.join(ROOT, "tools", "chunk_conv.c")])
inp = np.array([w.shape[0], H], np.int32).tobytes() + rec.tobytes()
print(subprocess.run([exe], input=inp, capture_output=True, check=True).stdout.decode())
