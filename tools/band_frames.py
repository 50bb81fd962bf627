"""Serial band frames for rocprofv3 --kernel-trace --stats: rank 0's band of
an N-way row split (as tools/time_band.py draws it), the host waiting after
every frame, so each kernel's duration is its own (no other frame overlaps).
usage: python tools/band_frames.py <c3b|c5> <N> [frames]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cpu-renderer_amd"))
import numpy as np  # noqa: E402

import prk  # noqa: E402
from prk import scenes  # noqa: E402

SCENES = {"c3b": dict(T=1_000_000, W=4096, H=4096, radius=16, seed=2024),
          "c5": dict(T=1_000_000, W=8192, H=8192, radius=32, seed=5)}
cfg = SCENES[sys.argv[1]]
N = int(sys.argv[2])
n = int(sys.argv[3]) if len(sys.argv) > 3 else 20
W, H = cfg["W"], cfg["H"]
s = scenes.random_soup(cfg["T"], W, H, radius=cfg["radius"], seed=cfg["seed"])
r = prk.Renderer(0)
row0, row1 = prk.band_rows(H, 0, N)
r.target_alloc(W, H, row0, row1)
r.set_camera(s.prk_transform(), s.prk_lights())
g = r.geometry(s.vertices, None, s.normals, s.uvs)
tex = r.texture(s.texture)
zmin = -float(np.finfo(np.float32).max)
for _ in range(n):
    r.clear_on_flush(0xFF000000, zmin)
    r.draw_model_optimized(g, s.tri_count, bitmap=tex)
    r.complete_all_work()
    r.synchronize()
print("band frames done: %s N=%d rows [%d, %d) x %d" % (sys.argv[1], N, row0, row1, n))
