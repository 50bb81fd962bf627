"""Per-rank frame time of an N-GPU row-band split, measured on one GPU: the
C3b scene drawn into band [0, H/N) only, back-to-back fused-clear frames (the
bench's loop without the gather).  usage:
    python tools/time_band.py N [tile ...]      e.g. 8 256x8 128x8
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cpu-renderer_amd"))
import numpy as np  # noqa: E402

import prk  # noqa: E402
from prk import scenes  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 8
tiles = sys.argv[2:] or ["256x8"]
W = H = 4096
s = scenes.random_soup(1_000_000, W, H, radius=16, seed=2024)
zmin = -float(np.finfo(np.float32).max)
for tile in tiles:
    r = prk.Renderer(0)
    r.target_alloc(W, H, 0, H // N)
    r.set_tile(*[int(x) for x in tile.split("x")])
    r.set_camera(s.prk_transform(), s.prk_lights())
    g = r.geometry(s.vertices, None, s.normals, s.uvs)
    tex = r.texture(s.texture)
    host = 0.0
    for i in range(23):
        if i == 3:
            r.synchronize()
            t0 = time.perf_counter()
            host = 0.0
        h0 = time.perf_counter()
        r.clear_on_flush(0xFF000000, zmin)
        r.draw_model_optimized(g, s.tri_count, bitmap=tex)
        r.complete_all_work()
        host += time.perf_counter() - h0
    r.synchronize()
    ms = (time.perf_counter() - t0) * 1e3 / 20
    print("N=%d band rows %d tile %s: %.3f ms/frame per rank (x%d ranks -> %.0f Mpixels/s before the gather); "
          "host time in the draw calls %.3f ms/frame" % (N, H // N, tile, ms, N, W * H / (ms * 1e-3) / 1e6,
                                                        host * 1e3 / 20), flush=True)
    r.close()
