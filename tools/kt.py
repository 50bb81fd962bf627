"""Serial per-stage kernel times of one scene config (A/B experiments).

Frames as bench.py runs them (fused clear, one draw of the whole soup), but
the host waits after every frame, so no kernel overlaps another frame's and
the HIP-event stage times (prk_stats) are serial durations.
usage: PRK_LIB=... python tools/kt.py [tris W H radius frames tile]"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cpu-renderer_amd"))
import prk  # noqa: E402
from prk import scenes  # noqa: E402

a = sys.argv[1:]
T = int(a[0]) if len(a) > 0 else 1_000_000
W = int(a[1]) if len(a) > 1 else 4096
H = int(a[2]) if len(a) > 2 else 4096
R = float(a[3]) if len(a) > 3 else 16.0
n = int(a[4]) if len(a) > 4 else 10
tile = a[5] if len(a) > 5 else ""
s = scenes.random_soup(T, W, H, radius=R, seed=2024)
r = prk.Renderer(0)
r.target_alloc(W, H)
if tile:
    r.set_tile(*[int(x) for x in tile.split("x")])
r.set_camera(s.prk_transform(), s.prk_lights())
g = r.geometry(s.vertices, None, s.normals, s.uvs)
tex = r.texture(s.texture)
zmin = -float(np.finfo(np.float32).max)
rows = {k: [] for k in ("bin", "vis", "walk", "pix", "frame")}
for i in range(n + 2):
    r.timing_reset()
    t0 = time.perf_counter()
    r.clear_on_flush(0xFF000000, zmin)
    r.draw_model_optimized(g, T, bitmap=tex)
    r.complete_all_work()
    r.synchronize()
    dt = time.perf_counter() - t0
    st = r.stats()
    if i < 2:
        continue
    rows["bin"].append(st["sum_ms_bin"])
    rows["vis"].append(st["sum_ms_vis"])
    rows["walk"].append(st["sum_ms_span"])
    rows["pix"].append(st["sum_ms_raster"] - st["sum_ms_vis"] - st["sum_ms_span"])
    rows["frame"].append(dt * 1e3)
m = {k: float(np.median(v)) for k, v in rows.items()}
print("lib=%s T=%d %dx%d R=%g tile=%s serial ms: bin %.3f vis %.3f walk %.3f pix %.3f | sum %.3f host-frame %.3f"
      % (os.path.basename(prk.LIB_PATH), T, W, H, R, tile or "default", m["bin"], m["vis"], m["walk"], m["pix"],
         m["bin"] + m["vis"] + m["walk"] + m["pix"], m["frame"]), flush=True)
