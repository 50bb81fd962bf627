"""Time k_raster / k_bin on one scene config (A/B experiments).
usage: PRK_LIB=... python tools/time_frame.py [tris W H radius steps tile]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cpu-renderer_amd"))
import prk  # noqa: E402
from prk import scenes  # noqa: E402

a = sys.argv[1:]
T = int(a[0]) if len(a) > 0 else 1_000_000
W = int(a[1]) if len(a) > 1 else 4096
H = int(a[2]) if len(a) > 2 else 4096
R = float(a[3]) if len(a) > 3 else 16.0
steps = int(a[4]) if len(a) > 4 else 10
tile = a[5] if len(a) > 5 else ""
s = scenes.random_soup(T, W, H, radius=R, seed=2024)
r = prk.Renderer(0)
r.target_alloc(W, H)
if tile:
    r.set_tile(*[int(x) for x in tile.split("x")])
r.set_camera(s.prk_transform(), s.prk_lights())
g = r.geometry(s.vertices, None, s.normals, s.uvs)
tex = r.texture(s.texture)
for i in range(steps + 2):
    if i == 2:
        r.synchronize()
        r.timing_reset()
        t0 = time.perf_counter()
    r.clear()
    r.draw_model_optimized(g, T, bitmap=tex)
    r.complete_all_work()
r.synchronize()
dt = (time.perf_counter() - t0) / steps
st = r.stats()
n = max(1, st["frames_timed"])
print("lib=%s T=%d %dx%d R=%g tile=%s: frame %.3f ms  bin %.3f ms  raster %.3f ms (vis %.3f shade %.3f [span %.3f])  "
      "entries %d anomalies %d slow_replays %d" % (
          os.path.basename(prk.LIB_PATH), T, W, H, R, tile or "default", dt * 1e3, st["sum_ms_bin"] / n,
          st["sum_ms_raster"] / n, st["sum_ms_vis"] / n, (st["sum_ms_raster"] - st["sum_ms_vis"]) / n,
          st["sum_ms_span"] / n,
          st["bin_entries"], st["anomalies"], st["slow_replays"]))
if os.environ.get("PRK_PROF_PRINT"):
    c = r.debug_counters(16)
    for name, off in (("vis", 0), ("shade", 4)):
        tot = sum(c[off:off + 4]) or 1
        print("  %-5s cycles: setup %.3g (%.0f%%)  walk %.3g (%.0f%%)  scan %.3g (%.0f%%)  items %.3g (%.0f%%)" % (
            (name,) + tuple(v for k in range(4) for v in (c[off + k], 100.0 * c[off + k] / tot))))
    f = float(steps)
    ch, it, win, items, act, sp = [c[8 + k] / f for k in range(6)]
    print("  vis events per frame: chunks %.0f  row iterations %.0f (%.2f per chunk)  item windows %.0f "
          "(%.2f per iteration)  items %.0f (%.1f per window)  active lanes %.1f per iteration  spans with items %.0f"
          % (ch, it, it / max(ch, 1), win, win / max(it, 1), items, items / max(win, 1), act / max(it, 1), sp))
