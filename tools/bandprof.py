"""Phase clocks of k_bin_band in a -DPRK_WPROF=1 build (make variant_all
NAME=wprof VARIANT=-DPRK_WPROF=1): rank 0's band of an N-way row split, as
tools/band_frames.py draws it, counters summed over the timed frames.
usage: PRK_LIB=cpu-renderer_amd/libprk_hip_wprof.so python tools/bandprof.py <c3b|c5> <N> [frames]"""
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
n = int(sys.argv[3]) if len(sys.argv) > 3 else 10
W, H = cfg["W"], cfg["H"]
s = scenes.random_soup(cfg["T"], W, H, radius=cfg["radius"], seed=cfg["seed"])
r = prk.Renderer(0)
row0, row1 = prk.band_rows(H, 0, N)
r.target_alloc(W, H, row0, row1)
r.set_camera(s.prk_transform(), s.prk_lights())
g = r.geometry(s.vertices, None, s.normals, s.uvs)
tex = r.texture(s.texture)
zmin = -float(np.finfo(np.float32).max)


def frame():
    r.clear_on_flush(0xFF000000, zmin)
    r.draw_model_optimized(g, s.tri_count, bitmap=tex)
    r.complete_all_work()
    r.synchronize()


for _ in range(3):
    frame()
r.timing_reset()
# one frame at a time: the launch window (counters 8, 9) is one frame's
names = ["first half in", "first half tested", "second half in", "second half tested", "lists joined",
         "records (in k_bin_band only with -DPRK_BAND_REC_KERNEL=0)"]
tot = np.zeros(16)
span = 0.0
for _ in range(n):
    r.timing_reset()
    frame()
    c = np.array([int(x) for x in r.debug_counters(16)], dtype=np.float64)
    tot += c
    first = (~int(c[8])) & (2 ** 64 - 1)
    span += (int(c[9]) - first) / 100.0  # s_memrealtime: 100 MHz
wgs = tot[6]
print("%s N=%d: %d workgroups a frame, %.0f listed triangles each" % (sys.argv[1], N, wgs / n, tot[7] / wgs))
print("  first workgroup start -> last workgroup end: %.1f us a frame" % (span / n))
print("  one workgroup start -> end: %.1f us on average" % (tot[10] / wgs / 100.0))
for k, nm in enumerate(names):
    print("  %-20s %8.0f clocks" % (nm, tot[k] / wgs))
