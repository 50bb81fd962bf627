"""Per-rank frame time of an N-GPU row-band split, measured on one GPU: the
scene drawn into band [0, H/N) only (rank 0's band; every band of these
uniform soups carries the same load), back-to-back fused-clear frames (the
bench's loop without the gather), plus the serial per-stage kernel times of
that band (host waits after each frame).
usage:
    python tools/time_band.py [--scene c3b|c5] [--n 1,2,4,8] [--tile 256x8] [--json out.json]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cpu-renderer_amd"))
import numpy as np  # noqa: E402

import prk  # noqa: E402
from prk import scenes  # noqa: E402

SCENES = {
    "c3b": dict(T=1_000_000, W=4096, H=4096, radius=16, seed=2024),
    "c5": dict(T=1_000_000, W=8192, H=8192, radius=32, seed=5),
}

ap = argparse.ArgumentParser()
ap.add_argument("--scene", default="c3b", choices=sorted(SCENES))
ap.add_argument("--n", default="1,2,4,8")
ap.add_argument("--tile", default="")
ap.add_argument("--frames", type=int, default=200)  # (20 frames read 0.257 ms at C3b N = 8, 200 0.197: fill and first frames)
ap.add_argument("--json", default="")
a = ap.parse_args()
cfg = SCENES[a.scene]
W, H = cfg["W"], cfg["H"]
s = scenes.random_soup(cfg["T"], W, H, radius=cfg["radius"], seed=cfg["seed"])
zmin = -float(np.finfo(np.float32).max)
out = []
for N in [int(x) for x in a.n.split(",")]:
    r = prk.Renderer(0)
    row0, row1 = prk.band_rows(H, 0, N)
    r.target_alloc(W, H, row0, row1)
    if a.tile:
        r.set_tile(*[int(x) for x in a.tile.split("x")])
    r.set_camera(s.prk_transform(), s.prk_lights())
    g = r.geometry(s.vertices, None, s.normals, s.uvs)
    tex = r.texture(s.texture)

    def frame():
        r.clear_on_flush(0xFF000000, zmin)
        r.draw_model_optimized(g, s.tri_count, bitmap=tex)
        r.complete_all_work()

    for _ in range(10):
        frame()
    r.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.frames):
        frame()
    r.synchronize()
    ms = (time.perf_counter() - t0) * 1e3 / a.frames
    serial = {k: [] for k in ("bin", "vis", "walk", "pix", "frame_wall")}
    for _ in range(5):
        r.timing_reset()
        t1 = time.perf_counter()
        frame()
        r.synchronize()
        serial["frame_wall"].append((time.perf_counter() - t1) * 1e3)  # (host calls + GPU, nothing overlapping)
        st = r.stats()
        serial["bin"].append(st["sum_ms_bin"])
        serial["vis"].append(st["sum_ms_vis"])
        serial["walk"].append(st["sum_ms_span"])
        serial["pix"].append(st["sum_ms_raster"] - st["sum_ms_vis"] - st["sum_ms_span"])
    ser = {k: float(np.median(v)) for k, v in serial.items()}
    rec = dict(scene=a.scene, n=N, band_rows=[row0, row1], tile=a.tile or "auto", ms_per_frame_rank=ms,
               projected_mpixels_s_before_gather=W * H / (ms * 1e-3) / 1e6, serial_ms=ser,
               bin_entries=int(r.stats()["bin_entries"]))
    out.append(rec)
    print(json.dumps(rec), flush=True)
    r.close()
if a.json:
    with open(a.json, "w") as f:
        json.dump(out, f, indent=1)
