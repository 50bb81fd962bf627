"""Frame times of every BASELINE.json config on one MI355X (GPU box).

bench.py measures the headline config (C3b); this times the others the same
way (inputs resident in HBM, clear fused into the frame where the frame
shades through span records, HIP-event kernel split from prk_get_stats) and
writes one JSON object per config:

    python tools/bench_configs.py [out.json]

C1  1 triangle, 256^2, scalar Gouraud (the CPU plumbing case, timed anyway)
C2  displaced-sphere bunny stand-in (~70k tris), 1920x1080, untextured Phong (scalar)
C3a 1M random tris, 4096^2, Gouraud colour interpolation (scalar)
C3b 1M random tris, 4096^2, Phong + texture (FillLineOptimized) -- bench.py's line
C4  Sponza-style atrium (~250k tris, 8 textures 1024^2), 3840x2160, Phong,
    nearest (the reference's sampling) and bilinear (extension)
C5  1M tris (offsets +-32 px), 8192^2, one GPU (the 8-GPU case shards this by rows)
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cpu-renderer_amd"))
import prk  # noqa: E402
from prk import abi, scenes  # noqa: E402


def time_scene(name, s, semantics, phong, steps=60, warmup=10, tile=None):
    r = prk.Renderer(0)
    try:
        r.target_alloc(s.width, s.height)
        if tile:
            r.set_tile(*tile)
        r.set_camera(s.prk_transform(), s.prk_lights())
        g = r.geometry(s.vertices, s.colors, s.normals, s.uvs)
        draws = s.draws if s.draws is not None else [(0, s.tri_count, s.texture)]
        texs = {}
        for _, _, t in draws:
            if t is not None and id(t) not in texs:
                texs[id(t)] = r.texture(t)

        def frame():
            r.clear_on_flush()
            for first, count, t in draws:
                tex = texs.get(id(t)) if t is not None else None
                if semantics == abi.PRK_SEM_AVX:
                    r.draw_model_optimized(g, count, first_tri=first, P=s.P, bitmap=tex, phong=phong)
                else:
                    r.draw_model(g, count, first_tri=first, P=s.P, bitmap=tex, phong=phong)
            r.complete_all_work()

        for _ in range(warmup):
            frame()
        r.synchronize()
        r.timing_reset()
        t0 = time.perf_counter()
        for _ in range(steps):
            frame()
        r.synchronize()
        ms = (time.perf_counter() - t0) * 1e3 / steps
        st = r.stats()
        n = max(1, st["frames_timed"])
        out = dict(config=name, tile="%dx%d" % tuple(tile) if tile else "default", width=s.width, height=s.height,
                   triangles=s.tri_count,
                   semantics="avx" if semantics == abi.PRK_SEM_AVX else "scalar", phong=bool(phong),
                   ms_per_frame=ms, mpixels_s=s.width * s.height / (ms * 1e-3) / 1e6,
                   mtri_s=s.tri_count / (ms * 1e-3) / 1e6, ms_bin=st["sum_ms_bin"] / n,
                   ms_raster=st["sum_ms_raster"] / n, ms_vis=st["sum_ms_vis"] / n,
                   bin_entries=int(st["bin_entries"]), anomalies=int(st["anomalies"]))
        print(json.dumps(out), flush=True)
        return out
    finally:
        r.close()


def main():
    if len(sys.argv) > 1 and sys.argv[1] == "--small-tiles":  # tile sweep of the small configs
        for tile in (None, (128, 8), (64, 8), (32, 8), (16, 8), (32, 4), (16, 16)):
            time_scene("C1", scenes.single_triangle(), abi.PRK_SEM_SCALAR, False, tile=tile, steps=30)
            time_scene("C2", scenes.displaced_sphere(70000, 1920, 1080, seed=3), abi.PRK_SEM_SCALAR, True, tile=tile)
        return
    if len(sys.argv) > 1 and sys.argv[1] == "--big-tiles":  # tile sweep of the large configs
        for tile in (None, (128, 8), (64, 8), (32, 8)):
            time_scene("C3a", scenes.random_soup(1_000_000, 4096, 4096, radius=16, seed=2025, textured=False),
                       abi.PRK_SEM_SCALAR, False, tile=tile)
            time_scene("C4-nearest", scenes.sponza_like(3840, 2160, seed=1, filt=abi.PRK_FILTER_NEAREST),
                       abi.PRK_SEM_AVX, True, tile=tile)
            time_scene("C3b", scenes.random_soup(1_000_000, 4096, 4096, radius=16, seed=2024), abi.PRK_SEM_AVX, True,
                       tile=tile)
        return
    if len(sys.argv) > 1 and sys.argv[1] == "--wide-tiles":  # 256x8 against 512x8 on the large configs
        for tile in (None, (512, 8)):
            time_scene("C3a", scenes.random_soup(1_000_000, 4096, 4096, radius=16, seed=2025, textured=False),
                       abi.PRK_SEM_SCALAR, False, tile=tile)
            time_scene("C3b", scenes.random_soup(1_000_000, 4096, 4096, radius=16, seed=2024), abi.PRK_SEM_AVX, True,
                       tile=tile)
            for filt, tag in ((abi.PRK_FILTER_NEAREST, "nearest"), (abi.PRK_FILTER_BILINEAR, "bilinear")):
                time_scene("C4-" + tag, scenes.sponza_like(3840, 2160, seed=1, filt=filt), abi.PRK_SEM_AVX, True,
                           tile=tile)
            time_scene("C5-1gpu", scenes.random_soup(1_000_000, 8192, 8192, radius=32, seed=5), abi.PRK_SEM_AVX, True,
                       tile=tile)
        return
    out_path = sys.argv[1] if len(sys.argv) > 1 else None
    res = []
    res.append(time_scene("C1", scenes.single_triangle(), abi.PRK_SEM_SCALAR, False))
    res.append(time_scene("C2", scenes.displaced_sphere(70000, 1920, 1080, seed=3), abi.PRK_SEM_SCALAR, True))
    res.append(time_scene("C3a", scenes.random_soup(1_000_000, 4096, 4096, radius=16, seed=2025, textured=False),
                          abi.PRK_SEM_SCALAR, False))
    res.append(time_scene("C3b", scenes.random_soup(1_000_000, 4096, 4096, radius=16, seed=2024),
                          abi.PRK_SEM_AVX, True))
    for filt, tag in ((abi.PRK_FILTER_NEAREST, "nearest"), (abi.PRK_FILTER_BILINEAR, "bilinear")):
        res.append(time_scene("C4-" + tag, scenes.sponza_like(3840, 2160, seed=1, filt=filt), abi.PRK_SEM_AVX, True))
    res.append(time_scene("C5-1gpu", scenes.random_soup(1_000_000, 8192, 8192, radius=32, seed=5),
                          abi.PRK_SEM_AVX, True))
    if out_path:
        with open(out_path, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
