"""Render N frames of one BASELINE config (for rocprofv3 kernel traces).

usage: python tools/frames.py <C1|C2|C3a|C3b|C4> [frames]
Frames as tools/bench_configs.py draws them; the host waits after each frame,
so kernel durations in a trace are serial (no overlap with other frames)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cpu-renderer_amd"))
import prk  # noqa: E402
from prk import abi, scenes  # noqa: E402

CONFIGS = {
    "C1": (lambda: scenes.single_triangle(), abi.PRK_SEM_SCALAR, False),
    "C2": (lambda: scenes.displaced_sphere(70000, 1920, 1080, seed=3), abi.PRK_SEM_SCALAR, True),
    "C3a": (lambda: scenes.random_soup(1_000_000, 4096, 4096, radius=16, seed=2025, textured=False),
            abi.PRK_SEM_SCALAR, False),
    "C3b": (lambda: scenes.random_soup(1_000_000, 4096, 4096, radius=16, seed=2024), abi.PRK_SEM_AVX, True),
    "C4": (lambda: scenes.sponza_like(3840, 2160, seed=1), abi.PRK_SEM_AVX, True),
}


def main():
    name = sys.argv[1]
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    make, sem, phong = CONFIGS[name]
    s = make()
    r = prk.Renderer(0)
    r.target_alloc(s.width, s.height)
    r.set_camera(s.prk_transform(), s.prk_lights())
    g = r.geometry(s.vertices, s.colors, s.normals, s.uvs)
    draws = s.draws if s.draws is not None else [(0, s.tri_count, s.texture)]
    texs = {id(t): r.texture(t) for _, _, t in draws if t is not None}
    for _ in range(n):
        r.clear_on_flush()
        for first, count, t in draws:
            tex = texs.get(id(t)) if t is not None else None
            if sem == abi.PRK_SEM_AVX:
                r.draw_model_optimized(g, count, first_tri=first, P=s.P, bitmap=tex, phong=phong)
            else:
                r.draw_model(g, count, first_tri=first, P=s.P, bitmap=tex, phong=phong)
        r.complete_all_work()
        r.synchronize()
    print("frames.py: %s x %d done" % (name, n))
    if os.environ.get("PRK_PROF_PRINT"):  # PRK_PROF=1 builds: per-phase s_memtime cycles, per frame
        c = r.debug_counters(16)
        for nm, off in (("vis", 0), ("shade", 4)):
            print("  %-5s cycles/frame: setup %.3g  walk %.3g  scan %.3g  items %.3g" % (
                (nm,) + tuple(c[off + k] / n for k in range(4))))
        e = [x / n for x in c[8:15]]
        print("  vis events/frame: chunks %.0f  row iterations %.0f  windows %.0f  items %.0f  "
              "active lanes/row it %.1f  spans/row it %.1f  items/window %.1f  regular chunks %.0f" % (
                  e[0], e[1], e[2], e[3], e[4] / max(1, e[1]), e[5] / max(1, e[1]), e[3] / max(1, e[2]), e[6]))
    r.close()


if __name__ == "__main__":
    main()
