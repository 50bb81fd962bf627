"""Time the whole-object (span) path: scenes drawn as objects of several
triangles (one active edge table per object, projekt.cpp:3615-3871 /
162-601), the configuration a reference caller gets when one
render_entry_3d_object holds a model.

usage: python tools/time_objects.py [--frames N] [--json OUT]
Per case: host wall time per frame with a device sync after every frame
(the span path reads two counts back per pass), in ms, and Mpixels/s of the
target."""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cpu-renderer_amd"))
import numpy as np  # noqa: E402
import prk  # noqa: E402
from prk import abi, scenes  # noqa: E402


def sphere_scene(W, H):
    V, Cc, N, UV = prk.construct_sphere()
    base = scenes.random_soup(1, W, H, seed=0)
    return scenes.Scene(W, H, V, Cc, N, UV, base.transform, scenes.LIGHTS_ONE, scenes.AMBIENT_ONE,
                        base.texture, P=(0.0, 0.0, 2.0), name="sphere")


def spheres64_scene(W, H):
    """64 ConstructSphere instances (r = 0.175 m) on an 8 x 8 grid, one
    object each (their offsets baked into the vertices, P = (0, 0, 2))."""
    V, Cc, N, UV = prk.construct_sphere()
    base = scenes.random_soup(1, W, H, seed=0)
    vs = []
    for i in range(8):
        for j in range(8):
            vs.append(V * 0.35 + np.array([(i - 3.5) * 0.5, (j - 3.5) * 0.5, 0.0], np.float32))
    k = 64
    return scenes.Scene(W, H, np.concatenate(vs).astype(np.float32), np.tile(Cc, (k, 1)), np.tile(N, (k, 1)),
                        np.tile(UV, (k, 1)), base.transform, scenes.LIGHTS_ONE, scenes.AMBIENT_ONE, base.texture,
                        P=(0.0, 0.0, 2.0), name="spheres64")


def cases():
    sph = sphere_scene(1024, 1024)
    sph64 = spheres64_scene(2048, 2048)
    c2 = scenes.displaced_sphere(70000, 1920, 1080, seed=3)
    c2t = c2.subset(0, c2.tri_count)
    c2t.texture = sph.texture  # FillLineOptimized needs a Bitmap (projekt.cpp:1506)
    soup = scenes.random_soup(1_000_000, 4096, 4096, radius=16, seed=2024)
    return [
        ("sphere_1obj_avx", sph, abi.PRK_SEM_AVX, True, sph.tri_count),
        ("sphere_1obj_scalar_gouraud", sph, abi.PRK_SEM_SCALAR, False, sph.tri_count),
        ("sphere_1obj_scalar_phong", sph, abi.PRK_SEM_SCALAR, True, sph.tri_count),
        ("c2_1obj_scalar_phong", c2, abi.PRK_SEM_SCALAR, True, c2.tri_count),
        ("c2_1obj_avx", c2t, abi.PRK_SEM_AVX, True, c2.tri_count),
        ("spheres64_64obj_avx", sph64, abi.PRK_SEM_AVX, True, sph.tri_count),
        ("c3b_obj16_avx", soup, abi.PRK_SEM_AVX, True, 16),
        ("c3b_1obj_avx", soup, abi.PRK_SEM_AVX, True, soup.tri_count),
        ("c3b_obj1_avx", soup, abi.PRK_SEM_AVX, True, 1),
    ]


def time_case(s, sem, phong, tpo, frames):
    r = prk.Renderer(0)
    try:
        r.target_alloc(s.width, s.height)
        r.set_camera(s.prk_transform(), s.prk_lights())
        untex = sem == abi.PRK_SEM_SCALAR
        g = r.geometry(s.vertices, s.colors, s.normals, s.uvs)
        tex = None if untex else r.texture(s.texture)
        dts = []
        for i in range(frames + 2):
            r.synchronize()
            t0 = time.perf_counter()
            r.clear_on_flush()
            r.draw(sem, g, s.tri_count, P=s.P, bitmap=tex, phong=phong, tris_per_object=tpo)
            r.complete_all_work()
            r.synchronize()
            if i >= 2:
                dts.append(time.perf_counter() - t0)
        st = r.stats()  # (cumulative over the frames + 2 warm-ups)
        return float(np.median(dts)) * 1e3, st["objects_chunked"] // (frames + 2), st["objects_walked"] // (frames + 2)
    finally:
        r.close()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=10)
    ap.add_argument("--json")
    ap.add_argument("--only", default="", help="comma-separated case names")
    a = ap.parse_args()
    only = set(x for x in a.only.split(",") if x)
    out = {}
    for name, s, sem, phong, tpo in cases():
        if only and name not in only:
            continue
        # (one object of the whole C3b soup: its walk takes long, fewer frames)
        ms, by_rows, walked = time_case(s, sem, phong, tpo, min(a.frames, 2) if name == "c3b_1obj_avx" else a.frames)
        out[name] = {"tris": s.tri_count, "tris_per_object": tpo, "target": "%dx%d" % (s.width, s.height),
                     "ms_per_frame": round(ms, 3), "mpixels_s": round(s.width * s.height / ms / 1e3, 1),
                     "large_objects_chunked": by_rows, "large_objects_walked": walked}
        print(json.dumps({name: out[name]}), flush=True)
    if a.json:
        with open(a.json, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
