"""Generate tests/golden/*.npz — regression fixtures of the CPU restatement.

The reference ships no tests or golden images and cannot be built here
(DESIGN.md §3), so these fixtures are produced by oracle/prk_oracle.c and
cross-checked by tests/pyref.py (an independent restatement) at generation
time.  They pin the restatement against regressions and give the GPU tests a
committed expected image; they do NOT pin parity with the reference itself.

Each fixture holds the inputs (geometry, texture, camera, lights, semantics)
and the expected colour, z and winning-triangle maps.

c3b_one_object.json: the headline C3b scene (4096^2, 1M triangles, Phong +
texture) drawn as ONE object (one active edge table): the oracle needs
minutes for it (its insertion scans the ~15k-entry list per edge, as the
reference's does), so only per-band SHA-256 digests of its colour, z and
winner maps are committed, with a digest of the generated inputs.
usage: python tools/make_golden.py [c3b_one_object]
"""
import hashlib
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cpu-renderer_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

from prk import abi, scenes  # noqa: E402
import oracle as O  # noqa: E402
import pyref  # noqa: E402

OUT = os.path.join(ROOT, "tests", "golden")


def sphere_scene(W, H, textured):
    import prk
    V, C, N, UV = prk.construct_sphere()
    base = scenes.random_soup(1, W, H, seed=0, tex_size=64)
    return scenes.Scene(W, H, V, C, N, UV, base.transform, scenes.LIGHTS_ONE, scenes.AMBIENT_ONE,
                        base.texture if textured else None, P=(0.0, 0.0, 2.0), name="sphere")


def cases():
    yield "c1_triangle_gouraud", scenes.single_triangle(), abi.PRK_SEM_SCALAR, False
    yield "c1_triangle_avx", scenes.single_triangle(textured=True, gouraud_only=False), abi.PRK_SEM_AVX, True
    yield "sphere_avx_128", sphere_scene(128, 128, True), abi.PRK_SEM_AVX, True
    yield "sphere_gouraud_128", sphere_scene(128, 128, False), abi.PRK_SEM_SCALAR, False
    yield ("soup_avx_128x96", scenes.random_soup(300, 128, 96, radius=12, seed=42, tex_size=32,
                                                 lights=scenes.LIGHTS_TWO, ambient=scenes.AMBIENT_TWO),
           abi.PRK_SEM_AVX, True)
    yield ("soup_avx_clip_96x64", scenes.random_soup(60, 96, 64, radius=50, seed=43, tex_size=32,
                                                     centroid_margin=40), abi.PRK_SEM_AVX, True)
    yield ("soup_gouraud_128x96", scenes.random_soup(300, 128, 96, radius=12, seed=44, textured=False,
                                                     lights=scenes.LIGHTS_TWO, ambient=scenes.AMBIENT_TWO),
           abi.PRK_SEM_SCALAR, False)
    yield ("soup_phongtex_128x96", scenes.random_soup(200, 128, 96, radius=12, seed=45, tex_size=32),
           abi.PRK_SEM_SCALAR, True)


def save(name, s, sem, phong):
    col, z, win, st = O.render(s, semantics=sem, phong=phong)
    pc, pz, pw = pyref.render(s, sem, phong)
    assert (pc == col).all() and (pz.view(np.uint32) == z.view(np.uint32)).all() and (pw == win).all(), name
    tex = s.texture
    np.savez_compressed(
        os.path.join(OUT, name + ".npz"),
        width=s.width, height=s.height, vertices=s.vertices, colors=s.colors, normals=s.normals, uvs=s.uvs,
        P=np.array(s.P, np.float32), transform=np.array(s.transform, np.float32),
        light_p=np.array([l[0] for l in s.lights], np.float32).reshape(-1, 3),
        light_i=np.array([l[1] for l in s.lights], np.float32).reshape(-1, 4),
        ambient=np.array(s.ambient, np.float32),
        texels=tex.texels if tex is not None else np.zeros((0, 0), np.uint32),
        tex_wh=np.array([tex.width, tex.height] if tex is not None else [0, 0], np.int32),
        semantics=sem, phong=int(phong), color=col, z=z, winners=win,
        spans=st["spans"], span_pixels=st["span_pixels"])
    print("%-24s %dx%d tris=%d covered=%d spans=%d" % (name, s.width, s.height, s.tri_count,
                                                      int((win >= 0).sum()), st["spans"]))


def load(path):
    d = np.load(path)
    tex = None
    if d["texels"].size:
        tex = scenes.Texture(d["texels"], int(d["tex_wh"][0]), int(d["tex_wh"][1]))
    lights = [(tuple(float(v) for v in p), tuple(float(v) for v in i)) for p, i in zip(d["light_p"], d["light_i"])]
    s = scenes.Scene(int(d["width"]), int(d["height"]), d["vertices"], d["colors"], d["normals"], d["uvs"],
                     tuple(float(v) for v in d["transform"]), lights, tuple(float(v) for v in d["ambient"]),
                     tex, P=tuple(float(v) for v in d["P"]), name=os.path.basename(path))
    return s, int(d["semantics"]), bool(d["phong"]), d


def scene_digest(s):
    h = hashlib.sha256()
    for a in (s.vertices, s.colors, s.normals, s.uvs, s.texture.texels if s.texture is not None else None):
        if a is not None:
            h.update(np.ascontiguousarray(a).tobytes())
    return h.hexdigest()


def band_digests(col, z, win, rows):
    return [[hashlib.sha256(np.ascontiguousarray(a[b * rows:(b + 1) * rows]).tobytes()).hexdigest()
             for a in (col, z, win)] for b in range(col.shape[0] // rows)]


def c3b_one_object(T=1_000_000, W=4096, H=4096, R=16.0, seed=2024, rows=64):
    import time
    s = scenes.random_soup(T, W, H, radius=R, seed=seed)
    t = time.time()
    col, z, win, st = O.render(s, tris_per_object=s.tri_count)
    out = dict(tris=T, width=W, height=H, radius=R, seed=seed, band_rows=rows, inputs=scene_digest(s),
               spans=int(st["spans"]), span_pixels=int(st["span_pixels"]), covered=int((win >= 0).sum()),
               bands=band_digests(col, z, win, rows))
    with open(os.path.join(OUT, "c3b_one_object.json"), "w") as f:
        json.dump(out, f, indent=0)
    print("c3b_one_object: %.0f s, spans=%d covered=%d" % (time.time() - t, st["spans"], out["covered"]))


if __name__ == "__main__":
    os.makedirs(OUT, exist_ok=True)
    if sys.argv[1:] == ["c3b_one_object"]:
        c3b_one_object()
    else:
        for name, s, sem, phong in cases():
            save(name, s, sem, phong)
