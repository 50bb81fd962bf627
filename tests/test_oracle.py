"""CPU tests of the oracle (the checker) — no GPU.

* Two independently written restatements (oracle/prk_oracle.c and
  tests/pyref.py) must agree bit for bit.
* Known answers derived by hand from projekt.cpp for the rules that shape
  coverage: half-open AVX spans, right-column clip, DrawModel's inclusive
  spans and its one-past-the-row store, strict z-test in submission order,
  back-face cull, near-plane collapse, FillEdgeTable fields.
* Committed golden fixtures (tests/golden, regression only: parity with the
  reference itself is unpinned).
"""
import glob
import os

import numpy as np
import pytest

import oracle as O
import pyref
from prk import abi, scenes

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
MODES = [(abi.PRK_SEM_AVX, True, True), (abi.PRK_SEM_SCALAR, False, False), (abi.PRK_SEM_SCALAR, True, False),
         (abi.PRK_SEM_SCALAR, False, True), (abi.PRK_SEM_SCALAR, True, True), (abi.PRK_SEM_AVX_ST, True, True)]


def same(a, b):
    return ((a[0] == b[0]).all() and (a[1].view(np.uint32) == b[1].view(np.uint32)).all()
            and (a[2] == b[2]).all())


@pytest.mark.parametrize("sem,phong,tex", MODES)
@pytest.mark.parametrize("seed", [1, 2])
def test_two_restatements_agree(sem, phong, tex, seed):
    s = scenes.random_soup(50, 96, 64, radius=14, seed=seed, textured=tex, lights=scenes.LIGHTS_TWO,
                           ambient=scenes.AMBIENT_TWO)
    o = O.render(s, semantics=sem, phong=phong)
    p = pyref.render(s, sem, phong)
    assert same(o, p)


@pytest.mark.parametrize("setup", [abi.PRK_SETUP_PHONG, abi.PRK_SETUP_BITMAP, abi.PRK_SETUP_PHONG | abi.PRK_SETUP_BITMAP])
def test_two_restatements_agree_fill_edge_table_inputs(setup):
    """FillEdgeTable's own PhongShading / Object->Bitmap (projekt.cpp:
    4012-4089) under an untextured non-Phong DrawModel: raw colours unlit
    (Phong setup), white-based lighting (Bitmap, no Phong)."""
    s = scenes.random_soup(60, 96, 64, radius=14, seed=60 + setup, textured=False, lights=scenes.LIGHTS_TWO,
                           ambient=scenes.AMBIENT_TWO)
    o = O.render(s, semantics=abi.PRK_SEM_SCALAR, phong=False, setup=setup)
    assert same(o, pyref.render(s, abi.PRK_SEM_SCALAR, False, setup=setup))
    # the three setups really differ from the draw-derived (vertex-lit) one
    d = O.render(s, semantics=abi.PRK_SEM_SCALAR, phong=False)
    assert (o[0] != d[0]).any()


def split_camera_scenes(s):
    """(setup scene, draw scene): the caller moved the camera and changed the
    lights between FillEdgeTable and DrawModel* (projekt.cpp:3885-3910 vs
    452-458 / 2042-2046)."""
    import copy
    a = copy.copy(s)
    b = copy.copy(s)
    D, F, M2P, cx, cy = s.transform
    b.transform = (D * 1.25, F, M2P, cx + 9.0, cy - 5.0)
    b.lights = [((-1.0, 2.0, 2.5), (0.3, 0.9, 0.5, 1.0))]
    b.ambient = (0.1, 0.15, 0.3, 1.0)
    return a, b


@pytest.mark.parametrize("sem,phong,tex", [MODES[0], MODES[1], MODES[2], MODES[4], MODES[5]])
def test_two_restatements_agree_split_camera(sem, phong, tex):
    """Setup with FillEdgeTable's camera and lights, span shading with the
    ones DrawModel* reads: both restatements agree, and the frame differs from
    either camera alone where the path reads it (Phong shading reads the
    draw's, Gouraud setup lighting and the projection FillEdgeTable's)."""
    s = scenes.random_soup(50, 96, 64, radius=14, seed=31, textured=tex, lights=scenes.LIGHTS_TWO,
                           ambient=scenes.AMBIENT_TWO)
    su, dr = split_camera_scenes(s)
    o = O.render(dr, semantics=sem, phong=phong, setup_camera=su)
    assert same(o, pyref.render(dr, sem, phong, setup_camera=su))
    # geometry (z, coverage) is FillEdgeTable's camera's
    g = O.render(su, semantics=sem, phong=phong)
    assert (o[1].view(np.uint32) == g[1].view(np.uint32)).all() and (o[2] == g[2]).all()
    if phong:  # the shading is the draw's camera's
        assert (o[0] != g[0]).any()
    else:  # Gouraud: every colour comes from the setup
        assert (o[0] == g[0]).all()


def test_oracle_rejects_undefined_setups():
    """A draw reading edge fields its FillEdgeTable never wrote is undefined
    (MinNormal without PhongShading, UV gradients without a Bitmap)."""
    s = scenes.random_soup(10, 64, 64, seed=1)
    for sem, phong, setup in [(abi.PRK_SEM_AVX, True, abi.PRK_SETUP_BITMAP),
                              (abi.PRK_SEM_SCALAR, False, abi.PRK_SETUP_PHONG)]:
        with pytest.raises(RuntimeError):
            O.render(s, semantics=sem, phong=phong, setup=setup)


@pytest.mark.parametrize("sem,phong,tex", [MODES[0], MODES[1], MODES[4], MODES[5]])
def test_two_restatements_agree_clipping(sem, phong, tex):
    """Big triangles hanging over every screen edge (top clip, left XOffset,
    right clamp, offscreen triangles, row-overflow store)."""
    s = scenes.random_soup(30, 64, 48, radius=60, seed=77, textured=tex, centroid_margin=50,
                           z_range=(-3.5, 3.0))
    assert same(O.render(s, semantics=sem, phong=phong), pyref.render(s, sem, phong))


def test_near_plane_collapse():
    """Vertices with D - z <= 0.2 project to (0,0,0) (projekt.cpp:86-90)."""
    s = scenes.random_soup(40, 64, 64, radius=20, seed=5, z_range=(3.7, 3.9), jitter=0.1)
    for sem, phong, _ in (MODES[0], MODES[1]):
        assert same(O.render(s, semantics=sem, phong=phong), pyref.render(s, sem, phong))


def test_threaded_and_banded_match_single():
    s = scenes.random_soup(3000, 256, 192, radius=20, seed=3)
    a = O.render(s)
    assert same(a, O.render(s, threads=5))
    for sem, phong, _ in (MODES[1], MODES[4]):
        s2 = scenes.random_soup(3000, 256, 192, radius=20, seed=4)
        b = O.render(s2, semantics=sem, phong=phong)
        assert same(b, O.render(s2, semantics=sem, phong=phong, threads=7))
        c = O.render(s2, semantics=sem, phong=phong, rows=(40, 131))
        assert (c[1][40:131].view(np.uint32) == b[1][40:131].view(np.uint32)).all()
        assert (c[2][40:131] == b[2][40:131]).all()


def _tri(screen, z=(0.0, 0.0, 0.0), W=64, H=32, textured=True):
    """One triangle given in screen space (unprojected through the default
    camera); the winding is left as given."""
    cam = scenes.default_camera(W, H)
    s = np.array(screen, np.float64)
    z = np.array(z, np.float64)
    D, F, M2P, cx, cy = cam
    x = (s[:, 0] - cx) * (D - z) / M2P / F
    y = (s[:, 1] - cy) * (D - z) / M2P / F
    V = np.stack([x, y, z], -1).astype(np.float32)
    tex = scenes.Texture(np.full((9, 8), 0xFF808080, np.uint32), 8, 8) if textured else None
    if tex is not None:
        tex.texels[8] = 0
    return scenes.Scene(W, H, V, np.ones((3, 4), np.float32), np.tile([[0, 0, 1]], (3, 1)).astype(np.float32),
                        np.array([[0.1, 0.1], [0.9, 0.1], [0.5, 0.9]], np.float32), cam,
                        [((0.0, 0.0, 3.0), (0.5, 0.5, 0.5, 0.5))], (0.5, 0.5, 0.5, 0.5), tex)


def front(pts):
    (x0, y0), (x1, y1), (x2, y2) = pts
    return pts if (x1 - x0) * (y2 - y0) - (y1 - y0) * (x2 - x0) < 0 else [pts[0], pts[2], pts[1]]


def test_backface_culled():
    pts = front([(10.2, 3.3), (50.7, 8.1), (20.4, 28.6)])
    assert (O.render(_tri(pts))[2] >= 0).sum() > 0
    assert (O.render(_tri([pts[0], pts[2], pts[1]]))[2] >= 0).sum() == 0  # 3926-3943


def test_avx_half_open_and_right_clip():
    """FillLineOptimized covers [round(L.X), round(R.X)) per row; a span
    overhanging the right edge is clamped to W-1 first, so column W-1 stays
    empty."""
    pts = front([(20.3, 2.2), (80.0, 2.6), (80.0, 29.4)])
    s = _tri(pts, W=64, H=32)
    _, _, w, _ = O.render(s)
    cov = w >= 0
    assert cov.sum() > 0
    assert not cov[:, 63].any()
    edges = O.fill_edge_table(s, 0, 1)
    assert len(edges) == 3


def test_scalar_inclusive_and_row_overflow():
    """DrawModel covers [round(L.X), round(R.X)] inclusive; with R.X in
    [W-0.5, W) MaxX == W and the store lands on (row+1, 0) (projekt.cpp:389-425)."""
    W, H = 64, 32
    pts = front([(40.2, 4.3), (63.7, 4.6), (63.7, 20.4)])  # right edge at x = 63.7 -> round = 64 = W
    s = _tri(pts, W=W, H=H, textured=False)
    _, _, w, _ = O.render(s, semantics=abi.PRK_SEM_SCALAR, phong=False)
    assert (w[:, 63] >= 0).sum() > 0            # inclusive end reaches the last column
    ovf = np.nonzero(w[:, 0] >= 0)[0]
    assert len(ovf) > 5                          # ... and one past it: (row+1, 0)
    assert (w[ovf - 1, 63] >= 0).all()           # each such store comes from a full row above
    assert (w[:, 1:10] < 0).all()                # nothing else on the left


def test_strict_z_first_triangle_wins():
    pts = front([(10.2, 3.3), (50.7, 8.1), (20.4, 28.6)])
    a = _tri(pts)
    two = scenes.Scene(a.width, a.height, np.concatenate([a.vertices, a.vertices]),
                       np.concatenate([a.colors, a.colors]), np.concatenate([a.normals, a.normals]),
                       np.concatenate([a.uvs, a.uvs]), a.transform, a.lights, a.ambient, a.texture)
    for sem, phong in ((abi.PRK_SEM_AVX, True), (abi.PRK_SEM_SCALAR, False)):
        _, _, w, st = O.render(two, semantics=sem, phong=phong)
        assert (w == 0).sum() > 0 and (w == 1).sum() == 0  # equal z never beats '>' (2219, 495)


def test_edge_table_known_answers():
    """FillEdgeTable on the C1 triangle, field by field from projekt.cpp:3882-4121."""
    s = scenes.single_triangle(textured=True)
    V = s.vertices.astype(np.float32)
    D, F, M2P, cx, cy = [np.float32(v) for v in s.transform]
    d = D - V[:, 2]
    k = (np.float32(1) / d) * F
    px = cx + M2P * (k * V[:, 0])
    py = cy + M2P * (k * V[:, 1])
    e = O.fill_edge_table(s, 0, 1, phong=True)
    assert len(e) == 3
    assert [x["YMin"] for x in e] == sorted(x["YMin"] for x in e)  # MergeSort on YMin
    for x in e:
        # Each edge starts at its upper vertex (no clipping here) ...
        i = int(np.argmin(np.abs(px - x["XMin"]) + np.abs(np.round(py) - x["YMin"])))
        assert x["XMin"] == px[i]
        assert x["YMin"] == int(np.floor(abs(py[i]) + 0.5))
        # ... 1/z' and u/z' at that vertex (4002-4008)
        assert x["OneOverZMin"] == np.float32(1) / d[i]
        assert x["UMin"] == s.uvs[i, 0] / d[i]
    # Gradient uses the float dy, ZGradient the integer row count (4070-4074).
    for x in e:
        assert np.isfinite(x["Gradient"])


def test_edge_table_top_clip():
    """A vertex above the screen: YMin = 0 and X/Z/U/V/(1/z) advance by
    ClippedY * gradient (projekt.cpp:3993-3997, 4075-4091)."""
    pts = front([(10.0, -7.4), (50.0, 20.2), (15.0, 28.9)])
    s = _tri(pts, W=64, H=32)
    e = O.fill_edge_table(s, 0, 1)
    assert e[0]["YMin"] == 0 and e[1]["YMin"] == 0
    tops = [x for x in e if x["YMin"] == 0]
    for x in tops:
        assert x["XMin"] != np.float32(10.0)  # advanced by ClippedY * Gradient


def test_avx_needs_texture_and_phong():
    s = scenes.random_soup(10, 64, 64, seed=0, textured=False)
    with pytest.raises(RuntimeError):
        O.render(s, semantics=abi.PRK_SEM_AVX, phong=True)
    s = scenes.random_soup(10, 64, 64, seed=0)
    with pytest.raises(RuntimeError):
        O.render(s, semantics=abi.PRK_SEM_AVX, phong=False)


GOLDEN = sorted(glob.glob(os.path.join(ROOT, "tests", "golden", "*.npz")))


@pytest.mark.parametrize("path", GOLDEN, ids=[os.path.basename(p) for p in GOLDEN])
def test_golden_fixtures(path):
    import sys
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    from make_golden import load
    s, sem, phong, d = load(path)
    col, z, win, st = O.render(s, semantics=sem, phong=phong)
    assert (col == d["color"]).all()
    assert (z.view(np.uint32) == d["z"].view(np.uint32)).all()
    assert (win == d["winners"]).all()
    assert st["spans"] == int(d["spans"]) and st["span_pixels"] == int(d["span_pixels"])


def test_golden_fixtures_present():
    assert len(GOLDEN) >= 8


@pytest.mark.parametrize("seed", [3, 4])
def test_two_restatements_agree_bilinear(seed):
    """The bilinear extension (no reference: BASELINE config 4) is defined by
    oracle/prk_oracle.c:or_bilinear; tests/pyref.py restates it separately."""
    s = scenes.random_soup(40, 96, 64, radius=14, seed=seed, tex_size=16)
    s.texture.filter = abi.PRK_FILTER_BILINEAR
    o = O.render(s)
    p = pyref.render(s, abi.PRK_SEM_AVX, True)
    assert same(o, p)
    s.texture.filter = abi.PRK_FILTER_NEAREST
    n = O.render(s)
    assert (n[2] == o[2]).all() and (n[1].view(np.uint32) == o[1].view(np.uint32)).all()  # same coverage / z
    assert (n[0] != o[0]).any()  # but a filtered colour


def test_bilinear_known_answer():
    """A 2x2 texture sampled at its centre is the mean of the four texels;
    at a texel centre it is that texel (weights exactly 0/1)."""
    tex = np.zeros((3, 2), np.uint32)
    tex[0] = [0xFF000000, 0xFFFF0000]
    tex[1] = [0xFF00FF00, 0xFF0000FF]
    t = scenes.Texture(tex, 2, 2, abi.PRK_FILTER_BILINEAR)
    c = pyref.bilinear(t, np.float32(0.5), np.float32(0.5))
    assert [float(v) for v in c] == [0.25, 0.25, 0.25, 1.0]  # R, G, B, A
    c = pyref.bilinear(t, np.float32(0.25), np.float32(0.25))
    assert [float(v) for v in c] == [0.0, 0.0, 0.0, 1.0]


def test_sponza_like_multi_draw_oracle():
    """C4 stand-in: 8 material draws into one frame; the chained oracle draws
    equal one oracle call per draw on the running target."""
    s = scenes.sponza_like(320, 192, tex_size=64, detail=0.4)
    assert len(s.draws) == 8 and s.tri_count > 10000
    c, z, w, _ = O.render(s, threads=4)
    assert (w >= 0).mean() > 0.9
    assert len(np.unique(w[w >= 0])) > 1000


def test_single_thread_overload_ties_and_left_clip():
    """DrawModelOptimized(Buffer,...) (projekt.cpp:2350-3358) against
    FillLineOptimized: equal z goes to the LATER fragment (GE_OQ, 3205 vs
    GT_OQ, 2219), and a left-clipped span starts its lane interpolation at
    the left edge's values (XOffset = -XOffset = -0.0f, 2508, instead of
    -L.X).  Everywhere else the two agree bit for bit; both restatements
    agree on both."""
    s = scenes.with_ties(scenes.random_soup(300, 128, 96, radius=24, seed=31, textured=True,
                                            centroid_margin=-26), seed=3)  # no clipped span
    a = O.render(s, semantics=abi.PRK_SEM_AVX)
    st = O.render(s, semantics=abi.PRK_SEM_AVX_ST)
    assert same(st, pyref.render(s, abi.PRK_SEM_AVX_ST, True))
    # ties: some pixel's winner flips from a triangle to its later duplicate
    diff = a[2] != st[2]
    assert diff.any()
    assert (a[1].view(np.uint32)[diff] == st[1].view(np.uint32)[diff]).all()  # same z, other winner
    # left clip: XOffset differs only for spans whose left edge is at x < 0
    c = scenes.random_soup(40, 64, 48, radius=40, seed=8, textured=True, centroid_margin=10)
    c.vertices[:, 0] -= np.float32(0.35)  # push everything over the left border
    ca = O.render(c, semantics=abi.PRK_SEM_AVX)
    cs = O.render(c, semantics=abi.PRK_SEM_AVX_ST)
    assert same(cs, pyref.render(c, abi.PRK_SEM_AVX_ST, True))
    zd = ca[1].view(np.uint32) != cs[1].view(np.uint32)
    assert zd.any() and zd[:, 0].any()  # the clipped column differs


def test_edge_list_draw_equals_object_draw():
    """FillEdgeTable + DrawModelOptimized composed: drawing an object's
    exported edge list (oracle_draw_edges, the prk_draw_edges checker) gives
    the object draw's frame exactly (whole-object AET)."""
    s = scenes.random_soup(24, 96, 64, radius=30, seed=41, textured=True)
    for sem in (abi.PRK_SEM_AVX, abi.PRK_SEM_AVX_ST):
        ref = O.render(s, semantics=sem, tris_per_object=24)
        words = O.fill_edge_table_words(s, 0, 24)
        assert words.shape[0] > 30
        got = O.render_edges(s, words, semantics=sem)
        assert same(ref, got)


def test_span_list_draw_equals_per_triangle_spans():
    """A one-triangle draw is the spans its AET emits: the span list from the
    walk (left/right end points per row, thread_edge_info, projekt.h:39-63)
    drawn through oracle_draw_spans gives the same frame."""
    s = scenes.random_soup(1, 64, 48, radius=18, seed=3, textured=True, centroid_margin=-20)
    ref = O.render(s)
    E = [dict(e) for e in O.fill_edge_table(s, 0, 1)]
    spans = []
    row, lst = E[0]["YMin"], []
    def step(e):
        e["XMin"] = np.float32(e["XMin"] + e["Gradient"]); e["ZMin"] = np.float32(e["ZMin"] + e["ZGradient"])
        n = np.array(e["MinNormal"], np.float32) + np.array(e["NormalGradient"], np.float32)
        inv = np.float32(1) / np.sqrt(np.float32((n[0] * n[0] + n[1] * n[1]) + n[2] * n[2]))
        e["MinNormal"] = (inv * n).astype(np.float32)
        e["UMin"] = np.float32(e["UMin"] + e["UGradient"]); e["VMin"] = np.float32(e["VMin"] + e["VGradient"])
        e["OneOverZMin"] = np.float32(e["OneOverZMin"] + e["OneOverZGradient"])
    maxy = min(max(e["YMax"] for e in E), s.height)
    while row < maxy:
        for e in E:
            if e["YMin"] == row:
                pos = len(lst)
                for j, o in enumerate(lst):
                    if (e["XMin"], e["Gradient"], e["Left"]) < (o["XMin"], o["Gradient"], o["Left"]):
                        pos = j
                        break
                lst.insert(pos, e)
        lst = [e for e in lst if not e["YMax"] <= row]
        if len(lst) >= 2:
            L, R = lst[0], lst[1]
            w = np.zeros(25, np.uint32)
            f = w.view(np.float32)
            for k, ee in enumerate((L, R)):
                o = 12 * k
                f[o:o + 5] = [ee["XMin"], ee["ZMin"], ee["OneOverZMin"], ee["UMin"], ee["VMin"]]
                f[o + 5:o + 9] = ee["MinColor"]
                f[o + 9:o + 12] = ee["MinNormal"]
            w[24] = row
            spans.append(w)
            step(L); step(R)
            if L["XMin"] > R["XMin"]:
                lst[0], lst[1] = R, L
        row += 1
    got = O.render_spans(s, np.stack(spans))
    assert (got[1].view(np.uint32) == ref[1].view(np.uint32)).all() and (got[0] == ref[0]).all()
