"""GPU parity: libprk_hip.so on an MI355X vs the CPU restatement (oracle/).

Bar (BASELINE.json north_star): z-buffer bit-exact, winning-triangle map
bit-exact, RGBA within +-1 LSB per channel.  The kernels replay the
reference's float recurrences op for op, so colours are checked exact
everywhere; `COLOR_TOL` is the contract, reported in the message.  The scalar
Phong path's double pow is exact too: test_phong_pow.py shows x^16 never comes
within 8 double ulps of a float rounding boundary for x in [0, 1].

Oracle parity is UNPINNED: the reference cannot be built here.
"""
import ctypes

import numpy as np
import pytest

import oracle as O
import prk
from prk import abi, scenes

pytestmark = pytest.mark.gpu

COLOR_TOL = 1  # LSB per channel (north_star)


def channel_diff(a, b):
    a = a.view(np.uint8).reshape(a.shape + (4,)).astype(np.int16)
    b = b.view(np.uint8).reshape(b.shape + (4,)).astype(np.int16)
    return np.abs(a - b).max(-1)


def compare(g, o, label=""):
    gc, gz, gw, _ = g
    oc, oz, ow, _ = o
    zbad = gz.view(np.uint32) != oz.view(np.uint32)
    wbad = gw != ow
    cd = channel_diff(gc, oc)
    msg = "%s: z mismatches %d, winner mismatches %d, colour >%d LSB %d, colour inexact %d" % (
        label, zbad.sum(), wbad.sum(), COLOR_TOL, (cd > COLOR_TOL).sum(), (cd > 0).sum())
    if zbad.any():
        ys, xs = np.nonzero(zbad)
        msg += "; first z diff at (%d,%d) gpu=%r ora=%r gw=%d ow=%d" % (
            ys[0], xs[0], gz[ys[0], xs[0]], oz[ys[0], xs[0]], gw[ys[0], xs[0]], ow[ys[0], xs[0]])
    assert not zbad.any() and not wbad.any() and not (cd > COLOR_TOL).any(), msg
    assert not (cd > 0).any(), msg  # exact: every colour op replayed, the scalar pow included


def run_both(scene, semantics=abi.PRK_SEM_AVX, phong=True, tile=None, threads=8, label="", tris_per_object=1,
             setup=None):
    o = O.render(scene, semantics=semantics, phong=phong, threads=threads if tris_per_object == 1 else 1,
                 tris_per_object=tris_per_object, setup=setup)
    g = prk.render_scene(scene, semantics=semantics, phong=phong, tile=tile, tris_per_object=tris_per_object,
                         setup=setup)
    compare(g, o, label=label or scene.name)
    return g, o


@pytest.mark.parametrize("semantics,phong,textured,tpo", [
    (abi.PRK_SEM_AVX, True, True, 1), (abi.PRK_SEM_AVX_ST, True, True, 1), (abi.PRK_SEM_SCALAR, True, False, 1),
    (abi.PRK_SEM_SCALAR, False, False, 1), (abi.PRK_SEM_SCALAR, True, True, 1), (abi.PRK_SEM_AVX, True, True, 8),
    (abi.PRK_SEM_SCALAR, True, False, 8), (abi.PRK_SEM_AVX, True, True, 64)])
def test_split_setup_and_shade_camera(gpu, semantics, phong, textured, tpo):
    """prk_set_camera + prk_set_shade_camera: the setup (projection, Gouraud
    lighting) with FillEdgeTable's camera, the span shading (Phong,
    unprojection) with the one DrawModel* reads (projekt.cpp:3885-4063 vs
    452-458, 2042-2046, 3030-3034), per triangle and as whole objects, against
    the oracle's split (or_draw_desc.SetupT / SetupLights)."""
    import copy
    s = scenes.random_soup(6000, 256, 256, radius=16, seed=41, textured=textured, lights=scenes.LIGHTS_TWO,
                           ambient=scenes.AMBIENT_TWO)
    b = copy.copy(s)
    D, F, M2P, cx, cy = s.transform
    b.transform = (D * 1.25, F, M2P, cx + 9.0, cy - 5.0)
    b.lights = [((-1.0, 2.0, 2.5), (0.3, 0.9, 0.5, 1.0))]
    b.ambient = (0.1, 0.15, 0.3, 1.0)
    o = O.render(b, semantics=semantics, phong=phong, tris_per_object=tpo, setup_camera=s)
    g = prk.render_scene(s, semantics=semantics, phong=phong, tris_per_object=tpo, shade_camera=b)
    compare(g, o, label="split camera")
    if phong:  # the shading camera made a difference
        assert (channel_diff(g[0], O.render(s, semantics=semantics, phong=phong, tris_per_object=tpo)[0]) > 1).any()


@pytest.mark.parametrize("n,bits", [(1, 8), (100, 26), (6624, 26), (70000, 30), (262145, 31), (3000000, 36)])
def test_span_path_sort_and_scan(gpu, n, bits):
    """csrc/prk_sort.hip: the span path's radix sort (MergeSort keys,
    projekt.cpp:2-72) is a stable sort and its scan an exclusive prefix sum:
    tools/sort_bench checks both against std::stable_sort / a host sum on
    random keys with ties, short and long tiles, one and many look-back
    tiles."""
    import os
    import subprocess
    exe = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools", "sort_bench")
    assert os.path.exists(exe), "tools/sort_bench not built (__graft_entry__.build())"
    r = subprocess.run([exe, str(n), str(bits), "3"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and "sort mismatches 0, scan mismatches 0" in r.stdout, (r.stdout, r.stderr)


@pytest.mark.parametrize("seed", [1, 2])
def test_shared_divisor_exact(gpu, seed):
    """The kernels' shared-reciprocal quotients (prk_device.h DivBy) equal the
    compiler's IEEE x / d bit for bit: 2^24 hashed draws with exponents on
    both sides of the fast range, signed zeros, and normalisations."""
    nq, nn = prk.selftest_div(n=1 << 24, seed=seed)
    assert (nq, nn) == (0, 0)


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_avx_soup_256(gpu, seed):
    run_both(scenes.random_soup(2000, 256, 256, radius=16, seed=seed))


def test_avx_soup_512_20k(gpu):
    g, o = run_both(scenes.random_soup(20000, 512, 512, radius=16, seed=7))
    assert (g[2] >= 0).sum() > 100000  # the scene actually covers the screen


def test_avx_two_lights_r40(gpu):
    run_both(scenes.random_soup(20000, 512, 512, radius=40, seed=3, lights=scenes.LIGHTS_TWO,
                                ambient=scenes.AMBIENT_TWO))


def test_avx_big_triangles_clipping(gpu):
    # Spans up to ~600 px crossing many tiles, heavy clipping on every side.
    run_both(scenes.random_soup(3000, 1024, 1024, radius=300, seed=5, centroid_margin=200))


def test_avx_zero_lights(gpu):
    run_both(scenes.random_soup(5000, 256, 256, radius=16, seed=11, lights=[]))


def test_avx_1024_100k(gpu):
    run_both(scenes.random_soup(100000, 1024, 1024, radius=64, seed=9))


@pytest.mark.parametrize("phong,textured", [(False, False), (True, False), (False, True), (True, True)])
def test_scalar_modes(gpu, phong, textured):
    s = scenes.random_soup(20000, 512, 512, radius=16, seed=21, textured=textured,
                           lights=scenes.LIGHTS_TWO, ambient=scenes.AMBIENT_TWO)
    run_both(s, semantics=abi.PRK_SEM_SCALAR, phong=phong,
             label="scalar phong=%d tex=%d" % (phong, textured))


def test_scalar_big_triangles(gpu):
    s = scenes.random_soup(1500, 1024, 1024, radius=120, seed=4, textured=False)
    run_both(s, semantics=abi.PRK_SEM_SCALAR, phong=False)


def test_single_triangle_c1(gpu):
    s = scenes.single_triangle()
    g, o = run_both(s, semantics=abi.PRK_SEM_SCALAR, phong=False)
    assert (g[2] == 0).sum() == o[3]["writes"] > 10000
    s2 = scenes.single_triangle(textured=True, gouraud_only=False)
    run_both(s2, semantics=abi.PRK_SEM_AVX, phong=True)


def test_construct_sphere(gpu):
    V, Cc, N, UV = prk.construct_sphere()
    assert V.shape == (6624, 3)
    base = scenes.random_soup(1, 512, 512, seed=0)
    s = scenes.Scene(512, 512, V, Cc, N, UV, base.transform, scenes.LIGHTS_ONE, scenes.AMBIENT_ONE,
                     base.texture, P=(0.0, 0.0, 2.0), name="sphere")
    run_both(s, semantics=abi.PRK_SEM_AVX, phong=True)
    run_both(s, semantics=abi.PRK_SEM_SCALAR, phong=False)


@pytest.mark.parametrize("tile", [(8, 8), (32, 16), (64, 32), (128, 64), (512, 8), (512, 16)])
def test_tile_sizes(gpu, tile):
    run_both(scenes.random_soup(8000, 512, 384, radius=24, seed=13), tile=tile)


def test_prior_contents_two_flushes(gpu):
    """Second frame draws over the first one's colour/z (strict '>' against
    the prior z-buffer, untouched pixels keep their colour)."""
    a = scenes.random_soup(4000, 256, 256, radius=16, seed=1)
    b = scenes.random_soup(4000, 256, 256, radius=16, seed=2)
    oc, oz, _, _ = O.render(a)
    oc2, oz2, ow2, _ = O.render(b, color=oc, z=oz)
    gc, gz, _, _ = prk.render_scene(a)
    gc2, gz2, gw2, st = prk.render_scene(b, color=gc, z=gz)
    assert (gz2.view(np.uint32) == oz2.view(np.uint32)).all()
    assert (gc2 == oc2).all()
    assert (gw2 == ow2).all()


@pytest.mark.parametrize("tile", [None, (128, 64)])
@pytest.mark.parametrize("W,H", [(256, 256), (200, 150)])
def test_fused_clear(gpu, W, H, tile):
    """prk_target_clear_on_flush: the AVX frame's kernels write every pixel of
    the target (edge tiles, tiles no triangle touches) over stale contents."""
    s = scenes.random_soup(3000, W, H, radius=16, seed=41)
    rng = np.random.default_rng(5)
    stale_c = rng.integers(0, 2**32, (H, W), dtype=np.uint32)
    stale_z = np.full((H, W), 1e30, np.float32)  # would block every fragment if kept
    g = prk.render_scene(s, color=stale_c, z=stale_z, fused_clear=True, tile=tile)
    compare(g, O.render(s), label="fused clear %dx%d" % (W, H))


@pytest.mark.parametrize("case", ["clear", "fused", "prior", "band", "st", "negzero", "scalar"])
def test_early_z(gpu, case):
    """prk_set_early_z: span-record frames write z in k_vis (from the winner's
    key, or the fused clear's z) and k_pix only the colour; the download
    takes z from the event after k_vis.  Plain, fused-clear, prior-contents,
    row-band and single-thread frames, a scalar frame (not a span-record
    frame: the plain path), and flat triangles at z = -0.0 (every fragment
    ties at zero; the interpolation yields +0.0 there -- -0.0 + o * +0.0 with
    o >= 0 -- so the key's +0.0 is the z; k_pix's -0.0 fix-up stays a
    guard): the oracle and the default path, bit for bit."""
    s = scenes.random_soup(5000, 256, 192, radius=18, seed=60, centroid_margin=20)
    kw, okw = {}, {}
    sem = abi.PRK_SEM_AVX
    if case == "fused" or case == "prior":
        rng = np.random.default_rng(6)
        c0 = rng.integers(0, 2**32, (192, 256), dtype=np.uint32)
        z0 = rng.uniform(-2.0, 2.0, (192, 256)).astype(np.float32)
        kw = dict(color=c0, z=z0, fused_clear=case == "fused")
        okw = {} if case == "fused" else dict(color=c0, z=z0)
    elif case == "band":
        kw = dict(rows=(40, 131))
    elif case == "st":
        sem = abi.PRK_SEM_AVX_ST
    elif case == "negzero":
        s.vertices[:, 2] = np.float32(-0.0)
    elif case == "scalar":
        sem = abi.PRK_SEM_SCALAR
    o = O.render(s, semantics=sem, **okw)
    e = prk.render_scene(s, semantics=sem, early_z=True, **kw)
    d = prk.render_scene(s, semantics=sem, **kw)
    if case == "band":
        o = tuple(x[40:131] if x is not None and getattr(x, "ndim", 0) == 2 else x for x in o)
    compare(e, o, label="early z " + case)
    for k in range(3):
        assert np.array_equal(e[k].view(np.uint32), d[k].view(np.uint32)), (case, k)
    if case == "negzero":
        assert (o[1] == 0.0).sum() > 1000  # (the fragments did land at zero)


@pytest.mark.parametrize("first", ["scalar", "objects"])
def test_early_z_after_z_writing_frame(gpu, first):
    """Early z with frames queued back to back, no download between them: a
    scalar (k_shade) or whole-object (k_span_shade / k_pix) frame writes z on
    the flush stream, then a fused-clear per-triangle AVX frame writes its z
    in k_vis on the visibility stream.  k_vis must wait for the earlier
    frame's z writers (prk_api.hip, the vis stream's wait on s_mark), or
    their late stores land over the new frame's z.  Debug off (debug frames
    always wait).  z, colour bit for bit against early z off and the oracle."""
    a = scenes.random_soup(60000, 512, 384, radius=40, seed=71, textured=True)
    b = scenes.random_soup(4000, 512, 384, radius=16, seed=72)
    out = {}
    for early in (False, True):
        r = prk.Renderer(0)
        try:
            r.target_alloc(512, 384)
            r.set_debug(False)
            r.set_early_z(early)
            r.set_camera(a.prk_transform(), a.prk_lights())
            ga = r.geometry(a.vertices, a.colors, a.normals, a.uvs)
            gb = r.geometry(b.vertices, b.colors, b.normals, b.uvs)
            ta, tb = r.texture(a.texture), r.texture(b.texture)
            for k in range(3):
                r.clear_on_flush()
                if first == "scalar":
                    r.draw(abi.PRK_SEM_SCALAR, ga, a.tri_count, bitmap=ta, phong=True)
                else:
                    r.draw(abi.PRK_SEM_AVX, ga, a.tri_count, bitmap=ta, phong=True, tris_per_object=8)
                r.complete_all_work()
                r.clear_on_flush()
                r.draw_model_optimized(gb, b.tri_count, bitmap=tb, phong=True)
                r.complete_all_work()
            r.synchronize()
            out[early] = r.download()
        finally:
            r.close()
    oc, oz, _, _ = O.render(b)
    for early in (False, True):
        c, z = out[early]
        assert np.array_equal(z.view(np.uint32), oz.view(np.uint32)), (first, early)
        assert np.array_equal(c, oc), (first, early)


def test_fused_clear_fallbacks(gpu):
    """Scalar frames and empty flushes fill first instead of fusing."""
    s = scenes.random_soup(2000, 256, 192, radius=16, seed=43, textured=False)
    stale_c = np.full((192, 256), 0x12345678, np.uint32)
    stale_z = np.full((192, 256), 1e30, np.float32)
    g = prk.render_scene(s, semantics=abi.PRK_SEM_SCALAR, phong=False, color=stale_c, z=stale_z,
                         fused_clear=True)
    compare(g, O.render(s, semantics=abi.PRK_SEM_SCALAR, phong=False), label="fused clear scalar")
    r = prk.Renderer(0)
    try:
        r.target_alloc(64, 32)
        r.upload(np.full((32, 64), 7, np.uint32), np.full((32, 64), 3.0, np.float32))
        r.set_camera(s.prk_transform(), s.prk_lights())
        r.clear_on_flush(0xFF000000)
        r.complete_all_work()
        r.synchronize()
        c, z = r.download()
        assert (c == 0xFF000000).all() and (z == -np.finfo(np.float32).max).all()
    finally:
        r.close()


def test_pipelined_frames_one_target(gpu):
    """Back-to-back flushes without a host sync (the bench's pattern): frame k
    bins while k-1 rasterises and k's k_vis overlaps k-1's shading, scratch
    sets alternate.  Fused-clear frames must each end as their own frame; a
    frame without a clear must see the previous frame's z and colour."""
    scs = [scenes.random_soup(3000, 256, 192, radius=16, seed=50 + k) for k in range(4)]
    r = prk.Renderer(0)
    try:
        r.target_alloc(256, 192)
        r.set_camera(scs[0].prk_transform(), scs[0].prk_lights())
        geoms = [r.geometry(s.vertices, s.colors, s.normals, s.uvs) for s in scs]
        tex = r.texture(scs[0].texture)
        for k, s in enumerate(scs):  # frames 0..2 fused-clear, frame 3 over frame 2
            if k < 3:
                r.clear_on_flush()
            r.draw_model_optimized(geoms[k], s.tri_count, P=s.P, bitmap=tex, phong=True)
            r.complete_all_work()
        r.synchronize()
        gc, gz = r.download()
    finally:
        r.close()
    for s in scs:
        s.texture = scs[0].texture
    oc, oz, _, _ = O.render(scs[2])
    oc, oz, _, _ = O.render(scs[3], color=oc, z=oz)
    assert (gz.view(np.uint32) == oz.view(np.uint32)).all()
    assert (gc == oc).all()


@pytest.mark.parametrize("sem,phong", [(abi.PRK_SEM_SCALAR, False), (abi.PRK_SEM_AVX, True)])
def test_auto_tile_sparse_then_dense(gpu, sem, phong):
    """The automatic tile: a sparse frame (a few large triangles, under 8 and
    under 64 bin entries per 256x8 tile) switches the context to 64x8 / 32x8
    tiles from its next frame (more bin entries), a frame with many more
    triangles switches back; every frame, before and after each switch,
    equals the oracle's."""
    sparse1 = scenes.single_triangle(512, 512, textured=True, gouraud_only=False)
    sparse2 = scenes.random_soup(40, 512, 512, radius=90, seed=91)
    dense = scenes.random_soup(6000, 512, 512, radius=12, seed=92)
    r = prk.Renderer(0)
    got = []
    try:
        r.target_alloc(512, 512)
        for sc, n in ((sparse1, 3), (sparse2, 3), (dense, 2)):
            r.set_camera(sc.prk_transform(), sc.prk_lights())
            g = r.geometry(sc.vertices, sc.colors, sc.normals, sc.uvs)
            tex = r.texture(sc.texture)
            for _ in range(n):
                r.clear_on_flush()
                if sem == abi.PRK_SEM_AVX:
                    r.draw_model_optimized(g, sc.tri_count, P=sc.P, bitmap=tex, phong=True)
                else:
                    r.draw_model(g, sc.tri_count, P=sc.P, bitmap=tex, phong=False)
                r.complete_all_work()
                r.synchronize()
                got.append((sc, r.stats()["bin_entries"], r.download()))
    finally:
        r.close()
    ent = [e for _, e, _ in got]
    assert ent[1] > ent[0] and ent[4] > ent[3], ent  # narrower tiles from the second frame on
    for sc, _, (gc, gz) in got:
        oc, oz, _, _ = O.render(sc, semantics=sem, phong=phong)
        assert (gz.view(np.uint32) == oz.view(np.uint32)).all()
        assert (gc == oc).all()


@pytest.mark.parametrize("sem,rows", [(abi.PRK_SEM_AVX, None), (abi.PRK_SEM_AVX, (128, 256)),
                                      (abi.PRK_SEM_SCALAR, None)])
def test_auto_tile_wide(gpu, sem, rows):
    """The automatic wide tile: an all-AVX frame of large triangles (>= 4.5
    bin entries a triangle at 256x8; in a row band, per its share of the
    triangles) switches the context to 512x8 from its next frame (fewer
    entries); a scalar frame keeps 256x8.  Every frame equals the oracle's."""
    sc = scenes.random_soup(3000, 1024, 512, radius=48, seed=93)
    r0, r1 = rows if rows else (0, sc.height)
    r = prk.Renderer(0)
    got = []
    try:
        r.target_alloc(sc.width, sc.height, r0, r1)
        r.set_camera(sc.prk_transform(), sc.prk_lights())
        g = r.geometry(sc.vertices, sc.colors, sc.normals, sc.uvs)
        tex = r.texture(sc.texture)
        for _ in range(3):
            r.clear_on_flush()
            if sem == abi.PRK_SEM_AVX:
                r.draw_model_optimized(g, sc.tri_count, P=sc.P, bitmap=tex, phong=True)
            else:
                r.draw_model(g, sc.tri_count, P=sc.P, bitmap=tex, phong=False)
            r.complete_all_work()
            r.synchronize()
            got.append((r.stats()["bin_entries"], r.download()))
    finally:
        r.close()
    ent = [e for e, _ in got]
    if sem == abi.PRK_SEM_AVX:
        assert ent[1] < ent[0] and ent[2] == ent[1], ent  # 512x8 from the second frame on
    else:
        assert ent[0] == ent[1] == ent[2], ent
    oc, oz, _, _ = O.render(sc, semantics=sem, phong=sem == abi.PRK_SEM_AVX)
    for _, (gc, gz) in got:
        assert (gz.view(np.uint32) == oz[r0:r1].view(np.uint32)).all()
        assert (gc == oc[r0:r1]).all()


def test_bin_capacity_rerun(gpu):
    """Counting-sort binning sizes its per-pair arrays from the previous
    frame's entry count; a frame with more entries leaves its bins empty and
    is re-run.  Frames queued without a host sync: a small frame, an
    over-capacity frame drawn over it, an over-capacity frame with a fused
    clear, and a small frame over that."""
    small = scenes.random_soup(3000, 512, 384, radius=16, seed=71)
    big = scenes.random_soup(3000, 512, 384, radius=220, seed=72)
    bigger = scenes.random_soup(6000, 512, 384, radius=300, seed=73)
    small2 = scenes.random_soup(2000, 512, 384, radius=24, seed=74)
    plan = [(small, True), (big, False), (bigger, True), (small2, False)]
    r = prk.Renderer(0)
    entries = []
    try:
        r.target_alloc(512, 384)
        r.set_camera(small.prk_transform(), small.prk_lights())
        tex = r.texture(small.texture)
        geos = [r.geometry(s.vertices, s.colors, s.normals, s.uvs) for s, _ in plan]
        for (s, clear), g in zip(plan, geos):
            if clear:
                r.clear_on_flush()
            r.draw_model_optimized(g, s.tri_count, P=s.P, bitmap=tex, phong=True)
            r.complete_all_work()
            entries.append(r.stats()["bin_entries"])
        r.synchronize()
        gc, gz = r.download()
    finally:
        r.close()
    assert entries[1] > 4 * entries[0] and entries[2] > entries[1], entries
    for s, _ in plan:
        s.texture = small.texture
    oc, oz, _, _ = O.render(bigger)
    oc, oz, _, _ = O.render(small2, color=oc, z=oz)
    assert (gz.view(np.uint32) == oz.view(np.uint32)).all()
    assert (gc == oc).all()


def test_deferred_count_overflow_rerun_across_rebind(gpu):
    """prk_flush returns without reading the frame's bin entry count once a
    previous frame has sized the scratch; the count is read by the next call
    that needs it.  Here an over-capacity frame is drawn into target B, the
    caller re-binds target A and queues another frame over A's contents
    without any sync: the next flush re-runs the overflowed frame into B
    (its own target, camera and clear) before queueing A's frame, and both
    targets end equal to the oracle.  (A and B are device targets owned by
    two other contexts.)"""
    small = scenes.random_soup(3000, 512, 384, radius=16, seed=91)
    big = scenes.random_soup(6000, 512, 384, radius=260, seed=92)
    small2 = scenes.random_soup(2500, 512, 384, radius=20, seed=93)
    for s in (big, small2):
        s.texture = small.texture
    W, H = 512, 384
    ra, rb, r = prk.Renderer(0), prk.Renderer(0), prk.Renderer(0)
    try:
        ra.target_alloc(W, H)
        rb.target_alloc(W, H)
        pa, pb = ra.target(), rb.target()
        r.set_camera(small.prk_transform(), small.prk_lights())
        tex = r.texture(small.texture)
        gs = [r.geometry(s.vertices, s.colors, s.normals, s.uvs) for s in (small, big, small2)]
        r.target_bind(pa[0], pa[1], pa[2], W, H)
        r.clear_on_flush()
        r.draw_model_optimized(gs[0], small.tri_count, P=small.P, bitmap=tex, phong=True)
        r.complete_all_work()  # first frame: counted at once (sizes the scratch)
        r.target_bind(pb[0], pb[1], pb[2], W, H)
        r.clear_on_flush()
        r.draw_model_optimized(gs[1], big.tri_count, P=big.P, bitmap=tex, phong=True)
        r.complete_all_work()  # over capacity: its count is read at the next flush
        r.target_bind(pa[0], pa[1], pa[2], W, H)
        r.draw_model_optimized(gs[2], small2.tri_count, P=small2.P, bitmap=tex, phong=True)
        r.complete_all_work()  # re-runs big into B first, then small2 over A
        r.synchronize()
        entries = r.stats()["bin_entries"]
        ga, gb = ra.download(), rb.download()
    finally:
        r.close()
        ra.close()
        rb.close()
    assert entries > 0
    oc, oz, _, _ = O.render(small)
    oc, oz, _, _ = O.render(small2, color=oc, z=oz)
    bc, bz, _, _ = O.render(big)
    assert (gb[1].view(np.uint32) == bz.view(np.uint32)).all(), "target B z"
    assert (gb[0] == bc).all(), "target B colour"
    assert (ga[1].view(np.uint32) == oz.view(np.uint32)).all(), "target A z"
    assert (ga[0] == oc).all(), "target A colour"


def test_resolve_before_strip_read_on_another_stream(gpu):
    """A caller that reads the target through its own pointers on its own
    stream (bench.py's torch RCCL strip gather) calls Renderer.resolve(stream)
    after the flush: an over-capacity frame is re-run first and the reading
    stream waits for the re-run's end, so the copy it takes is the finished
    frame — with no host sync in between."""
    import torch

    small = scenes.random_soup(3000, 512, 384, radius=16, seed=91)
    big = scenes.random_soup(6000, 512, 384, radius=260, seed=92)
    big.texture = small.texture
    W, H = 512, 384
    dev = torch.device("cuda:0")
    color = torch.empty((H, W), dtype=torch.int32, device=dev)
    zbuf = torch.empty((H, W), dtype=torch.float32, device=dev)
    r = prk.Renderer(0)
    try:
        r.target_bind(color.data_ptr(), W * 4, zbuf.data_ptr(), W, H)
        r.set_camera(small.prk_transform(), small.prk_lights())
        tex = r.texture(small.texture)
        gs = [r.geometry(s.vertices, s.colors, s.normals, s.uvs) for s in (small, big)]
        stream = torch.cuda.current_stream().cuda_stream
        r.clear_on_flush()
        r.draw_model_optimized(gs[0], small.tri_count, P=small.P, bitmap=tex, phong=True)
        r.complete_all_work(stream)  # first frame: counted at once (sizes the scratch)
        r.clear_on_flush()
        r.draw_model_optimized(gs[1], big.tri_count, P=big.P, bitmap=tex, phong=True)
        r.complete_all_work(stream)  # over capacity: re-run when resolved
        side = torch.cuda.Stream(device=dev)
        r.resolve(side.cuda_stream)
        with torch.cuda.stream(side):
            got_c, got_z = color.clone(), zbuf.clone()
        side.synchronize()
        entries = r.stats()["bin_entries"]
    finally:
        r.close()
    bc, bz, _, _ = O.render(big)
    assert entries > 0
    assert (got_z.cpu().numpy().view(np.uint32) == bz.view(np.uint32)).all(), "z"
    assert (got_c.cpu().numpy().view(np.uint32) == bc.view(np.uint32)).all(), "colour"


def test_pipelined_identical_frames_and_band_rebind(gpu):
    """Identical fused-clear frames queued back to back (every scratch set in
    turn) end as the one frame; then the target is re-bound from a full frame
    (two scratch sets) to a band small enough for three and back, frames
    queued across each re-bind."""
    s = scenes.random_soup(16000, 4096, 2048, radius=16, seed=81)
    oc, oz, _, _ = O.render(s)
    r = prk.Renderer(0)
    try:
        r.set_camera(s.prk_transform(), s.prk_lights())
        g = r.geometry(s.vertices, s.colors, s.normals, s.uvs)
        tex = r.texture(s.texture)
        got = []
        for rows in [(0, 2048), (0, 2048), (512, 1024), (0, 2048)]:  # 8 Mpx -> 2 sets, 2 Mpx -> 3 sets
            r.target_alloc(4096, 2048, *rows)
            for _ in range(5):
                r.clear_on_flush()
                r.draw_model_optimized(g, s.tri_count, P=s.P, bitmap=tex, phong=True)
                r.complete_all_work()
            r.synchronize()
            got.append((rows, r.download()))
    finally:
        r.close()
    for (r0, r1), (gc, gz) in got:
        assert (gz.view(np.uint32) == oz[r0:r1].view(np.uint32)).all(), (r0, r1)
        assert (gc == oc[r0:r1]).all(), (r0, r1)


def test_draw_tables_change_between_frames(gpu):
    """Each scratch set re-sends its draw / texture tables only when their
    bytes change: frames that alternate geometry and texture on the same set
    (frame k uses set k % 2) must each render their own draws."""
    a = scenes.random_soup(3000, 256, 192, radius=16, seed=61)
    b = scenes.random_soup(3000, 256, 192, radius=16, seed=62)
    plan = [(a, a), (a, a), (b, b), (a, a), (a, b), (b, a), (b, a), (a, a)]  # (geometry, texture source)
    r = prk.Renderer(0)
    try:
        r.target_alloc(256, 192)
        r.set_camera(a.prk_transform(), a.prk_lights())
        geo = {id(a): r.geometry(a.vertices, a.colors, a.normals, a.uvs),
               id(b): r.geometry(b.vertices, b.colors, b.normals, b.uvs)}
        tex = {id(a): r.texture(a.texture), id(b): r.texture(b.texture)}
        got = []
        for g, t in plan:
            r.clear_on_flush()
            r.draw_model_optimized(geo[id(g)], g.tri_count, P=g.P, bitmap=tex[id(t)], phong=True)
            r.complete_all_work()
            r.synchronize()
            got.append(r.download())
    finally:
        r.close()
    ta, tb = a.texture, b.texture
    for k, ((g, t), (gc, gz)) in enumerate(zip(plan, got)):
        g.texture = ta if t is a else tb
        oc, oz, _, _ = O.render(g)
        g.texture = ta if g is a else tb
        assert (gz.view(np.uint32) == oz.view(np.uint32)).all(), k
        assert (gc == oc).all(), k


def test_row_band(gpu):
    s = scenes.random_soup(10000, 512, 512, radius=20, seed=17)
    oc, oz, ow, _ = O.render(s)
    for r0, r1 in [(0, 128), (128, 300), (300, 512), (37, 91)]:
        gc, gz, gw, _ = prk.render_scene(s, rows=(r0, r1))
        assert (gz.view(np.uint32) == oz[r0:r1].view(np.uint32)).all(), (r0, r1)
        assert (gc == oc[r0:r1]).all(), (r0, r1)
        assert (gw == ow[r0:r1]).all(), (r0, r1)


def _band_edge_soup(n, W, H, edges, seed):
    """Small triangles crowded around the band boundaries `edges` (centroid y
    within 4 px of one), some large ones, and one in twenty with a vertex at
    or behind the near plane (D - z <= 0.2: ProjectVertex's (0, 0, 0))."""
    s = scenes.random_soup(n, W, H, radius=3, seed=seed)
    rng = np.random.default_rng(seed + 1)
    cam = s.transform
    cy = np.asarray(edges, float)[rng.integers(0, len(edges), n)] + rng.uniform(-4, 4, n)
    cxy = np.stack([rng.uniform(0, W, n), cy], 1)
    rad = np.where(rng.random(n) < 0.1, 40.0, np.where(rng.random(n) < 0.5, 1.5, 3.0))
    sc = cxy[:, None, :] + rng.uniform(-1, 1, (n, 3, 2)) * rad[:, None, None]
    e1, e2 = sc[:, 1] - sc[:, 0], sc[:, 2] - sc[:, 0]
    flip = e1[:, 0] * e2[:, 1] - e1[:, 1] * e2[:, 0] > 0
    sc[flip, 1], sc[flip, 2] = sc[flip, 2].copy(), sc[flip, 1].copy()
    z = rng.uniform(-1, 1, n)[:, None] + rng.uniform(-0.1, 0.1, (n, 3))
    near = rng.random(n) < 0.05
    z[near, rng.integers(0, 3, int(near.sum()))] = rng.choice([3.81, 3.9, 4.0, 4.5], int(near.sum()))
    D, F, M2P, cx0, cy0 = cam
    x = (sc[..., 0] - cx0) * (D - z) / M2P / F
    y = (sc[..., 1] - cy0) * (D - z) / M2P / F
    s.vertices = np.stack([x, y, z], -1).reshape(-1, 3).astype(np.float32)
    return s


@pytest.mark.parametrize("draws", ["one", "two"])
def test_band_edges_quick_test(gpu, draws):
    """k_bin_band's quick band test (band_far, the hardware reciprocal in
    place of ProjectVertex's division) only drops triangles the exact test
    drops: triangles crowded around the band boundaries, near-plane vertices,
    an object offset P, runs of 2048 (coalesced) and a tail run; "two": two
    draws (every run through the per-thread loads).  Every band equals the
    oracle's frame rows."""
    W = H = 512
    bands = [(0, 128), (128, 300), (300, 301), (37, 91), (91, 512), (255, 257)]
    edges = sorted({e for b in bands for e in b if 0 < e < H})
    s = _band_edge_soup(7000, W, H, edges, seed=91)
    s.P = (0.0, 0.003, 0.01)
    if draws == "two":
        s.draws = [(0, 3001, s.texture), (3001, s.tri_count - 3001, s.texture)]
    oc, oz, ow, _ = O.render(s)
    for r0, r1 in bands:
        gc, gz, gw, _ = prk.render_scene(s, rows=(r0, r1))
        compare((gc, gz, gw, None), (oc[r0:r1], oz[r0:r1], ow[r0:r1], None), label="band %d-%d" % (r0, r1))


def test_mixed_semantics_one_frame(gpu):
    """Draws of different semantics in one flush share the z-buffer in order."""
    a = scenes.random_soup(3000, 256, 256, radius=16, seed=31)
    b = scenes.random_soup(3000, 256, 256, radius=16, seed=32, textured=False)
    oc, oz, ow, _ = O.render(a)
    oc, oz, ow2, _ = O.render(b, semantics=abi.PRK_SEM_SCALAR, phong=False, color=oc, z=oz)
    ow = np.where(ow2 >= 0, ow2 + a.tri_count, ow)
    r = prk.Renderer()
    try:
        r.target_alloc(256, 256)
        r.clear()
        r.set_debug(True)
        r.set_camera(a.prk_transform(), a.prk_lights())
        ga = r.geometry(a.vertices, a.colors, a.normals, a.uvs)
        gb = r.geometry(b.vertices, b.colors, b.normals, b.uvs)
        tex = r.texture(a.texture)
        r.draw_model_optimized(ga, a.tri_count, bitmap=tex)
        r.draw_model(gb, b.tri_count, phong=False)
        r.complete_all_work()
        gc, gz = r.download()
        gw = r.winners()
    finally:
        r.close()
    assert (gz.view(np.uint32) == oz.view(np.uint32)).all()
    assert (gc == oc).all()
    assert (gw == ow).all()


@pytest.mark.parametrize("sem", [abi.PRK_SEM_AVX, abi.PRK_SEM_AVX_ST])
def test_tie_rules(gpu, sem):
    """Exact positional duplicates (equal z at every shared pixel): strict
    '>' keeps the EARLIER fragment (projekt.cpp:2219), the single-thread
    overload's '>=' the LATER one (3205)."""
    s = scenes.with_ties(scenes.random_soup(4000, 256, 256, radius=20, seed=12), seed=5)
    run_both(s, semantics=sem)


def test_single_thread_overload_clipping(gpu):
    """DrawModelOptimized(Buffer,...) (2350-3358) with spans over every
    border: its left-clip XOffset quirk (2508) on every left-clipped span."""
    run_both(scenes.random_soup(3000, 512, 512, radius=200, seed=6, centroid_margin=150),
             semantics=abi.PRK_SEM_AVX_ST)


def test_mixed_tie_rules_one_frame(gpu):
    """Queue and single-thread draws alternating in one frame over tie-heavy
    geometry: each pair's tie rule holds against every earlier fragment."""
    s = scenes.with_ties(scenes.random_soup(6000, 256, 256, radius=20, seed=13), seed=6)
    T = s.tri_count
    cut = [0, T // 5, 2 * T // 5, 3 * T // 5, T]
    s.draws = [(cut[k], cut[k + 1] - cut[k], s.texture, abi.PRK_SEM_AVX if k % 2 == 0 else abi.PRK_SEM_AVX_ST)
               for k in range(4)]
    run_both(s)


def test_mixed_tie_rules_with_scalar(gpu):
    """Single-thread, queue and scalar draws in one frame (the mixed-mode
    sweep path, not the all-AVX one)."""
    s = scenes.with_ties(scenes.random_soup(3000, 256, 256, radius=20, seed=14), seed=7)
    T = s.tri_count
    s.draws = [(0, T // 3, s.texture, abi.PRK_SEM_AVX_ST), (T // 3, T // 3, None, abi.PRK_SEM_SCALAR),
               (2 * T // 3, T - 2 * (T // 3), s.texture, abi.PRK_SEM_AVX)]
    run_both(s)


def _sphere_scene(W=512, H=512):
    V, Cc, N, UV = prk.construct_sphere()
    base = scenes.random_soup(1, W, H, seed=0)
    return scenes.Scene(W, H, V, Cc, N, UV, base.transform, scenes.LIGHTS_ONE, scenes.AMBIENT_ONE,
                        base.texture, P=(0.0, 0.0, 2.0), name="sphere")


@pytest.mark.parametrize("sem", [abi.PRK_SEM_AVX, abi.PRK_SEM_AVX_ST])
def test_whole_object_construct_sphere(gpu, sem):
    """ConstructSphere (projekt.cpp:4123-4289) submitted as ONE
    render_entry_3d_object: one active edge table for all 2208 triangles, so
    spans pair edges of different triangles (3654-3869), against the oracle's
    whole-object walk.  Differs from the per-triangle image."""
    s = _sphere_scene()
    g, o = run_both(s, semantics=sem, tris_per_object=s.tri_count, threads=1)
    per_tri = O.render(s, semantics=sem)
    assert (g[1].view(np.uint32) != per_tri[1].view(np.uint32)).any()  # whole-object is really different
    assert (g[2] >= 0).sum() > 10000


@pytest.mark.parametrize("tile", [(32, 8), (64, 8)])
def test_whole_object_narrow_tiles(gpu, tile):
    """The span path (whole-object AETs) at the automatic tile's narrow
    widths: ConstructSphere as one object and random 5-triangle objects."""
    s = _sphere_scene()
    g = prk.render_scene(s, tile=tile, tris_per_object=s.tri_count)
    compare(g, O.render(s, tris_per_object=s.tri_count), label="sphere %dx%d" % tile)
    s2 = scenes.random_soup(600, 256, 256, radius=40, seed=17)
    g2 = prk.render_scene(s2, tile=tile, tris_per_object=5)
    compare(g2, O.render(s2, tris_per_object=5), label="objects %dx%d" % tile)


@pytest.mark.parametrize("tpo,seed", [(2, 1), (5, 2), (16, 3), (24, 4), (40, 5)])
def test_whole_object_random_objects(gpu, tpo, seed):
    """Random objects of several triangles, clipped on every side, with ties:
    spans across unrelated triangles, crossing swaps, expiry mid-list.  The
    thread walk keeps the list in LDS for objects of up to 48 edges and the
    walked pair's records in registers (dense rows evict them pair by pair);
    24 and 40 triangles mix objects under and over that size in one launch."""
    s = scenes.with_ties(scenes.random_soup(3000, 256, 256, radius=30, seed=seed, centroid_margin=30), seed=seed)
    run_both(s, tris_per_object=tpo)


def test_whole_object_mixed_passes(gpu):
    """Per-triangle and whole-object draws, queue and single-thread, in one
    frame: the passes z-test against each other in submission order."""
    s = scenes.with_ties(scenes.random_soup(4000, 256, 256, radius=20, seed=17), seed=8)
    T = s.tri_count
    q = T // 4
    s.draws = [(0, q, s.texture, abi.PRK_SEM_AVX, 1), (q, q, s.texture, abi.PRK_SEM_AVX, 6),
               (2 * q, q, s.texture, abi.PRK_SEM_AVX_ST, 1), (3 * q, T - 3 * q, s.texture, abi.PRK_SEM_AVX_ST, 3)]
    run_both(s)


def _render_src(scene, kind, words, semantics, phong=True, textured=True):
    r = prk.Renderer()
    try:
        r.target_alloc(scene.width, scene.height)
        r.clear()
        r.set_debug(True)
        r.set_camera(scene.prk_transform(), scene.prk_lights())
        tex = r.texture(scene.texture) if textured else None
        (r.draw_edges if kind == "edges" else r.draw_spans)(words, semantics=semantics, bitmap=tex, phong=phong)
        r.complete_all_work()
        c, z = r.download()
        return c, z, r.winners(), r.stats()
    finally:
        r.close()


@pytest.mark.parametrize("sem", [abi.PRK_SEM_AVX, abi.PRK_SEM_AVX_ST])
def test_draw_caller_edge_list(gpu, sem):
    """DrawModelOptimized* on a ready edge_info list (prk_draw_edges): the
    oracle's FillEdgeTable output of a 60-triangle object, drawn by the GPU's
    AET walk, equals the oracle's walk of the same list."""
    s = scenes.random_soup(60, 256, 256, radius=60, seed=43, textured=True, centroid_margin=40)
    words = O.fill_edge_table_words(s, 0, 60)
    compare(_render_src(s, "edges", words, sem), O.render_edges(s, words, semantics=sem), label="edges")


@pytest.mark.parametrize("local", ["1", "0"])
def test_small_objects_and_caller_edges_one_pass(gpu, local, monkeypatch):
    """Small triangle objects and a caller edge list in one span pass: the
    objects' edges sorted per object (k_obj_sort_local) or by the radix sort
    (PRK_OBJ_LOCAL_SORT=0), the caller's list gathered after them; the
    oracle draws the objects, then the list over them."""
    monkeypatch.setenv("PRK_OBJ_LOCAL_SORT", local)
    s = scenes.with_ties(scenes.random_soup(2400, 256, 256, radius=18, seed=44, centroid_margin=18), seed=44)
    lst = scenes.random_soup(40, 256, 256, radius=50, seed=45, centroid_margin=40)
    lst.transform, lst.lights, lst.ambient, lst.texture = s.transform, s.lights, s.ambient, s.texture
    words = O.fill_edge_table_words(lst, 0, 40)
    r = prk.Renderer()
    try:
        r.target_alloc(s.width, s.height)
        r.clear()
        r.set_camera(s.prk_transform(), s.prk_lights())
        tex = r.texture(s.texture)
        g = r.geometry(s.vertices, s.colors, s.normals, s.uvs)
        r.draw(abi.PRK_SEM_AVX, g, s.tri_count, P=s.P, bitmap=tex, phong=True, tris_per_object=8)
        r.draw_edges(words, semantics=abi.PRK_SEM_AVX, bitmap=tex, phong=True)
        r.complete_all_work()
        gc, gz = r.download()
    finally:
        r.close()
    oc, oz, _, _ = O.render(s, tris_per_object=8)
    oc, oz, _, _ = O.render_edges(lst, words, color=oc, z=oz)
    assert np.array_equal(gz.view(np.uint32), oz.view(np.uint32))
    assert np.array_equal(gc, oc)


@pytest.mark.parametrize("sem", [abi.PRK_SEM_AVX, abi.PRK_SEM_AVX_ST])
def test_draw_caller_spans(gpu, sem):
    """Caller-built spans (DoLineRenderWork / DoBufferLineRenderWork work
    records, prk_draw_spans): random end points over every border, random
    rows, overlapping spans with equal z."""
    rng = np.random.default_rng(5)
    s = scenes.random_soup(1, 256, 192, seed=0, textured=True)
    n = 3000
    w = np.zeros((n, 25), np.uint32)
    f = w.view(np.float32)
    x0 = rng.uniform(-40, 260, n)
    x1 = x0 + rng.uniform(-5, 120, n)
    for k, x in ((0, x0), (12, x1)):
        zc = rng.uniform(-1, 1, n)
        iz = 1.0 / (4.0 - zc)
        f[:, k + 0] = x
        f[:, k + 1] = zc
        f[:, k + 2] = iz
        f[:, k + 3] = rng.uniform(-0.1, 1.1, n) * iz
        f[:, k + 4] = rng.uniform(-0.1, 1.1, n) * iz
        f[:, k + 5:k + 9] = rng.uniform(0, 1, (n, 4))
        nv = rng.normal(size=(n, 3))
        f[:, k + 9:k + 12] = nv / np.linalg.norm(nv, axis=1, keepdims=True)
    f[n // 2:, 1] = f[: n - n // 2, 1]  # repeat z: ties between spans
    f[n // 2:, 13] = f[: n - n // 2, 13]
    w[:, 24] = rng.integers(0, 192, n).astype(np.uint32)
    compare(_render_src(s, "spans", w, sem), O.render_spans(s, w, semantics=sem), label="spans")


@pytest.mark.parametrize("phong", [False, True])
def test_whole_object_scalar_construct_sphere(gpu, phong):
    """DrawModel (projekt.cpp:162-601) on ConstructSphere submitted as ONE
    render_entry_3d_object: one active edge table for the whole object
    (insertion / expiry / pairing 168-300, stepping 540-598), Gouraud and
    untextured Phong spans paired across triangles, against the oracle's
    whole-object walk.  Differs from the per-triangle image."""
    s = _sphere_scene()
    s.texture = None
    g, o = run_both(s, semantics=abi.PRK_SEM_SCALAR, phong=phong, tris_per_object=s.tri_count, threads=1,
                    label="sphere scalar phong=%d" % phong)
    per_tri = O.render(s, semantics=abi.PRK_SEM_SCALAR, phong=phong)
    assert (g[1].view(np.uint32) != per_tri[1].view(np.uint32)).any()
    assert (g[2] >= 0).sum() > 10000


@pytest.mark.parametrize("phong,textured", [(False, False), (True, False), (False, True), (True, True)])
@pytest.mark.parametrize("tpo,seed", [(2, 1), (5, 2), (16, 3)])
def test_whole_object_scalar_random_objects(gpu, tpo, seed, phong, textured):
    """Random DrawModel objects of several triangles in every scalar mode,
    clipped on every side (the one-past-the-row store at the right border
    included), with ties."""
    s = scenes.with_ties(scenes.random_soup(2000, 256, 192, radius=30, seed=seed, centroid_margin=30,
                                            textured=textured, lights=scenes.LIGHTS_TWO,
                                            ambient=scenes.AMBIENT_TWO), seed=seed)
    run_both(s, semantics=abi.PRK_SEM_SCALAR, phong=phong, tris_per_object=tpo,
             label="scalar objects tpo=%d phong=%d tex=%d" % (tpo, phong, textured))


@pytest.mark.parametrize("phong", [False, True])
def test_whole_object_scalar_c2_one_object(gpu, phong):
    """C2 (the ~70k-triangle bunny stand-in, 1920x1080) submitted as ONE
    object through DrawModel, Gouraud and untextured Phong: a wave walks its
    active edge table (hundreds of edges per row), against the oracle's
    whole-object walk."""
    s = scenes.displaced_sphere(70000, 1920, 1080, seed=3)
    g, o = run_both(s, semantics=abi.PRK_SEM_SCALAR, phong=phong, tris_per_object=s.tri_count,
                    label="C2 one object phong=%d" % phong)
    assert (g[2] >= 0).sum() > 100000


@pytest.mark.parametrize("sem", [abi.PRK_SEM_AVX, abi.PRK_SEM_AVX_ST, abi.PRK_SEM_SCALAR])
def test_whole_object_chunked_walk(gpu, sem, monkeypatch):
    """The chunked walk of large objects (prk_spans.hip k_pr_*): the rows cut
    into chunks walked at once, each from its first row's sorted list, the
    chunks whose start was not the true list walked again in order.
    ConstructSphere as one object: bit for bit the oracle's sequential walk
    and the plain workgroup walk (PRK_OBJ_ROWS=0).  Overlapping random
    700-triangle objects (crossing edges: many chunk starts are not the sorted
    list) against both too.  Sphere strips next to soup objects whose
    triangles cross the top border (rows with one active edge: walked row by
    row from the first) in one pass."""
    s = _sphere_scene()
    if sem == abi.PRK_SEM_SCALAR:
        s.texture = None
    g, o = run_both(s, semantics=sem, phong=True, tris_per_object=s.tri_count, threads=1,
                    label="sphere chunked sem=%d" % sem)
    assert g[3]["objects_chunked"] == 1 and g[3]["objects_walked"] == 0, g[3]
    monkeypatch.setenv("PRK_OBJ_ROWS", "0")
    w = prk.render_scene(s, semantics=sem, phong=True, tris_per_object=s.tri_count)
    monkeypatch.delenv("PRK_OBJ_ROWS")
    assert w[3]["objects_chunked"] == 0 and w[3]["objects_walked"] == 1, w[3]
    for k in range(3):
        assert np.array_equal(g[k].view(np.uint32), w[k].view(np.uint32)), k
    soup = scenes.with_ties(scenes.random_soup(2800, 384, 256, radius=40, seed=9, centroid_margin=40), seed=9)
    if sem == abi.PRK_SEM_SCALAR:
        soup.texture = None
    inner = scenes.random_soup(2800, 384, 256, radius=40, seed=19, centroid_margin=-45)  # on screen: even rows
    if sem == abi.PRK_SEM_SCALAR:
        inner.texture = None
    c, _ = run_both(inner, semantics=sem, phong=True, tris_per_object=700, threads=1,
                    label="crossing objects chunked sem=%d" % sem)
    assert c[3]["objects_chunked"] == 4, c[3]
    monkeypatch.setenv("PRK_OBJ_ROWS", "0")
    cw = prk.render_scene(inner, semantics=sem, phong=True, tris_per_object=700)
    monkeypatch.delenv("PRK_OBJ_ROWS")
    for k in range(3):
        assert np.array_equal(c[k].view(np.uint32), cw[k].view(np.uint32)), k
    # without the warm-up most chunks start from a list that is not the true
    # one: the check catches them and k_pr_fix walks them again
    monkeypatch.setenv("PRK_OBJ_CHUNK_WARMUP", "0")
    cf = prk.render_scene(inner, semantics=sem, phong=True, tris_per_object=700)
    monkeypatch.delenv("PRK_OBJ_CHUNK_WARMUP")
    assert cf[3]["object_chunks_rewalked"] > 0, cf[3]
    for k in range(3):
        assert np.array_equal(cf[k].view(np.uint32), cw[k].view(np.uint32)), k
    # sphere strips (chunked) and soup objects crossing the top border (walked) in one pass
    V, Cc, N, UV = prk.construct_sphere()
    big = scenes.Scene(384, 256, np.concatenate([V[:3 * 64 * 20] * 0.6, soup.vertices[:3 * 64 * 10]]),
                       np.concatenate([Cc[:3 * 64 * 20], soup.colors[:3 * 64 * 10]]),
                       np.concatenate([N[:3 * 64 * 20], soup.normals[:3 * 64 * 10]]),
                       np.concatenate([UV[:3 * 64 * 20], soup.uvs[:3 * 64 * 10]]), soup.transform, soup.lights,
                       soup.ambient, soup.texture, P=(0.0, 0.0, 2.0), name="mixed rows")
    g2, _ = run_both(big, semantics=sem, phong=True, tris_per_object=64, threads=1, label="mixed rows sem=%d" % sem)
    st = g2[3]
    assert st["objects_chunked"] > 0 and st["objects_walked"] > 0, st
    assert st["objects_chunked"] + st["objects_walked"] == 30, st


@pytest.mark.parametrize("sem", [abi.PRK_SEM_AVX, abi.PRK_SEM_AVX_ST, abi.PRK_SEM_SCALAR])
@pytest.mark.parametrize("tpo", [3, 16, 40])
def test_whole_object_segments(gpu, sem, tpo, monkeypatch):
    """Small objects walked as segments (prk_spans.hip k_obj_seg): an
    object's rows split where its list runs empty, each stretch walked by a
    thread of its own from an empty list.  Scattered triangles (many
    segments per object, some overlapping: crossings and ties inside a
    segment), clipped on every side: the oracle's whole-object walk, and the
    thread-per-object walk (PRK_OBJ_SEGMENTS=0), bit for bit."""
    s = scenes.with_ties(scenes.random_soup(4000, 512, 384, radius=24, seed=tpo, centroid_margin=24), seed=tpo)
    if sem == abi.PRK_SEM_SCALAR:
        s.texture = None
    g, _ = run_both(s, semantics=sem, phong=True, tris_per_object=tpo, threads=1,
                    label="segments tpo=%d sem=%d" % (tpo, sem))
    monkeypatch.setenv("PRK_OBJ_SEGMENTS", "0")
    w = prk.render_scene(s, semantics=sem, phong=True, tris_per_object=tpo)
    monkeypatch.delenv("PRK_OBJ_SEGMENTS")
    for k in range(3):
        assert np.array_equal(g[k].view(np.uint32), w[k].view(np.uint32)), k


@pytest.mark.parametrize("segments", ["1", "0"])
def test_span_slots_marked_by_the_walks(gpu, segments, monkeypatch):
    """Frames without large objects skip the memset of the span slots: the
    thread and segment walks mark the slots they leave unused (spans that
    cover nothing, rounding of the segments' bounds) themselves.  One context
    draws frames whose slot ranges shrink and move (stale slots of the
    previous frame would be binned), scalar and AVX, objects of 1-21
    triangles, clipped: each frame equals the oracle's."""
    monkeypatch.setenv("PRK_OBJ_SEGMENTS", segments)
    frames = [(scenes.random_soup(6000, 384, 256, radius=30, seed=81, centroid_margin=30), abi.PRK_SEM_AVX, 16),
              (scenes.random_soup(1500, 384, 256, radius=10, seed=82, centroid_margin=12), abi.PRK_SEM_AVX, 5),
              (scenes.random_soup(3000, 384, 256, radius=20, seed=83, centroid_margin=40), abi.PRK_SEM_SCALAR, 21),
              (scenes.random_soup(800, 384, 256, radius=6, seed=84), abi.PRK_SEM_AVX, 1)]
    r = prk.Renderer(0)
    try:
        r.target_alloc(384, 256)
        for s, sem, tpo in frames:
            if sem == abi.PRK_SEM_SCALAR:
                s.texture = None
            r.clear()
            r.set_camera(s.prk_transform(), s.prk_lights())
            g = r.geometry(s.vertices, s.colors, s.normals, s.uvs)
            tex = r.texture(s.texture) if sem == abi.PRK_SEM_AVX else None
            r.draw(sem, g, s.tri_count, P=s.P, bitmap=tex, phong=True, tris_per_object=tpo)
            r.complete_all_work()
            r.synchronize()
            gc, gz = r.download()
            oc, oz, _, _ = O.render(s, semantics=sem, phong=True, tris_per_object=tpo)
            assert (gz.view(np.uint32) == oz.view(np.uint32)).all(), (sem, tpo)
            assert (gc == oc).all(), (sem, tpo)
    finally:
        r.close()


@pytest.mark.parametrize("sem", [abi.PRK_SEM_AVX, abi.PRK_SEM_SCALAR])
@pytest.mark.parametrize("tpo", [2, 16, 21])
def test_whole_object_local_sort(gpu, sem, tpo, monkeypatch):
    """Passes whose objects have at most 64 edges sort each object's edges in
    one wave (prk_spans.hip k_obj_sort_local: rank of the MergeSort key) in
    place of the device radix sort + gather: equal YMin everywhere (ties in
    MergeSort's recursion order), 21 triangles = 63 edges at the limit; the
    oracle, and the radix sort (PRK_OBJ_LOCAL_SORT=0), bit for bit."""
    s = scenes.with_ties(scenes.random_soup(3000, 384, 256, radius=20, seed=70 + tpo, centroid_margin=20),
                         seed=tpo)
    if sem == abi.PRK_SEM_SCALAR:
        s.texture = None
    g, _ = run_both(s, semantics=sem, phong=True, tris_per_object=tpo, threads=1,
                    label="local sort tpo=%d sem=%d" % (tpo, sem))
    monkeypatch.setenv("PRK_OBJ_LOCAL_SORT", "0")
    w = prk.render_scene(s, semantics=sem, phong=True, tris_per_object=tpo)
    monkeypatch.delenv("PRK_OBJ_LOCAL_SORT")
    for k in range(3):
        assert np.array_equal(g[k].view(np.uint32), w[k].view(np.uint32)), k


@pytest.mark.parametrize("sem", [abi.PRK_SEM_AVX, abi.PRK_SEM_AVX_ST, abi.PRK_SEM_SCALAR])
@pytest.mark.parametrize("tpo", [64, 700])
def test_whole_object_wave_walk(gpu, sem, tpo):
    """Objects large enough for the one-wave walk (k_obj_walk_wave): random
    triangles with ties and clipping, so spans pair unrelated triangles, lists
    cross 64-entry chunks, both swap passes fire and entries expire mid-list."""
    s = scenes.with_ties(scenes.random_soup(2800, 384, 256, radius=40, seed=tpo, centroid_margin=40), seed=tpo)
    run_both(s, semantics=sem, phong=True, tris_per_object=tpo,
             label="wave objects tpo=%d sem=%d" % (tpo, sem))


@pytest.mark.parametrize("sem", [abi.PRK_SEM_AVX, abi.PRK_SEM_SCALAR])
def test_whole_object_long_active_lists(gpu, sem):
    """One object whose active edge list holds ~14k edges per row (beyond the
    wave walk's 4096-entry LDS list: the list lives in device memory), with
    hundreds of insertions per row: the batched insertion against the
    oracle's one-at-a-time list scan (projekt.cpp:3654-3713)."""
    s = scenes.random_soup(30000, 1024, 128, radius=24, seed=17)
    if sem == abi.PRK_SEM_SCALAR:
        s.texture = None
    run_both(s, semantics=sem, phong=sem != abi.PRK_SEM_SCALAR, tris_per_object=s.tri_count, threads=1,
             label="long lists sem=%d" % sem)


@pytest.mark.parametrize("lds", ["1", "0"])
@pytest.mark.parametrize("sem", [abi.PRK_SEM_AVX, abi.PRK_SEM_AVX_ST, abi.PRK_SEM_SCALAR])
def test_whole_object_big_walk(gpu, sem, lds, monkeypatch):
    """The huge-object walk (prk_spans.hip k_obj_walk_lds / k_obj_walk_big:
    one workgroup over a list in LDS or in device memory, the spans set up
    afterwards from a replay of every pair) forced onto objects that would
    fit the LDS slot classes (PRK_OBJ_BIG_MIN=0,
    PRK_OBJ_ROWS=0), and their sizes by the many-workgroup histogram
    (PRK_OBJ_HUGE_EDGES): ConstructSphere as one object, overlapping 700- and
    64-triangle objects with ties and clipping on every side (odd rows: an
    unpaired last entry), a row band (rows above it paired, not emitted) —
    against the oracle and the one-wave walk (PRK_OBJ_BIG=0), bit for bit."""
    monkeypatch.setenv("PRK_OBJ_BIG_MIN", "0")
    monkeypatch.setenv("PRK_OBJ_ROWS", "0")
    monkeypatch.setenv("PRK_OBJ_HUGE_EDGES", "1000")  # the many-workgroup sizing (k_maxact_huge_*) too
    monkeypatch.setenv("PRK_OBJ_LDSWALK", lds)  # the list in LDS (k_obj_walk_lds) or device memory
    sph = _sphere_scene()
    soup = scenes.with_ties(scenes.random_soup(2800, 384, 256, radius=40, seed=23, centroid_margin=40), seed=23)
    if sem == abi.PRK_SEM_SCALAR:
        sph.texture = None
        soup.texture = None
    for s, tpo in ((sph, sph.tri_count), (soup, 700), (soup, 64)):
        label = "big walk %s tpo=%d sem=%d" % (s.name, tpo, sem)
        g, o = run_both(s, semantics=sem, phong=True, tris_per_object=tpo, threads=1, label=label)
        monkeypatch.setenv("PRK_OBJ_BIG", "0")
        w = prk.render_scene(s, semantics=sem, phong=True, tris_per_object=tpo)
        monkeypatch.delenv("PRK_OBJ_BIG")
        for k in range(3):
            assert np.array_equal(g[k].view(np.uint32), w[k].view(np.uint32)), (label, k)
    oc, oz, ow, _ = O.render(soup, semantics=sem, phong=True, threads=1, tris_per_object=700)
    r0, r1 = 61, 190
    gc, gz, gw, _ = prk.render_scene(soup, semantics=sem, phong=True, tris_per_object=700, rows=(r0, r1))
    assert (gz.view(np.uint32) == oz[r0:r1].view(np.uint32)).all()
    assert (gc == oc[r0:r1]).all()
    assert (gw == ow[r0:r1]).all()


def _degenerate_soup(seed):
    """A clipped soup with hostile vertices: at the camera plane (distance 0),
    behind it, NaN and infinite coordinates, and zero-area slivers — what
    FillEdgeTable's cull and clip (3926-4066) must sort out before any list
    sees an edge."""
    s = scenes.with_ties(scenes.random_soup(1500, 256, 160, radius=30, seed=seed, centroid_margin=30), seed=seed)
    D = s.transform[0]
    v = s.vertices.reshape(-1, 3, 3).copy()
    rng = np.random.default_rng(seed)
    idx = rng.choice(len(v), 60, replace=False)
    v[idx[:10], 0, 2] = D                 # on the camera plane
    v[idx[10:20], 1, 2] = D + 0.5         # behind the camera
    v[idx[20:30], 2, 0] = np.nan
    v[idx[30:40], 0, 1] = np.inf
    v[idx[40:50], 1] = v[idx[40:50], 0]   # two equal vertices: zero area
    v[idx[50:60], 2] = v[idx[50:60], 0] + (v[idx[50:60], 1] - v[idx[50:60], 0]) * 0.5  # collinear
    s.vertices = v.reshape(-1, 3).astype(np.float32)
    return s


@pytest.mark.parametrize("path", ["default", "big", "bigmem", "wave"])
@pytest.mark.parametrize("tpo", [1, 8, 64, 500])
def test_degenerate_geometry_every_walk(gpu, path, tpo, monkeypatch):
    """Hostile vertices (camera plane, behind the camera, NaN / inf, zero-area
    and collinear triangles) per triangle and in objects of 8 / 64 / 500
    triangles, through the default walks, the huge-object walk (forced) and
    the one-wave walk (forced): the oracle's image, bit for bit."""
    if path in ("big", "bigmem"):
        monkeypatch.setenv("PRK_OBJ_BIG_MIN", "0")
        monkeypatch.setenv("PRK_OBJ_ROWS", "0")
        monkeypatch.setenv("PRK_OBJ_HUGE_EDGES", "100")
        monkeypatch.setenv("PRK_OBJ_LDSWALK", "1" if path == "big" else "0")
    elif path == "wave":
        monkeypatch.setenv("PRK_OBJ_BIG_MIN", "0")
        monkeypatch.setenv("PRK_OBJ_ROWS", "0")
        monkeypatch.setenv("PRK_OBJ_BIG", "0")
    s = _degenerate_soup(11 + tpo)
    run_both(s, semantics=abi.PRK_SEM_AVX, phong=True, tris_per_object=tpo, threads=1,
             label="degenerate tpo=%d %s" % (tpo, path))


def test_whole_object_mid_lists_lds(gpu):
    """Objects whose lists stay in LDS (<= 4096 edges per object) while
    several hundred edges enter per row: the batched insertion in LDS."""
    s = scenes.with_ties(scenes.random_soup(2700, 512, 64, radius=30, seed=23), seed=23)
    run_both(s, tris_per_object=1300, threads=1, label="mid lists")


C3B_ONE_OBJECT = __import__("os").path.join(__import__("os").path.dirname(__import__("os").path.abspath(__file__)),
                                             "golden", "c3b_one_object.json")


def test_c3b_one_object_golden(gpu):
    """The headline C3b geometry (4096^2, 1M triangles, Phong + texture)
    submitted as ONE render_entry_3d_object: one active edge table of ~3M
    edges, ~15k active per row.  The oracle needs minutes for it (its
    insertion scans the list per edge, as the reference does), so its frame
    was rendered once by tools/make_golden.py and is pinned here as per-band
    SHA-256 digests of colour, z and winner map."""
    import hashlib
    import json
    ref = json.load(open(C3B_ONE_OBJECT))
    s = scenes.random_soup(ref["tris"], ref["width"], ref["height"], radius=ref["radius"], seed=ref["seed"])
    h = hashlib.sha256()
    for a in (s.vertices, s.colors, s.normals, s.uvs, s.texture.texels):
        h.update(np.ascontiguousarray(a).tobytes())
    assert h.hexdigest() == ref["inputs"], "the generated scene differs from the one the digests were made from"
    gc, gz, gw, st = prk.render_scene(s, tris_per_object=s.tri_count)
    assert int((gw >= 0).sum()) == ref["covered"]
    rows = ref["band_rows"]
    bad = []
    for b, want in enumerate(ref["bands"]):
        sl = slice(b * rows, (b + 1) * rows)
        got = [hashlib.sha256(np.ascontiguousarray(a[sl]).tobytes()).hexdigest() for a in (gc, gz, gw)]
        if got != want:
            bad.append(b)
    assert not bad, "bands differing from the oracle's frame: %s" % bad[:16]


@pytest.mark.parametrize("tpo", [1, 5, 300])
@pytest.mark.parametrize("setup", [abi.PRK_SETUP_PHONG, abi.PRK_SETUP_BITMAP, abi.PRK_SETUP_PHONG | abi.PRK_SETUP_BITMAP,
                                   0])
def test_fill_edge_table_inputs(gpu, tpo, setup):
    """FillEdgeTable's own PhongShading and Object->Bitmap decide the edge
    colours an untextured non-Phong DrawModel interpolates
    (projekt.cpp:4012-4063): PhongShading = 1 stores the raw colours (drawn
    unlit), PhongShading = 0 lights them per vertex from the vertex colour,
    or from white when the object has a Bitmap (4034-4054) — whatever the
    DrawModel call's own flags."""
    s = scenes.with_ties(scenes.random_soup(3000, 256, 256, radius=20, seed=31 + tpo, textured=False), seed=5)
    run_both(s, semantics=abi.PRK_SEM_SCALAR, phong=False, tris_per_object=tpo, threads=1, setup=setup,
             label="setup=%d tpo=%d" % (setup, tpo))


def test_fill_edge_table_inputs_undefined_rejected(gpu):
    """Edge fields FillEdgeTable never wrote are undefined in the reference:
    a Phong draw of edges set up without PhongShading (MinNormal,
    4012-4064), a textured draw of edges set up without a Bitmap (the
    U/V/(1/z) gradients, 4078-4089)."""
    s = scenes.random_soup(10, 64, 64, seed=0)
    r = prk.Renderer()
    try:
        g = r.geometry(s.vertices, s.colors, s.normals, s.uvs)
        tex = r.texture(s.texture)
        for sem, phong, t, setup in [(abi.PRK_SEM_AVX, True, tex, abi.PRK_SETUP_BITMAP),
                                     (abi.PRK_SEM_AVX, True, tex, abi.PRK_SETUP_PHONG),
                                     (abi.PRK_SEM_SCALAR, True, None, 0),
                                     (abi.PRK_SEM_SCALAR, False, tex, abi.PRK_SETUP_PHONG)]:
            with pytest.raises(prk.PrkError) as e:
                r.draw(sem, g, 10, bitmap=t, phong=phong, setup=setup)
            assert e.value.code == abi.PRK_ERR_UNSUPPORTED
    finally:
        r.close()


def test_whole_object_scalar_bands_and_passes(gpu):
    """Scalar whole objects in row bands (a band's first row receives the
    one-past-the-row store of the row above it) and mixed with per-triangle
    and AVX object passes in one frame."""
    s = scenes.with_ties(scenes.random_soup(3000, 256, 256, radius=24, seed=9, centroid_margin=30), seed=9)
    oc, oz, ow, _ = O.render(s, semantics=abi.PRK_SEM_SCALAR, phong=False, tris_per_object=7)
    for r0, r1 in [(0, 96), (96, 97), (97, 256)]:
        gc, gz, gw, _ = prk.render_scene(s, semantics=abi.PRK_SEM_SCALAR, phong=False, tris_per_object=7,
                                         rows=(r0, r1))
        compare((gc, gz, gw, None), (oc[r0:r1], oz[r0:r1], ow[r0:r1], None), label="band %d-%d" % (r0, r1))
    T = s.tri_count
    q = T // 4
    s.draws = [(0, q, None, abi.PRK_SEM_SCALAR, 5), (q, q, s.texture, abi.PRK_SEM_AVX, 4),
               (2 * q, q, None, abi.PRK_SEM_SCALAR, 1), (3 * q, T - 3 * q, s.texture, abi.PRK_SEM_SCALAR, 3)]
    run_both(s, phong=True, label="mixed scalar/AVX object passes")


def test_draw_caller_edge_list_scalar(gpu):
    """DrawModel on a ready edge_info list (prk_draw_edges, scalar)."""
    s = scenes.random_soup(60, 256, 256, radius=60, seed=44, textured=False, centroid_margin=40)
    words = O.fill_edge_table_words(s, 0, 60, phong=False)
    got = _render_src(s, "edges", words, abi.PRK_SEM_SCALAR, phong=False, textured=False)
    compare(got, O.render_edges(s, words, semantics=abi.PRK_SEM_SCALAR, phong=False), label="scalar edges")


def test_geometry_update_null_array_grows(gpu):
    """prk_geometry_update with a NULL colour array and a larger vertex count:
    the colour buffer grows (its old vertices kept, the new ones zero), so a
    scalar Gouraud draw of the new triangles reads inside its allocation and
    sees exactly those colours."""
    a = scenes.random_soup(800, 256, 256, radius=16, seed=51, textured=False)
    b = scenes.random_soup(3000, 256, 256, radius=16, seed=52, textured=False)
    expect = b.subset(0, b.tri_count)
    expect.colors = np.zeros_like(b.colors)
    expect.colors[: a.colors.shape[0]] = a.colors
    r = prk.Renderer()
    try:
        r.target_alloc(256, 256)
        r.clear()
        r.set_camera(b.prk_transform(), b.prk_lights())
        g = r.geometry(a.vertices, a.colors, a.normals, a.uvs)
        r.geometry_update(g, b.vertices, None, b.normals, b.uvs)
        r.draw_model(g, b.tri_count, P=b.P, phong=False)
        r.complete_all_work()
        r.synchronize()
        gc, gz = r.download()
    finally:
        r.close()
    oc, oz, _, _ = O.render(expect, semantics=abi.PRK_SEM_SCALAR, phong=False)
    assert (gz.view(np.uint32) == oz.view(np.uint32)).all()
    assert (gc == oc).all()


def test_geometry_write_chunks(gpu):
    """prk_geometry_write (the drop-in's chunked upload): a geometry created
    from the first 800 triangles gets the rest in two asynchronous writes of
    positions / normals / uvs (buffers growing, colours zero-extended), then
    a colour write for a scalar draw.  A write issued right after a flush
    waits for that frame's kernels: the frame still shows the old vertices."""
    b = scenes.random_soup(3000, 256, 256, radius=16, seed=53)
    old = scenes.random_soup(3000, 256, 256, radius=16, seed=54)
    old.texture = b.texture  # one texture handle serves both geometries
    r = prk.Renderer()
    try:
        r.target_alloc(256, 256)
        r.set_camera(b.prk_transform(), b.prk_lights())
        tex = r.texture(b.texture)
        g = r.geometry(old.vertices[:2400], old.colors[:2400], old.normals[:2400], old.uvs[:2400])
        r.geometry_write(g, 2400, old.vertices[2400:], None, old.normals[2400:], old.uvs[2400:])
        r.clear()
        r.draw_model_optimized(g, old.tri_count, bitmap=tex, P=old.P)
        r.complete_all_work()  # no wait: the next write is ordered after this frame's reads
        v, n, uv = b.vertices, b.normals, b.uvs
        # the asynchronous write reads page-locked host memory (prk.h)
        pinned = []
        for a in (v[:2400], n[:2400], uv[:2400]):
            p = ctypes.c_void_p()
            assert r._L.prk_host_alloc(r._h, a.nbytes, ctypes.byref(p)) == abi.PRK_OK
            h = np.frombuffer((ctypes.c_float * a.size).from_address(p.value), np.float32).reshape(a.shape)
            h[...] = a
            pinned.append(p)
        assert r._L.prk_geometry_write(r._h, g, 0, 2400, pinned[0], None, pinned[1], pinned[2]) == abi.PRK_OK
        c1, z1 = r.download()
        for p in pinned:
            r._L.prk_host_free(r._h, p)
        r.geometry_write(g, 2400, v[2400:5700], None, n[2400:5700], uv[2400:5700])
        r.geometry_write(g, 5700, v[5700:], None, n[5700:], uv[5700:])
        r.clear()
        r.draw_model_optimized(g, b.tri_count, bitmap=tex, P=b.P)
        r.complete_all_work()
        c2, z2 = r.download()
        r.geometry_write(g, 0, None, b.colors, None, None)
        r.clear()
        r.draw_model(g, b.tri_count, P=b.P, phong=False)
        r.complete_all_work()
        c3, z3 = r.download()
    finally:
        r.close()
    untex = b.subset(0, b.tri_count)
    untex.texture = None
    for f, ((gc, gz), (s, sem)) in enumerate((((c1, z1), (old, abi.PRK_SEM_AVX)), ((c2, z2), (b, abi.PRK_SEM_AVX)),
                                              ((c3, z3), (untex, abi.PRK_SEM_SCALAR)))):
        kw = {} if sem == abi.PRK_SEM_AVX else {"phong": False}
        oc, oz, _, _ = O.render(s, semantics=sem, **kw)
        assert (gz.view(np.uint32) == oz.view(np.uint32)).all(), "frame %d: z" % f
        assert (gc == oc).all(), "frame %d: colour (%d pixels)" % (f, (gc != oc).sum())


def test_unsupported_combinations(gpu):
    s = scenes.random_soup(10, 64, 64, seed=0)
    r = prk.Renderer()
    try:
        g = r.geometry(s.vertices, s.colors, s.normals, s.uvs)
        with pytest.raises(prk.PrkError) as e:
            r.draw_model_optimized(g, 10, bitmap=None)  # projekt.cpp:1506 needs a Bitmap
        assert e.value.code == abi.PRK_ERR_UNSUPPORTED
        tex = r.texture(s.texture)
        with pytest.raises(prk.PrkError) as e:
            r.draw_model_optimized(g, 10, bitmap=tex, phong=False)  # broken branch 2285-2316
        assert e.value.code == abi.PRK_ERR_UNSUPPORTED
        r.target_alloc(60, 64)  # AVX needs width % 8 == 0 (projekt.cpp:2218)
        r.set_camera(s.prk_transform(), s.prk_lights())
        r.draw_model_optimized(g, 10, bitmap=tex)
        with pytest.raises(prk.PrkError) as e:
            r.complete_all_work()
        assert e.value.code == abi.PRK_ERR_UNSUPPORTED
    finally:
        r.close()


def test_full_c3b_4096_1m(gpu):
    """The headline config (4096^2, 1M triangles, Phong + texture) against the
    oracle on the host cores: every pixel, bit for bit."""
    s = scenes.random_soup(1_000_000, 4096, 4096, radius=16, seed=2024)
    run_both(s, threads=16)


GOLDEN = sorted(__import__("glob").glob(__import__("os").path.join(
    __import__("os").path.dirname(__import__("os").path.abspath(__file__)), "golden", "*.npz")))


@pytest.mark.parametrize("path", GOLDEN, ids=[p.split("/")[-1] for p in GOLDEN])
def test_gpu_matches_golden_fixtures(gpu, path):
    """The GPU against the committed fixtures directly (no oracle build needed)."""
    import os
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
    from make_golden import load
    s, sem, phong, d = load(path)
    g = prk.render_scene(s, semantics=sem, phong=phong)
    compare(g, (d["color"], d["z"], d["winners"], None),
            label=os.path.basename(path))


def _dropin_scene(textured=True, salt=0):
    V, Cc, N, UV = prk.construct_sphere()
    tex = np.zeros((65, 64), np.uint32)
    y, x = np.mgrid[0:64, 0:64]
    tex[:64] = np.where(((x ^ y) & 8) != 0, 0xFFE0C080, 0xFF4060A0).astype(np.uint32) ^ np.uint32(salt * 0x00102030)
    return scenes.Scene(256, 256, V.copy(), Cc, N.copy(), UV, scenes.default_camera(256, 256), scenes.LIGHTS_ONE,
                        scenes.AMBIENT_ONE, scenes.Texture(tex, 64, 64) if textured else None, P=(0.0, 0.0, 2.0))


DROPIN_MODES = ["queue", "lines", "st", "scalar", "object", "mutate", "edges", "work", "scalar_object",
                "scalar_object_phong", "camera", "vertexlit", "interp", "interp_object", "split_st", "split_queue",
                "split_object", "records", "records_scalar", "records_queue"]


def _camera_b(s):
    """examples/dropin_demo.cpp's camera and lights B (the split modes)."""
    import copy
    b = copy.copy(s)
    b.transform = (4.5, 1.0, 128.0, 128.0 + 24.0, 128.0)
    b.lights = [((-1.0, 2.0, 2.5), (0.3, 0.9, 0.5, 1.0))]
    b.ambient = (0.1, 0.15, 0.3, 1.0)
    return b


@pytest.mark.parametrize("mode,bands", [(m, 1) for m in DROPIN_MODES] +
                         [("queue", 3), ("object", 2), ("mutate", 3), ("scalar", 3), ("work", 2),
                          ("scalar_object", 3), ("camera", 2), ("interp_object", 2), ("split_st", 2),
                          ("split_object", 2), ("records", 2)])
def test_dropin_demo_matches_oracle(gpu, tmp_path, mode, bands):
    """examples/dropin_demo.cpp drives the reference's own entry points
    through include/projekt.h (FillEdgeTable, DrawModelOptimized(RenderQueue),
    DrawModelOptimizedLines, the single-thread DrawModelOptimized, DrawModel,
    the three work-queue callbacks, a caller-built edge list, vertices and a
    texture rewritten in place between frames; its texture ends at an
    inaccessible page).  Its framebuffer must equal the oracle's.  bands > 1:
    the drop-in splits the frame into row bands, one context each
    (PRK_InitDevices; on a one-GPU box they share the GPU), every band
    downloaded into its rows of the caller's buffers."""
    import os
    import subprocess
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    exe = tmp_path / "dropin_demo"
    r = subprocess.run(["g++", "-std=c++17", "-O2", "-I", os.path.join(root, "include"),
                        os.path.join(root, "examples", "dropin_demo.cpp"), "-L",
                        os.path.join(root, "cpu-renderer_amd"), "-lprk_hip",
                        "-Wl,-rpath," + os.path.join(root, "cpu-renderer_amd"), "-o", str(exe)],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    scalar_modes = ("scalar", "scalar_object", "scalar_object_phong", "vertexlit", "interp", "interp_object",
                    "split_object", "records_scalar")
    s = _dropin_scene(textured=mode not in scalar_modes)
    # FillEdgeTable's own PhongShading / Object->Bitmap (the demo's objects
    # carry the Bitmap except in "vertexlit")
    setup = {"scalar": abi.PRK_SETUP_BITMAP, "vertexlit": 0, "interp": abi.PRK_SETUP_PHONG | abi.PRK_SETUP_BITMAP,
             "scalar_object": abi.PRK_SETUP_BITMAP, "interp_object": abi.PRK_SETUP_PHONG | abi.PRK_SETUP_BITMAP,
             "scalar_object_phong": abi.PRK_SETUP_PHONG | abi.PRK_SETUP_BITMAP,
             "records": abi.PRK_SETUP_PHONG | abi.PRK_SETUP_BITMAP, "records_scalar": abi.PRK_SETUP_BITMAP}.get(mode)
    T = s.tri_count
    extra = []
    if mode == "edges":
        words = O.fill_edge_table_words(s, 0, T)
        words.tofile(tmp_path / "edges.u32")
        extra = [str(tmp_path / "edges.u32")]
    if mode == "work":
        rng = np.random.default_rng(2)
        n = 400
        w = np.zeros((n, 25), np.uint32)
        f = w.view(np.float32)
        x0 = rng.uniform(-20, 250, n)
        for k, x in ((0, x0), (12, x0 + rng.uniform(0, 60, n))):
            zc = rng.uniform(-1, 1, n)
            f[:, k] = x
            f[:, k + 1] = zc
            f[:, k + 2] = 1.0 / (4.0 - zc)
            f[:, k + 3] = rng.uniform(0, 1, n) * f[:, k + 2]
            f[:, k + 4] = rng.uniform(0, 1, n) * f[:, k + 2]
            f[:, k + 5:k + 9] = rng.uniform(0, 1, (n, 4))
            nv = rng.normal(size=(n, 3))
            f[:, k + 9:k + 12] = nv / np.linalg.norm(nv, axis=1, keepdims=True)
        w[:, 24] = np.sort(rng.integers(0, 256, n)).astype(np.uint32)
        w.tofile(tmp_path / "spans.u32")
        extra = [str(tmp_path / "spans.u32")]
    if mode in ("records", "records_scalar"):
        extra = [str(tmp_path / "rec")]
    args = [str(exe), str(tmp_path / "c.u32"), str(tmp_path / "z.f32"), mode] + extra
    env = dict(os.environ, PRK_DEMO_BANDS=str(bands))
    run = subprocess.run(args, capture_output=True, text=True, timeout=120, env=env)
    assert run.returncode == 0, run.stderr
    gc = np.fromfile(tmp_path / "c.u32", np.uint32).reshape(256, 256)
    gz = np.fromfile(tmp_path / "z.f32", np.float32).reshape(256, 256)
    if mode in ("records", "records_scalar"):
        # record mode: EdgeMemory holds the reference's records after
        # FillEdgeTable (3894-4117) and after the draw's walk (3654-3869)
        def dump(ext):
            d = np.fromfile(str(tmp_path / "rec") + ext, np.uint32).reshape(-1, 28)
            return d[:, :27], d[:, 27].view(np.int32)
        fw, fn = dump(".fill")
        ow = O.fill_edge_table_words(s, 0, T, setup=setup)
        assert fw.shape == ow.shape and np.array_equal(fw, ow), (mode, fw.shape, ow.shape)
        assert (fn == -1).all()
        aw, an = dump(".adv")
        oaw, oan = O.advance_edges(ow, 256)
        assert np.array_equal(aw, oaw) and np.array_equal(an, oan), mode
        assert not np.array_equal(aw, fw)
    if mode in ("queue", "lines", "records_queue"):
        oc, oz, _, _ = O.render(s)
    elif mode == "st":
        oc, oz, _, _ = O.render(s, semantics=abi.PRK_SEM_AVX_ST)
    elif mode in ("scalar", "vertexlit", "interp"):
        oc, oz, _, _ = O.render(s, semantics=abi.PRK_SEM_SCALAR, phong=False, setup=setup)
    elif mode in ("object", "records"):
        oc, oz, _, _ = O.render(s, tris_per_object=T)
    elif mode in ("scalar_object", "scalar_object_phong", "interp_object", "records_scalar"):
        oc, oz, _, _ = O.render(s, semantics=abi.PRK_SEM_SCALAR, phong=mode.endswith("phong"), tris_per_object=T,
                                setup=setup)
    elif mode == "camera":  # the second half drawn with the moved camera and the new light, over the first
        half = T // 2
        a, b = s.subset(0, half), s.subset(half, T)
        b.transform = (4.0, 1.0, 128.0, 128.0 + 24.0, 128.0)
        b.lights = [((1.0, 1.0, 3.0), (0.3, 0.9, 0.5, 1.0))]
        oc, oz, _, _ = O.render(a)
        oc, oz, _, _ = O.render(b, color=oc, z=oz)
    elif mode in ("split_st", "split_queue"):  # set up under A, shaded under B (the draw call's Commands)
        sem = abi.PRK_SEM_AVX_ST if mode == "split_st" else abi.PRK_SEM_AVX
        oc, oz, _, _ = O.render(_camera_b(s), semantics=sem, setup_camera=s)
        a_only = O.render(s, semantics=sem)[0]
        assert (oc != a_only).any()  # the shading camera matters
    elif mode == "split_object":
        oc, oz, _, _ = O.render(_camera_b(s), semantics=abi.PRK_SEM_SCALAR, phong=True, tris_per_object=T,
                                setup=abi.PRK_SETUP_PHONG | abi.PRK_SETUP_BITMAP, setup_camera=s)
    elif mode == "mutate":
        m = _dropin_scene(salt=1)
        m.vertices[:, 0] = m.vertices[:, 0] * np.float32(0.75) + np.float32(0.125)
        m.vertices[:, 1] = m.vertices[:, 1] * np.float32(1.25) - np.float32(0.0625)
        m.normals[:, 2] = -m.normals[:, 2]
        oc, oz, _, _ = O.render(m)
    elif mode == "edges":
        oc, oz, _, _ = O.render_edges(s, words)
    else:  # work
        oc, oz, _, _ = O.render_spans(s, w[: n // 2])
        oc, oz, _, _ = O.render_spans(s, w[n // 2:], color=oc, z=oz)
        oc, oz, _, _ = O.render(s, semantics=abi.PRK_SEM_AVX_ST, tris_per_object=T, color=oc, z=oz)
    cd = channel_diff(gc, oc)
    assert (gz.view(np.uint32) == oz.view(np.uint32)).all(), mode
    assert (gc == oc).all(), (mode, int((cd > 0).sum()))
    assert (gz > -3e38).sum() > 2000
    # FillEdgeTable's return values (projekt.cpp:4119) summed over the frame's
    # calls equal the oracle's edge counts: per triangle, or the whole sphere
    edges = int(run.stdout.split("edges=")[1].split()[0])
    if mode in ("queue", "lines", "st", "scalar", "camera", "vertexlit", "interp", "split_st", "split_queue",
                "records_queue"):
        assert edges == sum(len(O.fill_edge_table(s, t, 1)) for t in range(T)), mode
    elif mode in ("records", "records_scalar"):
        assert edges == len(ow), mode
    elif mode.startswith("scalar_object") or mode == "interp_object":
        assert edges == len(O.fill_edge_table(s, 0, T, phong=mode.endswith("phong"))), mode


@pytest.mark.parametrize("semantics,phong,textured", [(abi.PRK_SEM_SCALAR, False, False),
                                                       (abi.PRK_SEM_SCALAR, True, True),
                                                       (abi.PRK_SEM_AVX, True, True)])
def test_sliver_x_ties(gpu, semantics, phong, textured):
    # Two top edges tied in X on every row: the order entering each tile comes
    # from history, which the fast replay must hand to the
    # X-only row-by-row replay.
    s = scenes.slivers(3000, 2048, 256, seed=4, textured=textured)
    g, o = run_both(s, semantics=semantics, phong=phong)
    assert (g[2] >= 0).sum() > 10000
    assert g[3]["slow_replays"] > 0 and g[3]["anomalies"] == 0


# ---- BASELINE configs as parity cases ----------------------

def test_c2_bunny_standin_1080p(gpu):
    """C2: ~70k-triangle closed displaced sphere (bunny stand-in), 1920x1080,
    untextured Phong -> scalar DrawModel semantics."""
    s = scenes.displaced_sphere(70000, 1920, 1080, seed=3)
    g, o = run_both(s, semantics=abi.PRK_SEM_SCALAR, phong=True, threads=16)
    assert (g[2] >= 0).sum() > 100000


def test_c3a_gouraud_4096_1m(gpu):
    """C3a: 1M triangles at 4096^2, colour interpolation only (scalar Gouraud)."""
    s = scenes.random_soup(1_000_000, 4096, 4096, radius=16, seed=2025, textured=False)
    run_both(s, semantics=abi.PRK_SEM_SCALAR, phong=False, threads=16)


@pytest.mark.parametrize("filt", [abi.PRK_FILTER_NEAREST, abi.PRK_FILTER_BILINEAR])
def test_c4_sponza_like_4k(gpu, filt):
    """C4: Sponza-style atrium (~250k triangles, 8 material draws of 1024^2
    textures) at 3840x2160, Phong; nearest = the reference's sampling,
    bilinear = the build's extension (defined by the oracle's restatement)."""
    s = scenes.sponza_like(3840, 2160, seed=1, filt=filt)
    g, o = run_both(s, threads=16)
    assert (g[2] >= 0).mean() > 0.95


def test_bilinear_soups_mixed_filters(gpu):
    """Bilinear and nearest textures in one frame (multi-draw, mixed samplers)."""
    s = scenes.random_soup(6000, 512, 384, radius=24, seed=11, tex_size=64)
    t2 = scenes.Texture(s.texture.texels.copy(), 64, 64, abi.PRK_FILTER_BILINEAR)
    s.draws = [(0, 3000, s.texture), (3000, 3000, t2)]
    run_both(s)


def test_c5_8192_two_bands(gpu):
    """C5 geometry (1M triangles, offsets +-32 px, 8192^2) rendered as two row
    bands (what two ranks draw before the gather) equals the full-frame oracle."""
    s = scenes.random_soup(1_000_000, 8192, 8192, radius=32, seed=5)
    oc, oz, ow, _ = O.render(s, threads=16)
    for r0, r1 in ((0, 4096), (4096, 8192)):
        gc, gz, gw, _ = prk.render_scene(s, rows=(r0, r1))
        compare((gc, gz, gw, None), (oc[r0:r1], oz[r0:r1], ow[r0:r1], None), label="band %d-%d" % (r0, r1))
    # the same band drawn twice by one context: its first frame (5.6 bin
    # entries a triangle at 256x8) switches it to the automatic 512x8 tile,
    # which the second frame draws with
    r0, r1 = 4096, 8192
    r = prk.Renderer(0)
    try:
        r.target_alloc(s.width, s.height, r0, r1)
        r.set_debug(True)
        r.set_camera(s.prk_transform(), s.prk_lights())
        g = r.geometry(s.vertices, s.colors, s.normals, s.uvs)
        tex = r.texture(s.texture)
        ent = []
        for _ in range(2):
            r.clear()
            r.draw_model_optimized(g, s.tri_count, P=s.P, bitmap=tex, phong=True)
            r.complete_all_work()
            r.synchronize()
            ent.append(r.stats()["bin_entries"])
        gc, gz = r.download()
        gw = r.winners()
    finally:
        r.close()
    assert ent[1] < ent[0], ent  # (512x8 tiles: fewer entries)
    compare((gc, gz, gw, None), (oc[r0:r1], oz[r0:r1], ow[r0:r1], None), label="band %d-%d at 512x8" % (r0, r1))


EXIT_CHILD = r"""
import sys
sys.path[:0] = [{pkg!r}]
import numpy as np
import torch
import prk
from prk import scenes
small = scenes.random_soup(3000, 512, 384, radius=16, seed=91)
big = scenes.random_soup(6000, 512, 384, radius=260, seed=92)
big.texture = small.texture
W, H = 512, 384
color = torch.zeros((H, W), dtype=torch.int32, device="cuda")
z = torch.zeros((H, W), dtype=torch.float32, device="cuda")
r = prk.Renderer(0)
r.set_camera(small.prk_transform(), small.prk_lights())
tex = r.texture(small.texture)
gs = [r.geometry(s.vertices, s.colors, s.normals, s.uvs) for s in (small, big)]
r.target_bind(color.data_ptr(), W * 4, z.data_ptr(), W, H)
r.clear_on_flush()
r.draw_model_optimized(gs[0], small.tri_count, P=small.P, bitmap=tex)
r.complete_all_work()          # counted at once: sizes the scratch
r.clear_on_flush()
r.draw_model_optimized(gs[1], big.tri_count, P=big.P, bitmap=tex)
r.complete_all_work()          # over capacity, its count never read
print("queued; exiting without close", flush=True)
{tail}
"""


@pytest.mark.parametrize("tail", ["", "del color, z", "import gc; r2 = r; del r; gc.collect()"])
def test_exit_with_pending_overflowed_frame(gpu, tmp_path, tail):
    """A process that queues an over-capacity frame into a torch-owned target
    and exits without close(): interpreter teardown must not run GPU work or
    free anything twice (prk_destroy never queues GPU work; the binding
    closes open contexts at exit before torch and the HIP runtime go away).
    Exit status 0, no glibc heap message."""
    import os
    import subprocess
    import sys
    pkg = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "cpu-renderer_amd")
    script = tmp_path / "child.py"
    script.write_text(EXIT_CHILD.format(pkg=pkg, tail=tail))
    run = subprocess.run([sys.executable, str(script)], capture_output=True, text=True, timeout=100)
    bad = [w for w in ("double free", "corruption", "Aborted", "Segmentation", "free():") if w in run.stderr]
    assert run.returncode == 0 and not bad, (run.returncode, run.stderr[-2000:])
    assert "exiting without close" in run.stdout
