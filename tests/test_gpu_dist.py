"""GPU: the C-ABI's multi-GPU path on one MI355X.

Row bands rendered by separate contexts and gathered into one device frame
must equal the single-context frame bit for bit:
  * prk_gather_frame_local (peer copies; here every band's context shares
    device 0, on a node each band is its own GPU),
  * prk_gather_frame / prk_gather_frame_all over RCCL with one rank (a one-GPU
    box cannot host two RCCL ranks: RCCL rejects two ranks on one device), so
    the communicator set-up, the group and rank 0's own-band copy run; the
    peer sends and receives run only on the 8-GPU node.
"""
import numpy as np
import pytest

import prk
from prk import abi, scenes

pytestmark = pytest.mark.gpu


def _band_renderers(s, n, devices=None):
    rs = []
    for r in range(n):
        R = prk.Renderer(0 if devices is None else devices[r])
        a, b = prk.band_rows(s.height, r, n)
        R.target_alloc(s.width, s.height, a, b)
        R.clear_on_flush()
        R.set_camera(s.prk_transform(), s.prk_lights())
        g = R.geometry(s.vertices, s.colors, s.normals, s.uvs)
        t = R.texture(s.texture)
        R.draw_model_optimized(g, s.tri_count, bitmap=t)
        R.complete_all_work()
        rs.append(R)
    return rs


def _frame(s):
    F = prk.Renderer(0)
    F.target_alloc(s.width, s.height)
    return F


@pytest.fixture(scope="module")
def scene_ref():
    s = scenes.random_soup(20000, 512, 384, radius=24, seed=41)
    col, z, _, _ = prk.render_scene(s, debug=False, fused_clear=True)
    return s, col, z


@pytest.mark.parametrize("n", [2, 3, 5])
def test_gather_frame_local(gpu, scene_ref, n):
    s, col, z = scene_ref
    rs = _band_renderers(s, n)
    F = _frame(s)
    cp, pitch, zp, *_ = F.target()
    prk.gather_frame_local(rs, cp, pitch, zp, with_z=True)
    rs[0].synchronize()
    gc, gz = F.download()
    assert (gc == col).all() and (gz.view(np.uint32) == z.view(np.uint32)).all()
    for R in rs + [F]:
        R.close()


def test_gather_frame_rccl_one_rank(gpu, scene_ref):
    if not prk.comm_available():
        pytest.fail("librccl did not load")
    s, col, z = scene_ref
    (R,) = _band_renderers(s, 1)
    F = _frame(s)
    cp, _, zp, *_ = F.target()
    c = prk.Comm.init(R, prk.comm_unique_id(), 1, 0)
    c.gather(R, cp, zp, with_z=True)
    R.synchronize()
    gc, gz = F.download()
    assert (gc == col).all() and (gz.view(np.uint32) == z.view(np.uint32)).all()
    c.close()
    # the single-process group form (ncclCommInitAll)
    (c1,) = prk.Comm.init_all([R])
    F2 = _frame(s)
    cp2, _, zp2, *_ = F2.target()
    prk.gather_frame_all([R], [c1], cp2, zp2, with_z=True)
    R.synchronize()
    gc2, gz2 = F2.download()
    assert (gc2 == col).all() and (gz2.view(np.uint32) == z.view(np.uint32)).all()
    c1.close()
    for x in (R, F, F2):
        x.close()


def test_c5_8192_eight_bands_gather(gpu):
    """C5 (1M triangles, offsets +-32 px, 8192^2) split as the 8-rank run
    splits it: 8 band contexts (prk_band_rows), each binning every triangle
    against its 1024 rows, gathered with prk_gather_frame_local into one
    device frame.  The gathered colour and z and every band's winner map equal
    the full-frame oracle bit for bit."""
    import oracle as O
    s = scenes.random_soup(1_000_000, 8192, 8192, radius=32, seed=5)
    oc, oz, ow, _ = O.render(s, threads=16)
    n = 8
    rs = []
    wins = []
    try:
        for r in range(n):
            R = prk.Renderer(0)
            rs.append(R)
            a, b = prk.band_rows(s.height, r, n)
            assert (a, b) == (r * 1024, (r + 1) * 1024)
            R.target_alloc(s.width, s.height, a, b)
            R.clear_on_flush()
            R.set_debug(True)
            R.set_camera(s.prk_transform(), s.prk_lights())
            g = R.geometry(s.vertices, None, s.normals, s.uvs)
            t = R.texture(s.texture)
            R.draw_model_optimized(g, s.tri_count, bitmap=t)
            R.complete_all_work()
        for R in rs:
            R.synchronize()
            wins.append(R.winners())
        F = _frame(s)
        rs.append(F)
        cp, pitch, zp, *_ = F.target()
        prk.gather_frame_local(rs[:n], cp, pitch, zp, with_z=True)
        rs[0].synchronize()
        gc, gz = F.download()
    finally:
        for R in rs:
            R.close()
    zbad = int((gz.view(np.uint32) != oz.view(np.uint32)).sum())
    cbad = int((gc != oc).sum())
    wbad = sum(int((w != ow[r * 1024:(r + 1) * 1024]).sum()) for r, w in enumerate(wins))
    assert zbad == 0 and cbad == 0 and wbad == 0, (zbad, cbad, wbad)
    assert (ow >= 0).mean() > 0.8


def test_gather_rejects_wrong_band(gpu, scene_ref):
    s, _, _ = scene_ref
    rs = _band_renderers(s, 2)
    F = _frame(s)
    cp, pitch, zp, *_ = F.target()
    with pytest.raises(prk.PrkError):  # bands in the wrong order
        prk.gather_frame_local([rs[1], rs[0]], cp, pitch, zp, with_z=True)
    with pytest.raises(prk.PrkError):  # z asked for, no z frame
        prk.gather_frame_local(rs, cp, pitch, None, with_z=True)
    for R in rs + [F]:
        R.close()


def test_gather_after_overflowed_frame_on_explicit_stream(gpu):
    """prk_gather_frame right after a frame whose bin entries overflowed the
    scratch, on a caller stream (torch): the gather resolves the count first,
    so the re-run lands in the band before it is sent, and the caller stream
    waits for it — the gathered frame is the finished frame (no host sync
    between the flush and the gather)."""
    import torch

    import oracle as O
    if not prk.comm_available():
        pytest.fail("librccl did not load")
    small = scenes.random_soup(3000, 512, 384, radius=16, seed=91)
    big = scenes.random_soup(6000, 512, 384, radius=260, seed=92)
    big.texture = small.texture
    (R,) = _band_renderers(small, 1)  # first frame: counted at once (sizes the scratch)
    F = _frame(big)
    cp, _, zp, *_ = F.target()
    c = prk.Comm.init(R, prk.comm_unique_id(), 1, 0)
    try:
        g = R.geometry(big.vertices, big.colors, big.normals, big.uvs)
        t = R.texture(big.texture)
        R.clear_on_flush()
        R.draw_model_optimized(g, big.tri_count, P=big.P, bitmap=t)
        R.complete_all_work()  # over capacity: its count is read by the gather
        side = torch.cuda.Stream(device=torch.device("cuda:0"))
        c.gather(R, cp, zp, with_z=True, stream=side.cuda_stream)
        side.synchronize()
        gc, gz = F.download()
        entries = R.stats()["bin_entries"]
    finally:
        c.close()
        R.close()
        F.close()
    oc, oz, _, _ = O.render(big)
    assert entries > 0
    assert (gz.view(np.uint32) == oz.view(np.uint32)).all(), "z"
    assert (gc == oc).all(), "colour"
