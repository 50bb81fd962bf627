"""CPU tests: the edge_info records the drop-in's record mode leaves in the
caller's memory (prk_fill_edge_records / prk_advance_edge_records, host code
of libprk_hip.so) against the oracle's FillEdgeTable (projekt.cpp:3894-4117)
and its AET walk (3654-3869), word for word, list pointers included.

Parity is against the restatement (oracle/prk_oracle.c): UNPINNED, DESIGN.md §3.
"""
import numpy as np
import pytest

import oracle as O
import prk
from prk import abi, scenes


def _sphere(P=(0.0, 0.0, 2.0), lights=None, ambient=None):
    V, Cc, N, UV = prk.construct_sphere()
    base = scenes.random_soup(1, 256, 256, seed=0)
    return scenes.Scene(256, 256, V.copy(), Cc.copy(), N.copy(), UV.copy(), base.transform,
                        lights or scenes.LIGHTS_ONE, ambient or scenes.AMBIENT_ONE, base.texture, P=P)


def _cases():
    yield "sphere", _sphere()
    yield "sphere_near", _sphere(P=(0.0, 0.0, 3.6))  # through the near plane (74-93)
    yield "soup_clip", scenes.random_soup(400, 192, 160, radius=90, seed=3, centroid_margin=60)
    yield "soup_two_lights", scenes.random_soup(300, 256, 256, radius=20, seed=4, lights=scenes.LIGHTS_TWO,
                                                ambient=scenes.AMBIENT_TWO)
    yield "soup_no_light", scenes.random_soup(300, 256, 256, radius=20, seed=5, lights=[])


def _fill(s, setup):
    return prk.fill_edge_records(s.vertices, s.colors, s.normals, s.uvs, s.P, s.prk_transform(), s.prk_lights(),
                                 setup)


@pytest.mark.parametrize("setup", [0, abi.PRK_SETUP_PHONG, abi.PRK_SETUP_BITMAP,
                                   abi.PRK_SETUP_PHONG | abi.PRK_SETUP_BITMAP])
@pytest.mark.parametrize("name,scene", list(_cases()))
def test_fill_edge_records_match_oracle(name, scene, setup):
    mem, n = _fill(scene, setup)
    words, nxt = prk.edge_record_words(mem, n)
    ow = O.fill_edge_table_words(scene, 0, scene.tri_count, setup=setup)
    assert n == ow.shape[0] > 0, (name, n, ow.shape)
    bad = np.nonzero((words != ow).any(1))[0]
    assert bad.size == 0, (name, setup, int(bad.size), bad[:5])
    assert (nxt == -1).all()  # 4094: Next = 0, MergeSort moves whole records
    # FillEdgeTable's return value is the library's host count too (4119)
    assert n == prk.fill_edge_count(scene.vertices, scene.P, scene.prk_transform())


@pytest.mark.parametrize("height_frac", [1.0, 0.5])
@pytest.mark.parametrize("name,scene", list(_cases()))
def test_advance_edge_records_match_oracle(name, scene, height_frac):
    setup = abi.PRK_SETUP_PHONG | abi.PRK_SETUP_BITMAP
    H = int(scene.height * height_frac)
    mem, n = _fill(scene, setup)
    w0, _ = prk.edge_record_words(mem, n)
    prk.advance_edge_records(mem, n, H)
    words, nxt = prk.edge_record_words(mem, n)
    ow, onxt = O.advance_edges(w0, H)
    assert (w0 != words).any()  # the walk did step edges
    bad = np.nonzero((words != ow).any(1))[0]
    assert bad.size == 0, (name, H, int(bad.size), bad[:5])
    assert np.array_equal(nxt, onxt), (name, H)


def test_fill_edge_records_in_place():
    """Fields the reference never writes keep the caller's bytes (a Gouraud
    edge's normal, an untextured edge's UV gradients, 4012-4089), and the
    arithmetic that reads them reads those bytes (NormalGradient = (0 -
    MinNormal) / YDiff); with zeroed memory that is the oracle's pin."""
    s = scenes.random_soup(200, 256, 256, radius=20, seed=9)
    mem = np.zeros((3 * s.tri_count, prk.EDGE_INFO_STRIDE), np.uint8)
    f = mem[:, :108].view(np.float32)
    f[:, 21:24] = 0.5  # stale MinNormal
    mem2, n = prk.fill_edge_records(s.vertices, s.colors, s.normals, s.uvs, s.P, s.prk_transform(),
                                    s.prk_lights(), 0, memory=mem)
    w, _ = prk.edge_record_words(mem2, n)
    wf = w.view(np.float32)
    assert (wf[:, 21:24] == 0.5).all()
    ydiff = (w.view(np.int32)[:, 0:1] - w.view(np.int32)[:, 7:8]).astype(np.float32)
    with np.errstate(divide="ignore"):
        assert np.array_equal(wf[:, 24:27], np.broadcast_to(np.float32(-0.5) / ydiff, (n, 3)))
    assert (wf[:, 10:12] == 0.0).all()  # no Bitmap: no UV gradients written


def test_edge_records_argument_checks():
    import ctypes as C
    L = prk.lib()
    n = C.c_uint32(0)
    t = scenes.random_soup(1, 64, 64).prk_transform()
    li = scenes.random_soup(1, 64, 64).prk_lights()
    buf = np.zeros((3, 120), np.uint8)
    v = np.zeros((3, 3), np.float32)
    # stride too small / Next overlapping the fields / no output count
    assert L.prk_fill_edge_records(v.ctypes.data, None, None, None, 3, None, C.byref(t), C.byref(li), 0,
                                   buf.ctypes.data, 100, 112, None, C.byref(n)) == abi.PRK_ERR_ARG
    assert L.prk_fill_edge_records(v.ctypes.data, None, None, None, 3, None, C.byref(t), C.byref(li), 0,
                                   buf.ctypes.data, 120, 100, None, C.byref(n)) == abi.PRK_ERR_ARG
    assert L.prk_fill_edge_records(v.ctypes.data, None, None, None, 3, None, C.byref(t), C.byref(li), 0,
                                   buf.ctypes.data, 120, 112, None, None) == abi.PRK_ERR_ARG
    assert L.prk_advance_edge_records(buf.ctypes.data, 0, 120, 112, 64) == abi.PRK_OK  # P1: no edges
    assert L.prk_advance_edge_records(buf.ctypes.data, 1, 120, 116, 64) == abi.PRK_ERR_ARG
