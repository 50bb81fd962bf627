"""ctypes loader for liboracle.so — TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import
this module, and only as the checker / the timed CPU baseline.  The product
path (cpu-renderer_amd/prk, libprk_hip.so) never imports it.

PARITY UNPINNED: see the header of oracle/prk_oracle.c and DESIGN.md §3.
"""
import ctypes as C
import os
import subprocess
import sys

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
# PRK_ORACLE_LIBDIR: load the libraries from another directory (the
# sanitizer builds of `make -C oracle san`, tests/test_sanitizers.py).
_LIBDIR = os.environ.get("PRK_ORACLE_LIBDIR") or _HERE


def _libpath(name):
    p = os.path.join(_LIBDIR, name)
    return p if os.path.exists(p) else os.path.join(_HERE, name)
sys.path.insert(0, os.path.join(os.path.dirname(_HERE), "cpu-renderer_amd"))
from prk import abi  # noqa: E402
from prk.scenes import CLEAR_COLOR, CLEAR_Z  # noqa: E402

_LIB = None
_CPU = None


class OrDrawDesc(C.Structure):
    _fields_ = [("Vertices", C.c_void_p), ("Colors", C.c_void_p), ("Normals", C.c_void_p),
                ("UVs", C.c_void_p), ("TriCount", C.c_uint32), ("TrisPerObject", C.c_uint32),
                ("P", C.c_float * 3), ("Semantics", C.c_int32), ("Phong", C.c_int32),
                ("Bitmap", C.POINTER(abi.PrkBitmap)), ("TriIndexBase", C.c_int32), ("Filter", C.c_int32),
                ("Setup", C.c_int32), ("SetupT", C.c_void_p), ("SetupLights", C.c_void_p)]


class OrTarget(C.Structure):
    _fields_ = [("Color", C.c_void_p), ("Pitch", C.c_int32), ("Z", C.c_void_p),
                ("Width", C.c_int32), ("Height", C.c_int32), ("Winners", C.c_void_p)]


def build():
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


def lib():
    global _LIB
    if _LIB is None:
        path = _libpath("liboracle.so")
        if not os.path.exists(path):
            build()
        _LIB = C.CDLL(path)
        for fn in ("oracle_draw", "oracle_draw_band", "oracle_draw_mt",
                   "oracle_fill_edge_table", "oracle_draw_edges", "oracle_draw_spans"):
            getattr(_LIB, fn).restype = C.c_int
    return _LIB


def cpu_lib():
    """liborcpu.so: the AVX2 CPU baseline (prk_cpu_avx.c), or None when the
    host has no AVX2."""
    global _CPU
    if _CPU is None:
        path = _libpath("liborcpu.so")
        if not os.path.exists(path):
            build()
        _CPU = C.CDLL(path)
        for fn in ("cpu_avx_draw", "cpu_avx_draw_banded", "cpu_avx_draw_queue", "cpu_avx_draw_rows",
                   "cpu_avx_supported"):
            getattr(_CPU, fn).restype = C.c_int
    return _CPU if _CPU.cpu_avx_supported() else None


def _ptr(a):
    return None if a is None else a.ctypes.data_as(C.c_void_p)


class _Keep:
    """Holds ctypes objects alive for the duration of a call."""

    def __init__(self, scene, semantics, phong, tris_per_object, tri_base=0, texture="scene", setup=None,
                 setup_camera=None):
        self.arrays = [np.ascontiguousarray(scene.vertices, np.float32),
                       np.ascontiguousarray(scene.colors, np.float32),
                       np.ascontiguousarray(scene.normals, np.float32),
                       np.ascontiguousarray(scene.uvs, np.float32)]
        self.bitmap = None
        texture = scene.texture if texture == "scene" else texture
        if texture is not None:
            self.tex = np.ascontiguousarray(texture.texels)
            self.bitmap = abi.PrkBitmap(self.tex.ctypes.data_as(C.c_void_p).value,
                                        texture.width, texture.height, texture.pitch)
        d = OrDrawDesc()
        d.Vertices, d.Colors, d.Normals, d.UVs = [_ptr(a) for a in self.arrays]
        d.TriCount = scene.tri_count
        d.TrisPerObject = tris_per_object
        for i in range(3):
            d.P[i] = scene.P[i]
        d.Semantics = semantics
        d.Phong = int(bool(phong))
        d.Bitmap = C.pointer(self.bitmap) if self.bitmap is not None else None
        d.TriIndexBase = tri_base
        d.Filter = getattr(texture, "filter", abi.PRK_FILTER_NEAREST) if texture is not None else 0
        d.Setup = -1 if setup is None else int(setup)  # FillEdgeTable's own inputs (PRK_SETUP_*)
        self.transform = scene.prk_transform()
        self.lights = scene.prk_lights()
        if setup_camera is not None:  # FillEdgeTable's camera / lights (a scene), the draw's shade
            self.setup_transform = setup_camera.prk_transform()
            self.setup_lights = setup_camera.prk_lights()
            d.SetupT = C.cast(C.pointer(self.setup_transform), C.c_void_p)
            d.SetupLights = C.cast(C.pointer(self.setup_lights), C.c_void_p)
        self.desc = d


def render(scene, semantics=abi.PRK_SEM_AVX, phong=True, tris_per_object=1, threads=1,
           color=None, z=None, winners=True, rows=None, cpu=None, setup=None, setup_camera=None):
    """Draw `scene` with the oracle.  Returns (color u32[H,W], z f32[H,W],
    winners i32[H,W] or None, stats dict).  `color`/`z` (optional) are the
    prior target contents (default: reference clear values).
    cpu: None = the scalar restatement (liboracle.so); "banded" / "queue" /
    "rows" = the AVX2 CPU baseline (liborcpu.so) with that schedule over
    `threads`.  setup: FillEdgeTable's own PhongShading / Object->Bitmap
    (PRK_SETUP_* bits; None: as the draw).  setup_camera: a scene whose
    transform / lights FillEdgeTable saw (the caller changed Commands before
    DrawModel*); `scene`'s own shade the spans.  None: `scene`'s for both."""
    W, H = scene.width, scene.height
    col = np.full((H, W), CLEAR_COLOR, np.uint32) if color is None else np.array(color, np.uint32)
    zb = np.full((H, W), CLEAR_Z, np.float32) if z is None else np.array(z, np.float32)
    win = np.full((H, W), -1, np.int32) if winners else None
    if scene.draws is not None:  # multi-draw scene: the draws in order, one target
        from prk.scenes import draw_spec
        tot = [0, 0, 0]
        for d in scene.draws:
            first, count, texture, sem, tpo = draw_spec(d, semantics, tris_per_object)
            sub = scene.subset(first, first + count)
            sub.texture, sub.draws = texture, None
            _, _, _, st = _render_one(sub, sem, phong, tpo, threads, col, zb, win, rows,
                                      tri_base=first, cpu=cpu, setup=setup, setup_camera=setup_camera)
            tot = [tot[0] + st["spans"], tot[1] + st["span_pixels"], tot[2] + st["writes"]]
        return col, zb, win, dict(spans=tot[0], span_pixels=tot[1], writes=tot[2])
    return _render_one(scene, semantics, phong, tris_per_object, threads, col, zb, win, rows, cpu=cpu, setup=setup,
                       setup_camera=setup_camera)


def _render_one(scene, semantics, phong, tris_per_object, threads, col, zb, win, rows, tri_base=0, cpu=None,
                setup=None, setup_camera=None):
    W, H = scene.width, scene.height
    k = _Keep(scene, semantics, phong, tris_per_object, tri_base=tri_base, setup=setup, setup_camera=setup_camera)
    tg = OrTarget(_ptr(col), W * 4, _ptr(zb), W, H, _ptr(win))
    stats = (C.c_uint64 * 3)()
    if cpu is not None:
        L = cpu_lib()
        if L is None:
            raise RuntimeError("AVX2 CPU baseline: host has no AVX2")
        fn = {"banded": L.cpu_avx_draw_banded, "queue": L.cpu_avx_draw_queue, "rows": L.cpu_avx_draw_rows}[cpu]
        rc = fn(C.byref(k.desc), C.byref(tg), C.byref(k.transform), C.byref(k.lights), int(threads), stats)
        if rc != 0:
            raise RuntimeError("cpu baseline failed: %s" % abi.STATUS_NAMES.get(rc, rc))
        return col, zb, win, dict(spans=stats[0], span_pixels=stats[1], writes=stats[2])
    L = lib()
    if rows is not None:
        rc = L.oracle_draw_band(C.byref(k.desc), C.byref(tg), C.byref(k.transform),
                                C.byref(k.lights), int(rows[0]), int(rows[1]), stats)
    elif threads > 1:
        rc = L.oracle_draw_mt(C.byref(k.desc), C.byref(tg), C.byref(k.transform),
                              C.byref(k.lights), int(threads), stats)
    else:
        rc = L.oracle_draw(C.byref(k.desc), C.byref(tg), C.byref(k.transform),
                           C.byref(k.lights), stats)
    if rc != 0:
        raise RuntimeError("oracle failed: %s" % abi.STATUS_NAMES.get(rc, rc))
    return col, zb, win, dict(spans=stats[0], span_pixels=stats[1], writes=stats[2])


EDGE_FIELDS = ["YMax", "XMin", "ZMin", "OneOverZMin", "Gradient", "ZGradient",
               "OneOverZGradient", "YMin", "UMin", "VMin", "UGradient", "VGradient", "Left",
               "MinColor", "ColorGradient", "MinNormal", "NormalGradient"]


def fill_edge_table(scene, tri0=0, n=1, phong=True, semantics=abi.PRK_SEM_AVX, setup=None):
    """FillEdgeTable (projekt.cpp:3882-4121) on triangles [tri0, tri0+n) as one
    object; returns the sorted edge list as dicts."""
    k = _Keep(scene, semantics, phong, n, setup=setup)
    words = np.zeros(27 * 3 * n, np.uint32)
    cnt = C.c_uint32(0)
    rc = lib().oracle_fill_edge_table(C.byref(k.desc), C.c_uint32(tri0), C.c_uint32(n),
                                      C.byref(k.transform), C.byref(k.lights),
                                      _ptr(words), C.byref(cnt))
    if rc != 0:
        raise RuntimeError("oracle_fill_edge_table failed: %d" % rc)
    out = []
    w = words.reshape(-1, 27)[: cnt.value]
    f = w.view(np.float32)
    i32 = w.view(np.int32)
    for r in range(cnt.value):
        out.append(dict(YMax=int(i32[r, 0]), XMin=f[r, 1], ZMin=f[r, 2], OneOverZMin=f[r, 3],
                        Gradient=f[r, 4], ZGradient=f[r, 5], OneOverZGradient=f[r, 6],
                        YMin=int(i32[r, 7]), UMin=f[r, 8], VMin=f[r, 9], UGradient=f[r, 10],
                        VGradient=f[r, 11], Left=int(i32[r, 12]), MinColor=f[r, 13:17].copy(),
                        ColorGradient=f[r, 17:21].copy(), MinNormal=f[r, 21:24].copy(),
                        NormalGradient=f[r, 24:27].copy()))
    return out


def fill_edge_table_words(scene, tri0=0, n=1, phong=True, semantics=abi.PRK_SEM_AVX, setup=None):
    """FillEdgeTable (projekt.cpp:3882-4121) on triangles [tri0, tri0+n) as one
    object: the sorted edges as uint32 words [count, 27] in prk_edge layout.
    setup: FillEdgeTable's own PhongShading / Object->Bitmap (PRK_SETUP_*)."""
    k = _Keep(scene, semantics, phong, n, setup=setup)
    words = np.zeros(27 * 3 * n + 27, np.uint32)
    cnt = C.c_uint32(0)
    rc = lib().oracle_fill_edge_table(C.byref(k.desc), C.c_uint32(tri0), C.c_uint32(n),
                                      C.byref(k.transform), C.byref(k.lights), _ptr(words), C.byref(cnt))
    if rc != 0:
        raise RuntimeError("oracle_fill_edge_table failed: %d" % rc)
    return words.reshape(-1, 27)[: cnt.value].copy()


def advance_edges(edge_words, height):
    """What DrawModel* leaves in the caller's edge list ([n, 27] prk_edge
    words, sorted as FillEdgeTable leaves them) after walking it over a frame
    of `height` rows (projekt.cpp:3654-3869, edge step 3811-3829): (advanced
    words, Next as an index into the list or -1)."""
    w = np.array(edge_words, np.uint32, copy=True, order="C")
    n = w.shape[0]
    nxt = np.full(n, -1, np.int32)
    L = lib()
    L.oracle_advance_edges.restype = C.c_int
    rc = L.oracle_advance_edges(_ptr(w), C.c_uint32(n), C.c_int32(height), _ptr(nxt))
    if rc != 0:
        raise RuntimeError("oracle_advance_edges failed: %d" % rc)
    return w, nxt


def _src_render(fn, scene, items, semantics, color, z, tri_index, phong=True):
    W, H = scene.width, scene.height
    col = np.full((H, W), CLEAR_COLOR, np.uint32) if color is None else color
    zb = np.full((H, W), CLEAR_Z, np.float32) if z is None else z
    win = np.full((H, W), -1, np.int32)
    k = _Keep(scene, semantics, phong, 1)
    tg = OrTarget(_ptr(col), W * 4, _ptr(zb), W, H, _ptr(win))
    stats = (C.c_uint64 * 3)()
    items = np.ascontiguousarray(items, np.uint32)
    bm = C.pointer(k.bitmap) if k.bitmap is not None else None
    rc = fn(_ptr(items), C.c_uint32(items.shape[0]), C.c_int32(semantics), bm, C.c_int32(int(bool(phong))),
            C.c_int32(k.desc.Filter), C.c_int32(tri_index), C.byref(tg), C.byref(k.transform), C.byref(k.lights),
            stats)
    if rc != 0:
        raise RuntimeError("oracle draw failed: %d" % rc)
    return col, zb, win, dict(spans=stats[0], span_pixels=stats[1], writes=stats[2])


def render_edges(scene, edge_words, semantics=abi.PRK_SEM_AVX, color=None, z=None, tri_index=0, phong=True):
    """DrawModelOptimized* (or, PRK_SEM_SCALAR, DrawModel) of one ready edge
    list ([n, 27] prk_edge words) with the scene's camera, lights and texture."""
    return _src_render(lib().oracle_draw_edges, scene, edge_words, semantics, color, z, tri_index, phong)


def render_spans(scene, span_words, semantics=abi.PRK_SEM_AVX, color=None, z=None, tri_index=0):
    """FillLineOptimized on caller spans ([n, 25] prk_span words)."""
    return _src_render(lib().oracle_draw_spans, scene, span_words, semantics, color, z, tri_index)
