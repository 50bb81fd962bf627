"""prk — Python binding of libprk_hip.so (the MI355X rasterizer C-ABI).

Mirrors the reference's draw interface (projekt.cpp, MacSpain/cpu-renderer):

    reference                                   here
    ------------------------------------------  ---------------------------------
    FillEdgeTable(Object, Commands, Phong)      Renderer.draw_* record the object
    DrawModelOptimized(Queue, Buffer, Edges,    Renderer.draw_model_optimized()
        EdgeCount, Commands, Bitmap, Phong)     (FillLineOptimized semantics)
    DrawModel(Buffer, Edges, EdgeCount,         Renderer.draw_model()
        Commands, Bitmap, Phong)                (scalar DrawModel semantics)
    Platform.CompleteAllWork(Queue)             Renderer.complete_all_work()

The HIP library is the only compute path: there is no CPU fallback, and every
entry point raises PrkError if libprk_hip.so or the GPU is missing.
"""
import atexit
import ctypes as C
import os
import sys
import weakref

import numpy as np

from . import abi
from . import scenes as scenes_mod
from .abi import PRK_SEM_AVX, PRK_SEM_AVX_ST, PRK_SEM_SCALAR  # noqa: F401

_HERE = os.path.dirname(os.path.abspath(__file__))
_DEFAULT_LIB = os.path.join(os.path.dirname(_HERE), "libprk_hip.so")
LIB_PATH = os.environ.get("PRK_LIB") or _DEFAULT_LIB
HEADER_PATH = os.path.join(os.path.dirname(os.path.dirname(_HERE)), "include", "prk.h")

_LIB = None


class PrkError(RuntimeError):
    def __init__(self, fn, code):
        super().__init__("%s failed: %s (%d)" % (fn, abi.STATUS_NAMES.get(code, "?"), code))
        self.code = code


_SIGS = {
    "prk_create": (C.c_int, [C.c_int, C.POINTER(C.c_void_p)]),
    "prk_destroy": (C.c_int, [C.c_void_p]),
    "prk_runtime_check": (C.c_int, []),
    "prk_device_count": (C.c_int, [C.POINTER(C.c_int)]),
    "prk_version": (C.c_char_p, []),
    "prk_target_bind": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int32, C.c_void_p, C.c_int32, C.c_int32,
                                  C.c_int32, C.c_int32]),
    "prk_target_alloc": (C.c_int, [C.c_void_p, C.c_int32, C.c_int32, C.c_int32, C.c_int32,
                                   C.POINTER(C.c_void_p), C.POINTER(C.c_void_p)]),
    "prk_target_clear": (C.c_int, [C.c_void_p, C.c_uint32, C.c_float]),
    "prk_target_clear_on_flush": (C.c_int, [C.c_void_p, C.c_uint32, C.c_float]),
    "prk_target_download": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int32, C.c_void_p]),
    "prk_target_upload": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int32, C.c_void_p]),
    "prk_target_upload_async": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int32, C.c_void_p]),
    "prk_set_camera": (C.c_int, [C.c_void_p, C.POINTER(abi.PrkTransform), C.POINTER(abi.PrkLightData)]),
    "prk_set_shade_camera": (C.c_int, [C.c_void_p, C.POINTER(abi.PrkTransform), C.POINTER(abi.PrkLightData)]),
    "prk_texture_create": (C.c_int, [C.c_void_p, C.POINTER(abi.PrkBitmap), C.POINTER(C.c_int32)]),
    "prk_texture_set_filter": (C.c_int, [C.c_void_p, C.c_int32, C.c_int32]),
    "prk_texture_update": (C.c_int, [C.c_void_p, C.c_int32, C.POINTER(abi.PrkBitmap)]),
    "prk_geometry_update": (C.c_int, [C.c_void_p, C.c_int32, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                                      C.c_uint32]),
    "prk_geometry_write": (C.c_int, [C.c_void_p, C.c_int32, C.c_uint32, C.c_uint32, C.c_void_p, C.c_void_p,
                                     C.c_void_p, C.c_void_p]),
    "prk_host_alloc": (C.c_int, [C.c_void_p, C.c_size_t, C.POINTER(C.c_void_p)]),
    "prk_host_free": (C.c_int, [C.c_void_p, C.c_void_p]),
    "prk_host_register": (C.c_int, [C.c_void_p, C.c_void_p, C.c_size_t]),
    "prk_host_unregister": (C.c_int, [C.c_void_p, C.c_void_p]),
    "prk_geometry_create": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                                      C.c_uint32, C.POINTER(C.c_int32)]),
    "prk_geometry_wrap_device": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                                           C.c_uint32, C.POINTER(C.c_int32)]),
    "prk_draw": (C.c_int, [C.c_void_p, C.c_int32, C.c_uint32, C.c_uint32, C.POINTER(C.c_float),
                           C.c_int32, C.c_int32, C.c_int32]),
    "prk_draw_objects": (C.c_int, [C.c_void_p, C.c_int32, C.c_uint32, C.c_uint32, C.c_uint32,
                                   C.POINTER(C.c_float), C.c_int32, C.c_int32, C.c_int32]),
    "prk_draw_objects_setup": (C.c_int, [C.c_void_p, C.c_int32, C.c_uint32, C.c_uint32, C.c_uint32,
                                         C.POINTER(C.c_float), C.c_int32, C.c_int32, C.c_int32, C.c_int32]),
    "prk_draw_edges": (C.c_int, [C.c_void_p, C.c_void_p, C.c_uint32, C.c_int32, C.c_int32, C.c_int32]),
    "prk_draw_spans": (C.c_int, [C.c_void_p, C.c_void_p, C.c_uint32, C.c_int32, C.c_int32, C.c_int32]),
    "prk_flush": (C.c_int, [C.c_void_p, C.c_void_p]),
    "prk_reset_draws": (C.c_int, [C.c_void_p]),
    "prk_synchronize": (C.c_int, [C.c_void_p]),
    "prk_resolve": (C.c_int, [C.c_void_p, C.c_void_p]),
    "prk_get_stats": (C.c_int, [C.c_void_p, C.POINTER(abi.PrkStats)]),
    "prk_timing_reset": (C.c_int, [C.c_void_p]),
    "prk_set_debug": (C.c_int, [C.c_void_p, C.c_int32]),
    "prk_set_early_z": (C.c_int, [C.c_void_p, C.c_int]),
    "prk_download_winners": (C.c_int, [C.c_void_p, C.c_void_p]),
    "prk_debug_counters": (C.c_int, [C.c_void_p, C.POINTER(C.c_uint64), C.c_int32]),
    "prk_set_tile": (C.c_int, [C.c_void_p, C.c_int32, C.c_int32]),
    "prk_construct_sphere": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                                       C.POINTER(C.c_uint32)]),
    "prk_fill_edge_records": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint32,
                                        C.POINTER(C.c_float), C.POINTER(abi.PrkTransform),
                                        C.POINTER(abi.PrkLightData), C.c_int32, C.c_void_p, C.c_size_t,
                                        C.c_size_t, C.c_void_p, C.POINTER(C.c_uint32)]),
    "prk_advance_edge_records": (C.c_int, [C.c_void_p, C.c_uint32, C.c_size_t, C.c_size_t, C.c_int32]),
    "prk_fill_edge_count": (C.c_int, [C.c_void_p, C.c_uint32, C.POINTER(C.c_float), C.POINTER(abi.PrkTransform),
                                      C.POINTER(C.c_uint32)]),
    "prk_get_target": (C.c_int, [C.c_void_p, C.POINTER(C.c_void_p), C.POINTER(C.c_int32), C.POINTER(C.c_void_p),
                                 C.POINTER(C.c_int32), C.POINTER(C.c_int32), C.POINTER(C.c_int32),
                                 C.POINTER(C.c_int32)]),
    "prk_get_device": (C.c_int, [C.c_void_p, C.POINTER(C.c_int32), C.POINTER(C.c_void_p)]),
    "prk_band_rows": (C.c_int, [C.c_int32, C.c_int32, C.c_int32, C.POINTER(C.c_int32), C.POINTER(C.c_int32)]),
    "prk_selftest_div": (C.c_int, [C.c_int32, C.c_uint32, C.c_uint64, C.POINTER(C.c_uint64)]),
    "prk_comm_available": (C.c_int, []),
    "prk_comm_unique_id": (C.c_int, [C.c_void_p]),
    "prk_comm_init": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int32, C.c_int32, C.POINTER(C.c_void_p)]),
    "prk_comm_init_all": (C.c_int, [C.POINTER(C.c_void_p), C.c_int32, C.POINTER(C.c_void_p)]),
    "prk_comm_destroy": (C.c_int, [C.c_void_p]),
    "prk_gather_frame": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int32, C.c_void_p, C.c_int32, C.c_void_p,
                                   C.c_void_p]),
    "prk_gather_frame_all": (C.c_int, [C.POINTER(C.c_void_p), C.POINTER(C.c_void_p), C.c_int32, C.c_int32,
                                       C.c_void_p, C.c_int32, C.c_void_p]),
    "prk_gather_frame_local": (C.c_int, [C.POINTER(C.c_void_p), C.c_int32, C.c_int32, C.c_void_p, C.c_int32,
                                         C.c_void_p]),
}

COMM_ID_BYTES = 128  # PRK_COMM_ID_BYTES


def exported_symbols():
    return list(_SIGS)


def lib(path=None):
    """Load libprk_hip.so (fails loudly if it has not been built)."""
    global _LIB
    if _LIB is None:
        p = path or LIB_PATH
        if not os.path.exists(p):
            raise PrkError("load libprk_hip.so (%s: not built; run __graft_entry__.build())" % p, -3)
        # One ROCm runtime per process: torch ships its own libamdhip64 /
        # librccl / librocm_smi64 under names (libamdhip64.so, librccl.so) that
        # do not match this library's (libamdhip64.so.7 via /opt/rocm, and the
        # librccl.so.1 prk_comm_* dlopens).  Loaded first, torch's copies
        # satisfy ours by SONAME; loaded after us, torch would map a second
        # copy of each, and two librocm_smi64 copies destroy the same
        # interposed static map at exit (glibc "double free").
        # PRK_NO_TORCH_PRELOAD=1 skips this (a process that never imports
        # torch: the library's own /opt/rocm stack alone, no torch import cost).
        if os.environ.get("PRK_NO_TORCH_PRELOAD", "0") != "1":
            try:
                import torch  # noqa: F401
            except Exception:  # no (usable) torch: this library's own ROCm stack alone
                pass
        atexit.register(_close_all)  # after torch's handlers: runs before them
        L = C.CDLL(p)
        # (A/B tools load older builds through PRK_LIB that may lack newer entry points)
        variant = os.path.abspath(p) != os.path.abspath(_DEFAULT_LIB)
        for name, (res, args) in _SIGS.items():
            if variant and not hasattr(L, name):
                continue
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _LIB = L
    return _LIB


def _check(fn, rc):
    if rc != abi.PRK_OK:
        raise PrkError(fn, rc)


def _ptr(a):
    return None if a is None else C.c_void_p(a.ctypes.data)


def device_count():
    n = C.c_int(0)
    _check("prk_device_count", lib().prk_device_count(C.byref(n)))
    return n.value


def construct_sphere():
    """ConstructSphere (projekt.cpp:4123-4289) -> (V[6624,3], C[6624,4], N[6624,3], UV[6624,2])."""
    V = np.zeros((6624, 3), np.float32)
    Cc = np.zeros((6624, 4), np.float32)
    N = np.zeros((6624, 3), np.float32)
    UV = np.zeros((6624, 2), np.float32)
    n = C.c_uint32(0)
    _check("prk_construct_sphere", lib().prk_construct_sphere(_ptr(V), _ptr(Cc), _ptr(N), _ptr(UV),
                                                               C.byref(n)))
    return V[: n.value], Cc[: n.value], N[: n.value], UV[: n.value]


def fill_edge_count(vertices, P, transform):
    """prk_fill_edge_count: FillEdgeTable's return value (projekt.cpp:4119)
    for one object (host-side, no device needed)."""
    v = np.ascontiguousarray(vertices, np.float32)
    Pc = (C.c_float * 3)(*(P or (0.0, 0.0, 0.0)))
    n = C.c_uint32(0)
    _check("prk_fill_edge_count", lib().prk_fill_edge_count(_ptr(v), v.shape[0], Pc, C.byref(transform),
                                                             C.byref(n)))
    return n.value


# x86-64 edge_info (projekt.h:17-37): 27 four-byte fields, pad, Next pointer
EDGE_INFO_STRIDE, EDGE_INFO_NEXT = 120, 112


def fill_edge_records(vertices, colors, normals, uvs, P, transform, lights, setup, memory=None):
    """prk_fill_edge_records: FillEdgeTable's records (projekt.cpp:3894-4117)
    written in place into `memory` (uint8 [>= 3T, 120]: x86-64 edge_info
    elements; default zeros).  Returns (memory, count)."""
    arrs = [None if a is None else np.ascontiguousarray(a, np.float32) for a in (vertices, colors, normals, uvs)]
    nv = arrs[0].shape[0]
    if memory is None:
        memory = np.zeros((max(1, nv), EDGE_INFO_STRIDE), np.uint8)
    Pc = (C.c_float * 3)(*(P or (0.0, 0.0, 0.0)))
    n = C.c_uint32(0)
    _check("prk_fill_edge_records", lib().prk_fill_edge_records(
        *[_ptr(a) for a in arrs], nv, Pc, C.byref(transform), C.byref(lights), int(setup), _ptr(memory),
        EDGE_INFO_STRIDE, EDGE_INFO_NEXT, None, C.byref(n)))
    return memory, n.value


def advance_edge_records(memory, count, height):
    """prk_advance_edge_records on an edge_info array (uint8 [n, 120]) in
    place: what DrawModel* leaves in it (projekt.cpp:3654-3869)."""
    _check("prk_advance_edge_records", lib().prk_advance_edge_records(
        _ptr(memory), count, EDGE_INFO_STRIDE, EDGE_INFO_NEXT, int(height)))
    return memory


def edge_record_words(memory, count):
    """(fields as uint32 [count, 27], Next as an element index or -1)."""
    w = memory[:count, :108].copy().view(np.uint32).reshape(count, 27)
    ptr = memory[:count, EDGE_INFO_NEXT:EDGE_INFO_NEXT + 8].copy().view(np.uint64).reshape(count)
    base = memory.ctypes.data
    nxt = np.where(ptr == 0, -1, (ptr.astype(np.int64) - base) // EDGE_INFO_STRIDE).astype(np.int32)
    return w, nxt


def selftest_div(n=1 << 22, seed=1, device=0):
    """prk_selftest_div: (quotient mismatches, normalisation mismatches) of the
    shared-divisor division against the compiler's x / d over n draws."""
    out = C.c_uint64()
    _check("prk_selftest_div", lib().prk_selftest_div(device, n, seed, C.byref(out)))
    return out.value & 0xFFFFFFFF, out.value >> 32


def band_rows(height, rank, nranks):
    """prk_band_rows: frame rows [row0, row1) of rank `rank` of `nranks`."""
    a, b = C.c_int32(0), C.c_int32(0)
    _check("prk_band_rows", lib().prk_band_rows(height, rank, nranks, C.byref(a), C.byref(b)))
    return a.value, b.value


def comm_available():
    """True when librccl can be loaded (prk_comm_*)."""
    return bool(lib().prk_comm_available())


def comm_unique_id():
    """prk_comm_unique_id (rank 0): the RCCL unique id as bytes."""
    buf = (C.c_uint8 * COMM_ID_BYTES)()
    _check("prk_comm_unique_id", lib().prk_comm_unique_id(buf))
    return bytes(buf)


class Comm:
    """An RCCL communicator of one rank (prk_comm_init) or of one context of
    a single-process group (Comm.init_all)."""

    def __init__(self, handle, rank, nranks):
        self._h, self.rank, self.nranks = handle, rank, nranks
        _LIVE.add(self)

    @classmethod
    def init(cls, renderer, uid, nranks, rank):
        buf = (C.c_uint8 * COMM_ID_BYTES).from_buffer_copy(uid)
        h = C.c_void_p()
        _check("prk_comm_init", lib().prk_comm_init(renderer._h, buf, nranks, rank, C.byref(h)))
        return cls(h, rank, nranks)

    @classmethod
    def init_all(cls, renderers):
        n = len(renderers)
        ctxs = (C.c_void_p * n)(*[r._h.value for r in renderers])
        out = (C.c_void_p * n)()
        _check("prk_comm_init_all", lib().prk_comm_init_all(ctxs, n, out))
        return [cls(C.c_void_p(out[i]), i, n) for i in range(n)]

    def close(self):
        if getattr(self, "_h", None):
            lib().prk_comm_destroy(self._h)
            self._h = None

    def gather(self, renderer, frame_color_ptr=None, frame_z_ptr=None, with_z=False, stream=None):
        """prk_gather_frame: rank 0 passes its device frame (packed rows),
        the other ranks nothing."""
        pitch = renderer.width * 4
        _check("prk_gather_frame", lib().prk_gather_frame(
            renderer._h, self._h, int(bool(with_z)), C.c_void_p(frame_color_ptr) if frame_color_ptr else None,
            pitch, C.c_void_p(frame_z_ptr) if frame_z_ptr else None,
            None if stream is None else C.c_void_p(stream)))


def gather_frame_all(renderers, comms, frame_color_ptr, frame_z_ptr=None, with_z=False):
    """prk_gather_frame_all: one process, N contexts, one RCCL group."""
    n = len(renderers)
    ctxs = (C.c_void_p * n)(*[r._h.value for r in renderers])
    cms = (C.c_void_p * n)(*[c._h.value for c in comms])
    _check("prk_gather_frame_all", lib().prk_gather_frame_all(
        ctxs, cms, n, int(bool(with_z)), C.c_void_p(frame_color_ptr), renderers[0].width * 4,
        C.c_void_p(frame_z_ptr) if frame_z_ptr else None))


def gather_frame_local(renderers, frame_color_ptr, frame_pitch, frame_z_ptr=None, with_z=False):
    """prk_gather_frame_local: every band's device copies its strip into
    renderers[0]'s device frame (peer copies, no RCCL)."""
    n = len(renderers)
    ctxs = (C.c_void_p * n)(*[r._h.value for r in renderers])
    _check("prk_gather_frame_local", lib().prk_gather_frame_local(
        ctxs, n, int(bool(with_z)), C.c_void_p(frame_color_ptr), frame_pitch,
        C.c_void_p(frame_z_ptr) if frame_z_ptr else None))


_LIVE = weakref.WeakSet()  # open Renderers / Comms, closed in a defined order at exit


def _close_all():
    """Interpreter exit: close every context still open, communicators first,
    while the HIP runtime (and torch, whose tensors a target may use) is still
    alive.  atexit runs the last-registered handler first; lib() registers
    this one right after it imports torch, so it runs before torch's.
    prk_destroy never queues GPU work (prk_api.hip), so a context whose last
    frame was never read just drops it."""
    objs = list(_LIVE)
    for o in sorted(objs, key=lambda o: 0 if isinstance(o, Comm) else 1):
        try:
            o.close()
        except Exception:
            pass


def _finalizing():
    return sys.is_finalizing()


class Renderer:
    """One GPU context: render target, camera/lights, resident geometry and
    textures, and the list of recorded draws of the current frame."""

    def __init__(self, device=0):
        self._L = lib()
        h = C.c_void_p()
        _check("prk_create", self._L.prk_create(int(device), C.byref(h)))
        self._h = h
        self._keep = []
        self.width = self.height = self.row0 = self.row1 = 0
        _LIVE.add(self)

    def close(self):
        if getattr(self, "_h", None):
            self._L.prk_destroy(self._h)
            self._h = None

    def __del__(self):
        # no GPU calls while the interpreter is tearing down (module globals,
        # torch's allocator and the HIP runtime may already be gone): the
        # atexit handler above closed every context before that began
        if _finalizing():
            return
        try:
            self.close()
        except Exception:
            pass

    # ---- target -----------------------------------------------------------
    def target_alloc(self, width, height, row0=0, row1=None):
        row1 = height if row1 is None else row1
        _check("prk_target_alloc", self._L.prk_target_alloc(self._h, width, height, row0, row1, None, None))
        self.width, self.height, self.row0, self.row1 = width, height, row0, row1

    def target_bind(self, color_ptr, pitch_bytes, z_ptr, width, height, row0=0, row1=None):
        """Bind caller-owned device memory (e.g. torch tensors' data_ptr())."""
        row1 = height if row1 is None else row1
        _check("prk_target_bind", self._L.prk_target_bind(self._h, C.c_void_p(color_ptr), pitch_bytes,
                                                          C.c_void_p(z_ptr), width, height, row0, row1))
        self.width, self.height, self.row0, self.row1 = width, height, row0, row1

    def clear(self, color=0xFF000000, z=None):
        z = -float(np.finfo(np.float32).max) if z is None else z
        _check("prk_target_clear", self._L.prk_target_clear(self._h, C.c_uint32(color), C.c_float(z)))

    def clear_on_flush(self, color=0xFF000000, z=None):
        """The same fill, fused into the next complete_all_work()."""
        z = -float(np.finfo(np.float32).max) if z is None else z
        _check("prk_target_clear_on_flush",
               self._L.prk_target_clear_on_flush(self._h, C.c_uint32(color), C.c_float(z)))

    def upload(self, color, z):
        color = np.ascontiguousarray(color, np.uint32)
        z = np.ascontiguousarray(z, np.float32)
        _check("prk_target_upload", self._L.prk_target_upload(self._h, _ptr(color), self.width * 4, _ptr(z)))

    def download(self):
        rows = self.row1 - self.row0
        color = np.empty((rows, self.width), np.uint32)
        z = np.empty((rows, self.width), np.float32)
        _check("prk_target_download", self._L.prk_target_download(self._h, _ptr(color), self.width * 4,
                                                                  _ptr(z)))
        return color, z

    def winners(self):
        rows = self.row1 - self.row0
        w = np.empty((rows, self.width), np.int32)
        _check("prk_download_winners", self._L.prk_download_winners(self._h, _ptr(w)))
        return w

    # ---- state ------------------------------------------------------------
    def set_camera(self, transform, lights):
        self._cam = (transform, lights)
        _check("prk_set_camera", self._L.prk_set_camera(self._h, C.byref(transform), C.byref(lights)))

    def set_shade_camera(self, transform, lights):
        """After set_camera: the span shading (Phong, unprojection) uses these
        instead -- Commands as DrawModel* sees them when the caller changed
        them after FillEdgeTable (projekt.cpp:452-458, 2042-2046)."""
        self._shade_cam = (transform, lights)
        _check("prk_set_shade_camera", self._L.prk_set_shade_camera(self._h, C.byref(transform),
                                                                    C.byref(lights)))

    def texture(self, tex):
        """tex: scenes.Texture (uint32 texels with the zeroed guard row)."""
        texels = np.ascontiguousarray(tex.texels, np.uint32)
        bm = abi.PrkBitmap(texels.ctypes.data, tex.width, tex.height, texels.shape[1] * 4)
        h = C.c_int32(-1)
        _check("prk_texture_create", self._L.prk_texture_create(self._h, C.byref(bm), C.byref(h)))
        if getattr(tex, "filter", abi.PRK_FILTER_NEAREST) != abi.PRK_FILTER_NEAREST:
            self.set_filter(h.value, tex.filter)
        return h.value

    def texture_update(self, handle, tex):
        """Re-read a texture's bitmap into `handle` (prk_texture_update)."""
        texels = np.ascontiguousarray(tex.texels, np.uint32)
        bm = abi.PrkBitmap(texels.ctypes.data, tex.width, tex.height, texels.shape[1] * 4)
        _check("prk_texture_update", self._L.prk_texture_update(self._h, handle, C.byref(bm)))

    def geometry_update(self, handle, vertices, colors=None, normals=None, uvs=None):
        arrs = [None if a is None else np.ascontiguousarray(a, np.float32)
                for a in (vertices, colors, normals, uvs)]
        _check("prk_geometry_update", self._L.prk_geometry_update(self._h, handle, *[_ptr(a) for a in arrs],
                                                                  arrs[0].shape[0]))

    def geometry_write(self, handle, first_vertex, vertices=None, colors=None, normals=None, uvs=None,
                       count=None):
        """prk_geometry_write of vertices [first_vertex, first_vertex+count)
        (count: the given arrays' length); waits for the copy, since the
        arrays here are temporaries."""
        arrs = [None if a is None else np.ascontiguousarray(a, np.float32)
                for a in (vertices, colors, normals, uvs)]
        if count is None:
            count = next(a.shape[0] for a in arrs if a is not None)
        _check("prk_geometry_write", self._L.prk_geometry_write(self._h, handle, first_vertex, count,
                                                                *[_ptr(a) for a in arrs]))
        self.synchronize()

    def set_filter(self, texture, filt):
        """Texture sampling: PRK_FILTER_NEAREST (the reference's) or
        PRK_FILTER_BILINEAR (an extension, AVX semantics only)."""
        _check("prk_texture_set_filter", self._L.prk_texture_set_filter(self._h, texture, filt))

    def geometry(self, vertices, colors=None, normals=None, uvs=None):
        arrs = [None if a is None else np.ascontiguousarray(a, np.float32)
                for a in (vertices, colors, normals, uvs)]
        h = C.c_int32(-1)
        nv = arrs[0].shape[0]
        _check("prk_geometry_create", self._L.prk_geometry_create(self._h, *[_ptr(a) for a in arrs],
                                                                  nv, C.byref(h)))
        return h.value

    def geometry_device(self, v_ptr, c_ptr, n_ptr, uv_ptr, vertex_count):
        h = C.c_int32(-1)
        ptrs = [C.c_void_p(p) if p else None for p in (v_ptr, c_ptr, n_ptr, uv_ptr)]
        _check("prk_geometry_wrap_device", self._L.prk_geometry_wrap_device(self._h, *ptrs, vertex_count,
                                                                            C.byref(h)))
        return h.value

    def target(self):
        """prk_get_target: (color_ptr, pitch, z_ptr, W, H, row0, row1)."""
        cp, zp = C.c_void_p(), C.c_void_p()
        v = [C.c_int32(0) for _ in range(5)]
        _check("prk_get_target", self._L.prk_get_target(self._h, C.byref(cp), C.byref(v[0]), C.byref(zp),
                                                        *[C.byref(x) for x in v[1:]]))
        return cp.value, v[0].value, zp.value, v[1].value, v[2].value, v[3].value, v[4].value

    def device_stream(self):
        """prk_get_device: (device, own stream as an int)."""
        d, s = C.c_int32(0), C.c_void_p()
        _check("prk_get_device", self._L.prk_get_device(self._h, C.byref(d), C.byref(s)))
        return d.value, s.value or 0

    def set_tile(self, tw, th):
        _check("prk_set_tile", self._L.prk_set_tile(self._h, tw, th))

    def set_debug(self, on=True):
        _check("prk_set_debug", self._L.prk_set_debug(self._h, int(bool(on))))

    def set_early_z(self, on=True):
        """prk_set_early_z: span-record frames write z in the visibility
        kernel, so download() copies it while the frame shades."""
        _check("prk_set_early_z", self._L.prk_set_early_z(self._h, int(bool(on))))

    # ---- draws (the reference's entry points) -----------------------------
    def _draw(self, geom, first_tri, tri_count, P, semantics, phong, texture, tris_per_object=1, setup=None):
        Pc = (C.c_float * 3)(*(P or (0.0, 0.0, 0.0)))
        tex = -1 if texture is None else texture
        if setup is None:
            _check("prk_draw_objects", self._L.prk_draw_objects(self._h, geom, first_tri, tri_count,
                                                                tris_per_object, Pc, semantics, int(bool(phong)), tex))
        else:  # FillEdgeTable's own PhongShading / Object->Bitmap (abi.PRK_SETUP_*)
            _check("prk_draw_objects_setup", self._L.prk_draw_objects_setup(
                self._h, geom, first_tri, tri_count, tris_per_object, Pc, semantics, int(bool(phong)), tex,
                int(setup)))

    def draw_model_optimized(self, geom, tri_count, first_tri=0, P=None, bitmap=None, phong=True):
        """DrawModelOptimized(RenderQueue, ...) -> FillLineOptimized semantics
        (projekt.cpp:3615-3871, 1492-2320).  Needs bitmap + phong."""
        self._draw(geom, first_tri, tri_count, P, abi.PRK_SEM_AVX, phong, bitmap)

    def draw_model(self, geom, tri_count, first_tri=0, P=None, bitmap=None, phong=False):
        """DrawModel (projekt.cpp:162-601) scalar semantics."""
        self._draw(geom, first_tri, tri_count, P, abi.PRK_SEM_SCALAR, phong, bitmap)

    def draw_model_optimized_st(self, geom, tri_count, first_tri=0, P=None, bitmap=None, phong=True):
        """The single-thread overload DrawModelOptimized(Buffer, ...)
        (projekt.cpp:2350-3358): FillLineOptimized's math with its left-clip
        XOffset quirk (2508) and the >= z-test (3205).  Needs bitmap + phong."""
        self._draw(geom, first_tri, tri_count, P, abi.PRK_SEM_AVX_ST, phong, bitmap)

    def draw(self, semantics, geom, tri_count, first_tri=0, P=None, bitmap=None, phong=True, tris_per_object=1,
             setup=None):
        """Any PRK_SEM_* draw; tris_per_object > 1: consecutive objects of that
        many triangles, one active edge table each (prk_draw_objects).
        setup: FillEdgeTable's own PhongShading / Object->Bitmap as
        abi.PRK_SETUP_* bits (None: as the draw; prk_draw_objects_setup)."""
        self._draw(geom, first_tri, tri_count, P, semantics, phong, bitmap, tris_per_object, setup)

    def draw_edges(self, edge_words, semantics=abi.PRK_SEM_AVX, bitmap=None, phong=True):
        """DrawModelOptimized* on a ready edge_info list: uint32 [n, 27] in
        prk_edge layout (prk.h), sorted by YMin as FillEdgeTable leaves it."""
        w = np.ascontiguousarray(edge_words, np.uint32)
        self._keep.append(w)
        _check("prk_draw_edges", self._L.prk_draw_edges(self._h, _ptr(w), w.shape[0], semantics, int(bool(phong)),
                                                        -1 if bitmap is None else bitmap))

    def draw_spans(self, span_words, semantics=abi.PRK_SEM_AVX, bitmap=None, phong=True):
        """Caller spans (the work records of DoLineRenderWork): uint32 [n, 25]
        in prk_span layout (prk.h)."""
        w = np.ascontiguousarray(span_words, np.uint32)
        self._keep.append(w)
        _check("prk_draw_spans", self._L.prk_draw_spans(self._h, _ptr(w), w.shape[0], semantics, int(bool(phong)),
                                                        -1 if bitmap is None else bitmap))

    def complete_all_work(self, stream=None):
        """Platform.CompleteAllWork: run every recorded draw (asynchronous)."""
        _check("prk_flush", self._L.prk_flush(self._h, None if stream is None else C.c_void_p(stream)))

    flush = complete_all_work

    def reset_draws(self):
        _check("prk_reset_draws", self._L.prk_reset_draws(self._h))

    def synchronize(self):
        _check("prk_synchronize", self._L.prk_synchronize(self._h))

    def resolve(self, stream=None):
        """Resolve the last flush's bin count (an overflowed frame is re-run
        first) and make `stream` wait for the frame's end, host-asynchronously:
        call before reading the target on another stream (prk.dist gathers)."""
        _check("prk_resolve", self._L.prk_resolve(self._h, None if stream is None else C.c_void_p(stream)))

    def timing_reset(self):
        _check("prk_timing_reset", self._L.prk_timing_reset(self._h))

    def debug_counters(self, n=16):
        out = (C.c_uint64 * n)()
        _check("prk_debug_counters", self._L.prk_debug_counters(self._h, out, n))
        return list(out)

    def stats(self):
        s = abi.PrkStats()
        _check("prk_get_stats", self._L.prk_get_stats(self._h, C.byref(s)))
        return {k: getattr(s, k) for k, _ in abi.PrkStats._fields_}


def render_scene(scene, semantics=abi.PRK_SEM_AVX, phong=True, device=0, tile=None, debug=True,
                 color=None, z=None, rows=None, fused_clear=False, tris_per_object=1, setup=None,
                 shade_camera=None, early_z=False):
    """Convenience: draw a whole scenes.Scene (per-triangle submission) and
    return (color, z, winners or None, stats).  fused_clear: upload
    color / z, then clear through prk_target_clear_on_flush (the frame must
    overwrite them).  setup: FillEdgeTable's own inputs (abi.PRK_SETUP_*) of
    every draw.  shade_camera: a scene whose transform / lights shade the
    spans (set_shade_camera); `scene`'s set the draws up.  early_z:
    set_early_z (z written by the visibility kernel, copied early)."""
    r = Renderer(device)
    try:
        r0, r1 = (0, scene.height) if rows is None else rows
        r.target_alloc(scene.width, scene.height, r0, r1)
        if color is None and z is None:
            r.clear()
        else:
            r.upload(color[r0:r1], z[r0:r1])
        if fused_clear:
            r.clear_on_flush()
        if tile:
            r.set_tile(*tile)
        r.set_debug(debug)
        if early_z:
            r.set_early_z(True)
        r.set_camera(scene.prk_transform(), scene.prk_lights())
        if shade_camera is not None:
            r.set_shade_camera(shade_camera.prk_transform(), shade_camera.prk_lights())
        g = r.geometry(scene.vertices, scene.colors, scene.normals, scene.uvs)
        draws = scene.draws if scene.draws is not None else [(0, scene.tri_count, scene.texture)]
        handles = {}
        for d in draws:
            first, count, texture, sem, tpo = scenes_mod.draw_spec(d, semantics, tris_per_object)
            tex = None
            if texture is not None:
                if id(texture) not in handles:
                    handles[id(texture)] = r.texture(texture)
                tex = handles[id(texture)]
            r.draw(sem, g, count, first_tri=first, P=scene.P, bitmap=tex, phong=phong, tris_per_object=tpo,
                   setup=setup)
        r.complete_all_work()
        r.synchronize()
        col, zb = r.download()
        win = r.winners() if debug else None
        return col, zb, win, r.stats()
    finally:
        r.close()
