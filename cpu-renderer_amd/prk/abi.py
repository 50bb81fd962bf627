"""ctypes mirror of include/prk.h (plain structs only).

These are the caller-owned types the reference takes at its draw entry
points and that live in its absent platform header: projective_transform,
light_info / light_data, loaded_bitmap (projekt.cpp:77-90, 452-484, 1506,
3885).  See include/prk.h for the field-by-field citations.
"""
import ctypes as C

PRK_MAX_LIGHTS = 8

PRK_OK = 0
PRK_ERR_ARG = -1
PRK_ERR_UNSUPPORTED = -2
PRK_ERR_DEVICE = -3
PRK_ERR_NOMEM = -4
PRK_ERR_NO_TARGET = -5
PRK_ERR_LIMIT = -6
PRK_ERR_RUNTIME_MIX = -7

PRK_SEM_SCALAR = 0  # DrawModel            projekt.cpp:162-601
PRK_SEM_AVX = 1     # FillLineOptimized    projekt.cpp:1492-2320
PRK_SEM_AVX_ST = 2  # DrawModelOptimized(Buffer,...) single-thread overload, projekt.cpp:2350-3358

# FillEdgeTable's own inputs (prk_draw_objects_setup): its PhongShading
# argument and Object->Bitmap != 0 (projekt.cpp:4012-4089)
PRK_SETUP_PHONG = 1
PRK_SETUP_BITMAP = 2

PRK_FILTER_NEAREST = 0   # the reference's sampling (projekt.cpp:1881-2032)
PRK_FILTER_BILINEAR = 1  # extension (AVX semantics)

STATUS_NAMES = {
    PRK_OK: "PRK_OK", PRK_ERR_ARG: "PRK_ERR_ARG", PRK_ERR_UNSUPPORTED: "PRK_ERR_UNSUPPORTED",
    PRK_ERR_DEVICE: "PRK_ERR_DEVICE", PRK_ERR_NOMEM: "PRK_ERR_NOMEM",
    PRK_ERR_NO_TARGET: "PRK_ERR_NO_TARGET", PRK_ERR_RUNTIME_MIX: "PRK_ERR_RUNTIME_MIX",
    PRK_ERR_LIMIT: "PRK_ERR_LIMIT",
}


class PrkTransform(C.Structure):
    _fields_ = [("DistanceAboveTarget", C.c_float), ("FocalLength", C.c_float),
                ("MetersToPixels", C.c_float), ("ScreenCenter", C.c_float * 2)]


class PrkLightInfo(C.Structure):
    _fields_ = [("P", C.c_float * 3), ("Intensity", C.c_float * 4)]


class PrkLightData(C.Structure):
    _fields_ = [("LightCount", C.c_uint32), ("AmbientIntensity", C.c_float * 4),
                ("Lights", PrkLightInfo * PRK_MAX_LIGHTS)]


class PrkBitmap(C.Structure):
    _fields_ = [("Memory", C.c_void_p), ("Width", C.c_int32), ("Height", C.c_int32),
                ("Pitch", C.c_int32)]


class PrkStats(C.Structure):
    _fields_ = [("triangles", C.c_uint64), ("bin_entries", C.c_uint64), ("tiles", C.c_uint32),
                ("frames_timed", C.c_uint32), ("ms_bin", C.c_float), ("ms_raster", C.c_float),
                ("sum_ms_bin", C.c_double), ("sum_ms_raster", C.c_double),
                ("anomalies", C.c_uint32), ("slow_replays", C.c_uint32), ("sum_ms_vis", C.c_double), ("sum_ms_span", C.c_double),
                ("objects_chunked", C.c_uint32), ("objects_walked", C.c_uint32),
                ("object_chunks", C.c_uint32), ("object_chunks_rewalked", C.c_uint32)]


def make_transform(D, F, M2P, cx, cy):
    t = PrkTransform()
    t.DistanceAboveTarget = D
    t.FocalLength = F
    t.MetersToPixels = M2P
    t.ScreenCenter[0] = cx
    t.ScreenCenter[1] = cy
    return t


def make_lights(lights, ambient):
    """lights: list of ((px,py,pz), (r,g,b,a)); ambient: (r,g,b,a)."""
    if len(lights) > PRK_MAX_LIGHTS:
        raise ValueError("at most %d lights" % PRK_MAX_LIGHTS)
    ld = PrkLightData()
    ld.LightCount = len(lights)
    for c in range(4):
        ld.AmbientIntensity[c] = ambient[c]
    for i, (p, inten) in enumerate(lights):
        for c in range(3):
            ld.Lights[i].P[c] = p[c]
        for c in range(4):
            ld.Lights[i].Intensity[c] = inten[c]
    return ld
