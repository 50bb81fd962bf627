"""Print the one-wave object walk's LDS capacity on device 0 (prk_obj_walk_lcap)."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cpu-renderer_amd"))
import prk  # noqa: E402

L = prk.lib()
f = L.prk_obj_walk_lcap
f.restype = ctypes.c_uint32
print("prk_obj_walk_lcap =", f())
