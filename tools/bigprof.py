"""Phase cycles of the huge-object walk (k_obj_walk_big) in a -DPRK_WPROF=1
build (tools/build_variant.sh, make variant_all NAME=wprof VARIANT=-DPRK_WPROF=1):
C3b as ONE object, one frame.
usage: PRK_LIB=cpu-renderer_amd/libprk_hip_wprof.so python tools/bigprof.py [case]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cpu-renderer_amd"))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import prk  # noqa: E402
import time_objects as T  # noqa: E402

want = sys.argv[1] if len(sys.argv) > 1 else "c3b_1obj_avx"
NAMES = {0: "window", 1: "insert+expire", 2: "expiry alone", 5: "pairing", 9: "samples", 10: "sample scan",
         11: "gap search", 12: "rank", 13: "scan+move", 14: "new edges placed", 15: "pairing reads (LDS walk)"}
# (k_obj_walk_lds's counters: 9 samples + their scan, 10 gap search, 11 bins + ranks, 12 old entries +
#  kept scan, 13 places, 14 moves, 15 pairing's read pass -- the labels above are k_obj_walk_big's)
for name, s, sem, phong, tpo in T.cases():
    if name != want:
        continue
    r = prk.Renderer(0)
    try:
        r.target_alloc(s.width, s.height)
        r.set_camera(s.prk_transform(), s.prk_lights())
        g = r.geometry(s.vertices, s.colors, s.normals, s.uvs)
        tex = None if sem == prk.abi.PRK_SEM_SCALAR else r.texture(s.texture)
        r.timing_reset()
        r.clear_on_flush()
        r.draw(sem, g, s.tri_count, P=s.P, bitmap=tex, phong=phong, tris_per_object=tpo)
        r.complete_all_work()
        r.synchronize()
        c = [int(x) for x in r.debug_counters(16)]
        rows = max(1, c[3])
        print("%s: rows %d batches %d new edges %d mean list %.0f, whole walk %.3g clocks (%.0f a row)"
              % (name, c[3], c[4], c[8], c[6] / rows, c[7], c[7] / rows))
        for k, v in sorted(NAMES.items()):
            print("  %-18s %10.0f clocks a row" % (v, c[k] / rows))
    finally:
        r.close()
