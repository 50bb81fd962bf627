"""Phase cycles of the one-wave object walk (a -DPRK_WPROF=1 build, PRK_LIB):
insertion / expiry / pairing per walked row, for the time_objects cases.
usage: PRK_LIB=cpu-renderer_amd/libprk_hip_wprof.so python tools/wprof.py [case ...]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cpu-renderer_amd"))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import prk  # noqa: E402
import time_objects as T  # noqa: E402

want = set(sys.argv[1:]) or {"sphere_1obj_avx", "c2_1obj_avx"}
for name, s, sem, phong, tpo in T.cases():
    if name not in want:
        continue
    r = prk.Renderer(0)
    try:
        r.target_alloc(s.width, s.height)
        r.set_camera(s.prk_transform(), s.prk_lights())
        g = r.geometry(s.vertices, s.colors, s.normals, s.uvs)
        tex = None if sem == prk.abi.PRK_SEM_SCALAR else r.texture(s.texture)
        for rep in range(2):
            r.timing_reset()
            r.clear_on_flush()
            r.draw(sem, g, s.tri_count, P=s.P, bitmap=tex, phong=phong, tris_per_object=tpo)
            r.complete_all_work()
            r.synchronize()
        c = [int(x) for x in r.debug_counters(16)]
        rows = max(1, c[3])
        print("%s: rows %d new edges %d batches %d one-at-a-time %d | clocks per row (s_memtime): insert %.0f "
              "expiry %.0f pair %.0f, walk %.0f per row, %.0f in all"
              % (name, c[3], c[8], c[4], c[6], c[0] / rows, c[1] / rows, c[2] / rows, c[7] / rows, c[7]),
              flush=True)

    finally:
        r.close()
