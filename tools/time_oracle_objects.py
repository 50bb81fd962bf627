"""CPU baseline of the whole-object cases of tools/time_objects.py: the
scalar C oracle (oracle/prk_oracle.c, the reference's list-pointer AET of
DrawModelOptimized / DrawModel restated, one thread, as the reference walks
one object) timed on the same scenes.  Test infrastructure: a reported
baseline for profiles/r05/objects_final.json, never the product.

usage: python tools/time_oracle_objects.py [--only a,b] [--json OUT]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import oracle as O  # noqa: E402
from time_objects import cases  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", default="")
    ap.add_argument("--json")
    a = ap.parse_args()
    only = set(x for x in a.only.split(",") if x)
    out = {}
    for name, s, sem, phong, tpo in cases():
        if only and name not in only:
            continue
        t0 = time.perf_counter()
        O.render(s, semantics=sem, phong=phong, threads=1, tris_per_object=tpo)
        ms = (time.perf_counter() - t0) * 1e3
        out[name] = {"tris": s.tri_count, "tris_per_object": tpo, "target": "%dx%d" % (s.width, s.height),
                     "oracle_ms_per_frame_1_thread": round(ms, 1)}
        print(json.dumps({name: out[name]}), flush=True)
    if a.json:
        with open(a.json, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
