"""Summarise rocprofv3 PMC passes into profiles/pmc_traffic.json.

Usage (on the GPU box, two separate passes as MI355X_MICROARCH.md prescribes:
FETCH_SIZE and WRITE_SIZE do not fit one TCC pass):
    rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d D -o fetch -- python3 bench.py ...
    rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d D -o write -- python3 bench.py ...
    python tools/pmc_traffic.py D <config-key> <round> [out.json]

Per frame: every dispatch of the profiled run (binning, the raster kernels,
library scans/sorts and fills) summed, divided by the number of frames
(k_pix dispatches).  FETCH_SIZE and WRITE_SIZE are in KiB.  gfx950
correction (MI355X_MICROARCH.md §HBM): FETCH_SIZE reports half the bytes of a
wide coalesced read, so the read side is doubled; WRITE_SIZE is taken as is.
The guide calibrates both only for 16-B/lane streams (most of these kernels
read 4-16 B per lane at scattered addresses), so the raw sum is kept beside
the corrected total and the truth lies between them.
"""
import collections
import csv
import glob
import json
import os
import sys


def per_kernel(d, counter):
    acc = collections.defaultdict(list)
    for p in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(p) as f:
            for r in csv.DictReader(f):
                if r.get("Counter_Name") != counter:
                    continue
                name = r.get("Kernel_Name", "").split("(")[0].replace("void ", "")
                acc[name].append(float(r["Counter_Value"]))
    return acc


def short(name):
    for k in ("k_vis", "k_walk", "k_pix", "k_bin_count", "k_bin_emit", "k_tile_offsets", "k_fill_target",
              "k_setup", "k_bin"):
        if k in name:
            return k
    if "k_cs_" in name or "k_won_" in name:  # the counting sort's own kernels (their "scan" is not rocprim's)
        return name.split("(")[0][:60]
    if "radix_sort" in name:
        return "rocprim radix sort"
    if "scan" in name:
        return "rocprim/hipcub scan"
    if "partition" in name or "select" in name:
        return "hipcub select"
    return name[:60]


def main():
    d, key = sys.argv[1], sys.argv[2]
    rnd = sys.argv[3] if len(sys.argv) > 3 else "?"
    out = sys.argv[4] if len(sys.argv) > 4 else os.path.join(os.path.dirname(os.path.dirname(
        os.path.abspath(__file__))), "profiles", "pmc_traffic.json")
    fetch, write = per_kernel(d, "FETCH_SIZE"), per_kernel(d, "WRITE_SIZE")
    frames_f = len([v for k, vs in fetch.items() if "k_pix" in k for v in vs])
    frames_w = len([v for k, vs in write.items() if "k_pix" in k for v in vs])
    if not frames_f or not frames_w:
        print("no k_pix FETCH_SIZE/WRITE_SIZE rows under %s" % d)
        sys.exit(1)
    per = collections.defaultdict(lambda: {"FETCH_SIZE_KiB": 0.0, "WRITE_SIZE_KiB": 0.0})
    for k, vs in fetch.items():
        per[short(k)]["FETCH_SIZE_KiB"] += sum(vs) / frames_f
    for k, vs in write.items():
        per[short(k)]["WRITE_SIZE_KiB"] += sum(vs) / frames_w
    fk = sum(v["FETCH_SIZE_KiB"] for v in per.values())
    wk = sum(v["WRITE_SIZE_KiB"] for v in per.values())
    for v in per.values():
        v["hbm_bytes_per_frame"] = (2.0 * v["FETCH_SIZE_KiB"] + v["WRITE_SIZE_KiB"]) * 1024.0
    entry = {
        "round": rnd,
        "frames": [frames_f, frames_w],
        "per_kernel_per_frame": dict(per),
        "FETCH_SIZE_KiB_per_frame": fk,
        "WRITE_SIZE_KiB_per_frame": wk,
        "hbm_bytes_per_frame": (2.0 * fk + wk) * 1024.0,
        "hbm_bytes_per_frame_raw": (fk + wk) * 1024.0,
        "correction": "FETCH_SIZE x2 (gfx950, MI355X_MICROARCH.md HBM section); raw sum kept beside it",
    }
    db = {}
    if os.path.exists(out):
        with open(out) as fh:
            db = json.load(fh)
    db[key] = entry
    with open(out, "w") as fh:
        json.dump(db, fh, indent=1, sort_keys=True)
    print(json.dumps({key: entry}, indent=1))


if __name__ == "__main__":
    main()
