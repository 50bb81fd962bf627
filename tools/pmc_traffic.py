"""Summarise rocprofv3 PMC passes into profiles/pmc_traffic.json.

Usage (on the GPU box, two separate passes as MI355X_MICROARCH.md prescribes:
FETCH_SIZE and WRITE_SIZE do not fit one TCC pass):
    rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d D -o fetch -- python3 bench.py ...
    rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d D -o write -- python3 bench.py ...
    python tools/pmc_traffic.py D <config-key> [out.json]

Per frame, summed over the raster stage's kernels (k_vis, k_walk, k_pix):
FETCH_SIZE and WRITE_SIZE are in KiB.  gfx950 correction (MI355X_MICROARCH.md
§HBM): FETCH_SIZE reports half the bytes of a read, so the read side is
doubled; WRITE_SIZE is taken as is.  The guide calibrates both only for
16-B/lane streams, so the raw sum is kept next to the corrected total.
"""
import csv
import glob
import json
import os
import sys


def per_launch(d, counter, kernel_substr):
    vals = []
    for p in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(p) as f:
            for r in csv.DictReader(f):
                if r.get("Counter_Name") != counter:
                    continue
                if kernel_substr not in r.get("Kernel_Name", ""):
                    continue
                vals.append(float(r["Counter_Value"]))
    return vals


STAGE = ("k_vis", "k_walk", "k_pix")  # the raster stage of an AVX frame


def main():
    d = sys.argv[1]
    key = sys.argv[2]
    out = sys.argv[3] if len(sys.argv) > 3 else os.path.join(os.path.dirname(os.path.dirname(
        os.path.abspath(__file__))), "profiles", "pmc_traffic.json")
    per = {}
    for k in STAGE:
        fetch = per_launch(d, "FETCH_SIZE", k + "<")
        write = per_launch(d, "WRITE_SIZE", k + "<")
        if not fetch or not write:
            print("no %s FETCH_SIZE/WRITE_SIZE rows found under %s" % (k, d))
            sys.exit(1)
        # Skip the first (warm-up / cold-cache) launch when there are several.
        f = fetch[1:] if len(fetch) > 2 else fetch
        w = write[1:] if len(write) > 2 else write
        per[k] = {"launches": [len(fetch), len(write)], "FETCH_SIZE_KiB": sum(f) / len(f),
                  "WRITE_SIZE_KiB": sum(w) / len(w)}
    fk = sum(v["FETCH_SIZE_KiB"] for v in per.values())
    wk = sum(v["WRITE_SIZE_KiB"] for v in per.values())
    entry = {
        "kernel": "raster stage (" + "+".join(STAGE) + ")",
        "per_kernel": per,
        "FETCH_SIZE_KiB": fk,
        "WRITE_SIZE_KiB": wk,
        # MI355X_MICROARCH.md §HBM: on gfx950 FETCH_SIZE reports half the
        # bytes of a read, so it is doubled; WRITE_SIZE is taken as is.
        "hbm_bytes_per_launch": (2.0 * fk + wk) * 1024.0,
        "hbm_bytes_per_launch_raw": (fk + wk) * 1024.0,
        "correction": "FETCH_SIZE x2 (gfx950, MI355X_MICROARCH.md HBM section); raw sum kept beside it",
    }
    db = {}
    if os.path.exists(out):
        with open(out) as fh:
            db = json.load(fh)
    db[key] = entry
    with open(out, "w") as fh:
        json.dump(db, fh, indent=1, sort_keys=True)
    print(json.dumps({key: entry}))


if __name__ == "__main__":
    main()
