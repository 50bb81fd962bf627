"""Summarise rocprofv3 PMC passes into profiles/pmc_traffic.json.

Usage (on the GPU box, two separate passes as MI355X_MICROARCH.md prescribes:
FETCH_SIZE and WRITE_SIZE do not fit one TCC pass):
    rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d D -o fetch -- python3 bench.py ...
    rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d D -o write -- python3 bench.py ...
    python tools/pmc_traffic.py D <config-key> [out.json]

Per k_raster launch: FETCH_SIZE and WRITE_SIZE are in KiB.  gfx950
correction (MI355X_MICROARCH.md §HBM): FETCH_SIZE reports half the bytes of a
wide coalesced streaming read, so the read side is doubled; WRITE_SIZE is
exact for 16-B/lane streaming stores.  Both are uncalibrated for other access
widths, so the raw values are kept next to the corrected total.
"""
import csv
import glob
import json
import os
import sys


def per_launch(d, counter, kernel_substr="k_raster"):
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


def main():
    d = sys.argv[1]
    key = sys.argv[2]
    out = sys.argv[3] if len(sys.argv) > 3 else os.path.join(os.path.dirname(os.path.dirname(
        os.path.abspath(__file__))), "profiles", "pmc_traffic.json")
    fetch = per_launch(d, "FETCH_SIZE")
    write = per_launch(d, "WRITE_SIZE")
    if not fetch or not write:
        print("no k_raster FETCH_SIZE/WRITE_SIZE rows found under", d)
        sys.exit(1)
    # Skip the first (warm-up / cold-cache) launch when there are several.
    f = fetch[1:] if len(fetch) > 2 else fetch
    w = write[1:] if len(write) > 2 else write
    fk = sum(f) / len(f)
    wk = sum(w) / len(w)
    entry = {
        "kernel": "k_raster",
        "launches": [len(fetch), len(write)],
        "FETCH_SIZE_KiB": fk,
        "WRITE_SIZE_KiB": wk,
        # k_raster's reads are 4-16 B gathers, not the 16-B/lane streams the
        # guide's x2 FETCH correction is calibrated for; the raw total matches
        # the expected re-read volume, so it is the one reported.
        "hbm_bytes_per_launch": (fk + wk) * 1024.0,
        "hbm_bytes_per_launch_fetch_x2": (2.0 * fk + wk) * 1024.0,
        "correction": "none applied (narrow gathers); fetch_x2 = guide's wide-stream correction",
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
