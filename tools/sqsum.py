"""Summarise rocprofv3 SQ counter CSVs per kernel (mean over launches).

Units (MI355X_MICROARCH.md, per-instruction constants row 's_memtime tick vs
SQ PMC units'): SQ_WAVE_CYCLES, SQ_WAIT_* and SQ_ACTIVE_INST_* count
quad-cycles, summed over every wave of the dispatch (all XCDs).  The VALU-time
estimate spreads SQ_ACTIVE_INST_VALU x 4 cycles over the chip's 1024 SIMDs at
2.4 GHz (an upper estimate: co-resident waves of one SIMD interleave their
VALU issue, so per-wave active cycles can add up to more than the SIMD's);
the issue floor prices SQ_INSTS_VALU at the SIMD's full rate, one wave64
VALU instruction per 2 cycles (v_fma_f32 throughput, MI355X_MICROARCH.md
constants table; transcendentals are slower).  A VALU-bound kernel's
duration lies between the two."""
import collections
import csv
import glob
import sys

args = sys.argv[1:]
json_out = None  # --json OUT KEY ROUND: per-kernel VALU figures into OUT[KEY] (bench.py roofline.valu)
if "--json" in args:
    i = args.index("--json")
    json_out = args[i + 1:i + 4]
    del args[i:i + 4]
d = args[0] if len(args) > 0 else "gpurun_out/sq"
csv_out = args[1] if len(args) > 1 else None  # optional compact CSV: kernel,counter,mean
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for p in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(p)):
        k = r["Kernel_Name"]
        if "k_" not in k:
            continue
        k = k.split("(")[0].replace("void prk::", "")
        acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, cs in acc.items():
    print(k)
    m = {c: sum(v) / len(v) for c, v in cs.items()}
    for c in sorted(m):
        print("   %-24s %16.0f" % (c, m[c]))
    if "SQ_THREAD_CYCLES_VALU" in m and "SQ_ACTIVE_INST_VALU" in m and m["SQ_ACTIVE_INST_VALU"]:
        print("   lane utilisation (THREAD_CYCLES_VALU / (64*ACTIVE_INST_VALU)) = %.3f"
              % (m["SQ_THREAD_CYCLES_VALU"] / (64 * m["SQ_ACTIVE_INST_VALU"])))
    if "SQ_ACTIVE_INST_VALU" in m:
        print("   VALU-time estimate (ACTIVE_INST_VALU*4 / 1024 SIMDs / 2.4 GHz) = %.3f ms"
              % (m["SQ_ACTIVE_INST_VALU"] * 4 / 1024 / 2.4e6))
    if "SQ_INSTS_VALU" in m:
        print("   VALU issue floor (INSTS_VALU*2 / 1024 SIMDs / 2.4 GHz)       = %.3f ms"
              % (m["SQ_INSTS_VALU"] * 2 / 1024 / 2.4e6))
    if "SQ_WAVE_CYCLES" in m and m["SQ_WAVE_CYCLES"]:
        for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
            if c in m:
                print("   %s / WAVE_CYCLES = %.3f" % (c, m[c] / m["SQ_WAVE_CYCLES"]))
if csv_out:
    with open(csv_out, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["kernel", "counter", "mean_per_dispatch", "dispatches"])
        for k, cs in sorted(acc.items()):
            for c, v in sorted(cs.items()):
                w.writerow([k, c, sum(v) / len(v), len(v)])
if json_out:
    import json
    import os
    out, key, rnd = json_out
    kern = {}
    for k, cs in acc.items():
        m = {c: sum(v) / len(v) for c, v in cs.items()}
        e = {"dispatches": len(next(iter(cs.values())))}
        if m.get("SQ_ACTIVE_INST_VALU"):
            e["valu_time_estimate_ms"] = m["SQ_ACTIVE_INST_VALU"] * 4 / 1024 / 2.4e6
            if "SQ_THREAD_CYCLES_VALU" in m:
                e["lane_utilisation"] = m["SQ_THREAD_CYCLES_VALU"] / (64 * m["SQ_ACTIVE_INST_VALU"])
        if "SQ_INSTS_VALU" in m:
            e["valu_issue_floor_ms"] = m["SQ_INSTS_VALU"] * 2 / 1024 / 2.4e6
            e["insts_valu"] = m["SQ_INSTS_VALU"]
        if m.get("SQ_WAVE_CYCLES"):
            e["wait_any_frac"] = m.get("SQ_WAIT_ANY", 0.0) / m["SQ_WAVE_CYCLES"]
        kern[k] = e
    db = {}
    if os.path.exists(out):
        with open(out) as fh:
            db = json.load(fh)
    db[key] = {"round": rnd, "source": d, "per_kernel": kern,
               "method": "rocprofv3 --pmc SQ counters (two passes), mean per dispatch; VALU-time estimate = "
                         "SQ_ACTIVE_INST_VALU*4/1024 SIMDs/2.4 GHz, lane utilisation = "
                         "SQ_THREAD_CYCLES_VALU/(64*SQ_ACTIVE_INST_VALU)"}
    with open(out, "w") as fh:
        json.dump(db, fh, indent=1, sort_keys=True)
