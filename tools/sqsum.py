"""Summarise tools/sqprof.sh counter CSVs per kernel (mean over launches)."""
import collections
import csv
import glob
import sys

d = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/sq"
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
    if "SQ_WAVE_CYCLES" in m and m["SQ_WAVE_CYCLES"]:
        for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
            if c in m:
                print("   %s / WAVE_CYCLES = %.3f" % (c, m[c] / m["SQ_WAVE_CYCLES"]))
