"""Timeline of back-to-back frames from a rocprofv3 --kernel-trace CSV.

usage: python tools/timeline.py <kernel_trace.csv> [first_k_vis_index] [frames]

Prints every kernel (and copy) of `frames` consecutive frames, counted from
the first_k_vis_index-th k_vis launch: start offset (us) from that k_vis,
duration, and the fraction of the window with at least one kernel running
(GPU busy) — the gaps are what the host, events and launch latency cost.
"""
import csv
import sys


def main():
    path = sys.argv[1]
    k0 = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    nf = int(sys.argv[3]) if len(sys.argv) > 3 else 3
    rows = []
    for r in csv.DictReader(open(path)):
        name = r.get("Kernel_Name") or r.get("Name") or "?"
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), name.split("(")[0][-40:]))
    rows.sort()
    vis = [i for i, r in enumerate(rows) if "k_vis" in r[2]]
    if len(vis) <= k0 + nf:
        print("not enough frames: %d k_vis launches" % len(vis))
        return
    t0 = rows[vis[k0]][0]
    t1 = rows[vis[k0 + nf]][0]
    win = [r for r in rows if t0 - 200_000 <= r[0] < t1]
    for s, e, n in win:
        print("%9.1f %8.1f  %s" % ((s - t0) / 1e3, (e - s) / 1e3, n))
    # busy union inside [t0, t1)
    busy, cur_s, cur_e = 0, None, None
    for s, e, _ in sorted(r for r in rows if r[1] > t0 and r[0] < t1):
        s, e = max(s, t0), min(e, t1)
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                busy += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    if cur_e is not None:
        busy += cur_e - cur_s
    span = t1 - t0
    print("window %.1f us = %d frames (%.1f us/frame), GPU busy %.1f %%" % (span / 1e3, nf, span / 1e3 / nf,
                                                                           100.0 * busy / span))


if __name__ == "__main__":
    main()
