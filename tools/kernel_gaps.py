"""Per-kernel mean durations and the last dispatches with the gaps between them, from a rocprofv3
--kernel-trace CSV (diagnostic tool).   python tools/kernel_gaps.py <kernel_trace.csv> [n_last]"""
import csv
import sys
from collections import defaultdict


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    n_last = int(sys.argv[2]) if len(sys.argv) > 2 else 16
    ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
    agg = defaultdict(list)
    for s, e, n in ev:
        agg[n].append((e - s) / 1e3)
    print("%-72s %6s %9s" % ("kernel", "calls", "mean_us"))
    for n, d in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
        print("%-72s %6d %9.2f" % (n[:72], len(d), sum(d) / len(d)))
    print("\nlast %d dispatches: start offset, duration, gap before (us)" % n_last)
    tail = ev[-n_last:]
    t0 = tail[0][0]
    prev = None
    for s, e, n in tail:
        gap = (s - prev) / 1e3 if prev is not None else 0.0
        print("%9.1f %8.2f %8.2f  %s" % ((s - t0) / 1e3, (e - s) / 1e3, gap, n[:80]))
        prev = e


if __name__ == "__main__":
    main()
