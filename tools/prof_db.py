"""Summarise a rocprofv3 results database (rocpd sqlite, the ROCm 7 default output): per-kernel count /
mean / total duration (the --stats table), and the sequence + gaps of the last N dispatches.
    python tools/prof_db.py <run_results.db> [n_tail]"""
import sqlite3
import sys

con = sqlite3.connect(sys.argv[1])
rows = con.execute("select name, start, end from kernels order by start").fetchall()
stats = {}
for n, s, e in rows:
    d = stats.setdefault(n, [0, 0.0])
    d[0] += 1
    d[1] += (e - s) / 1e3
tot = sum(v[1] for v in stats.values())
print("%-70s %6s %10s %10s %6s" % ("kernel", "calls", "mean_us", "total_us", "pct"))
for n, (c, t) in sorted(stats.items(), key=lambda kv: -kv[1][1])[:25]:
    print("%-70s %6d %10.2f %10.1f %6.1f" % (n[:70], c, t / c, t, 100 * t / tot))
k = int(sys.argv[2]) if len(sys.argv) > 2 else 0
if k:
    print("\nlast %d dispatches: start offset, duration, gap before (us)" % k)
    tail = rows[-k:]
    t0 = tail[0][1]
    prev = None
    for n, s, e in tail:
        gap = (s - prev) / 1e3 if prev is not None else 0.0
        print("%9.1f %8.2f %8.2f  %s" % ((s - t0) / 1e3, (e - s) / 1e3, gap, n[:80]))
        prev = e
