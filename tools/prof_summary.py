"""rocprofv3 --kernel-trace --stats rocpd database -> per-kernel stats CSV
(the same columns as rocprofv3's kernel_stats.csv, plus ms per step).

usage: python tools/prof_summary.py <run_results.db> <out.csv> <steps-in-run>"""
import csv
import sqlite3
import sys

db, out, steps = sys.argv[1], sys.argv[2], int(sys.argv[3])
c = sqlite3.connect(db)
rows = c.execute("select name, count(*), sum(end - start), avg(end - start), min(end - start), "
                 "max(end - start) from kernels group by name order by sum(end - start) desc").fetchall()
tot = sum(r[2] for r in rows)
with open(out, "w", newline="") as f:
    wr = csv.writer(f)
    wr.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "MinNs", "MaxNs", "Percentage",
                 "MsPerStep"])
    for name, n, s, a, mn, mx in rows:
        wr.writerow([name, n, s, round(a, 1), mn, mx, round(100.0 * s / tot, 3),
                     round(s / steps / 1e6, 4)])
print(f"{len(rows)} kernels, {tot / steps / 1e6:.3f} ms GPU time per step")
for name, n, s, a, *_ in rows[:12]:
    print(f"{s / steps / 1e6:8.3f} ms/step  {n:5d} x {a / 1e3:8.1f} us  {name[:110]}")
