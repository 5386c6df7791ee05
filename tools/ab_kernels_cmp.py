"""Compare per-kernel average durations of tools/ab_kernels.sh runs.

usage: python tools/ab_kernels_cmp.py [substring ...]   (kernels whose name contains any)"""
import glob
import os
import sqlite3
import sys
from collections import defaultdict


def stats(db):
    c = sqlite3.connect(db)
    return {n: (cnt, s / cnt) for n, cnt, s in
            c.execute("select name, count(*), sum(end - start) from kernels group by name")}


runs = defaultdict(list)
for d in sorted(glob.glob("gpurun_out/abk/*_*")):
    if os.path.isdir(d):
        dbs = glob.glob(os.path.join(d, "**", "*results.db"), recursive=True)
        if dbs:
            runs[os.path.basename(d).rsplit("_", 1)[0]].append(stats(dbs[0]))
subs = sys.argv[1:]
names = sorted({n for r in runs["cur"] for n in r})
tot = {"cur": 0.0, "other": 0.0}
for n in names:
    if subs and not any(s in n for s in subs):
        continue
    av = {}
    for L in ("cur", "other"):
        v = [r[n][1] for r in runs[L] if n in r]
        av[L] = sum(v) / len(v) if v else float("nan")
        tot[L] += sum(r[n][0] * r[n][1] for r in runs[L] if n in r) / max(len(runs[L]), 1)
    print(f"{av['cur'] / 1e3:9.1f} us  {av['other'] / 1e3:9.1f} us  {av['cur'] / av['other']:6.3f}  "
          f"{n.replace('(anonymous namespace)::', '')[:90]}")
print(f"total (selected, per run): cur {tot['cur'] / 1e6:.3f} ms, other {tot['other'] / 1e6:.3f} ms")
