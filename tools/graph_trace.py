"""Graph-replay kernel trace of bench.py (rocprofv3 --kernel-trace rocpd
database) -> does the sum of the replayed kernels account for ms_per_step?

Steps are cut at every `distort_draw_kernel` dispatch (the first kernel of a
bench step: the per-image distortion draws, 14:31-64).  For the last N
complete steps it reports the kernel-time sum per step, the union of the
kernel intervals (the GPU-busy time: side-stream kernels overlap the main
stream's, so the plain sum exceeds the wall time), the wall span per
step (first start -> next step's first start), the idle share, the per-family
sums and -- for one median step -- every dispatch in order with its
duration (the layer a conv launch serves follows from its place in the
schedule, engine.py).

usage: python tools/graph_trace.py <results.db> <out.json> [steps]"""
import json
import re
import sqlite3
import statistics
import sys

db, out = sys.argv[1], sys.argv[2]
nsteps = int(sys.argv[3]) if len(sys.argv) > 3 else 10
c = sqlite3.connect(db)
rows = c.execute("select name, start, end from kernels order by start").fetchall()
marks = [i for i, r in enumerate(rows) if r[0].startswith("distort_draw_kernel")]
if len(marks) < 3:
    raise SystemExit(f"only {len(marks)} step markers in {len(rows)} dispatches")
steps = []
for a, b in zip(marks[:-1], marks[1:]):
    steps.append(rows[a:b])
steps = steps[-nsteps:]


def fam(name):
    n = re.sub(r"^void ", "", name)
    n = re.sub(r"\(anonymous namespace\)::", "", n)
    return n.split("(")[0]


def busy(st):
    """union of the step's kernel intervals (kernels on the side streams
    overlap the main stream's: their durations sum past the wall time)"""
    iv = sorted((s, e) for _, s, e in st)
    tot, cs, ce = 0, iv[0][0], iv[0][1]
    for s, e in iv[1:]:
        if s > ce:
            tot += ce - cs
            cs, ce = s, e
        else:
            ce = max(ce, e)
    return tot + ce - cs


per = []
for st in steps:
    ksum = sum(e - s for _, s, e in st)
    per.append((ksum, st))
unions = [busy(st) for st in steps]
walls = []
for i in range(len(steps) - 1):
    walls.append(steps[i + 1][0][1] - steps[i][0][1])
med = sorted(per, key=lambda p: p[0])[len(per) // 2]
fams = {}
for name, s, e in med[1]:
    f = fams.setdefault(fam(name), [0, 0.0])
    f[0] += 1
    f[1] += (e - s) / 1e6
gaps = [med[1][i + 1][1] - med[1][i][2] for i in range(len(med[1]) - 1)]
res = {
    "db": db, "steps": len(steps), "dispatches_per_step": len(med[1]),
    "kernel_ms_per_step": [round(k / 1e6, 4) for k, _ in per],
    "wall_ms_per_step": [round(w / 1e6, 4) for w in walls],
    "median_kernel_ms": round(statistics.median(k for k, _ in per) / 1e6, 4),
    "busy_union_ms_per_step": [round(u / 1e6, 4) for u in unions],
    "median_busy_union_ms": round(statistics.median(unions) / 1e6, 4),
    "median_wall_ms": round(statistics.median(walls) / 1e6, 4) if walls else None,
    "median_step_gap_ms": round(sum(g for g in gaps if g > 0) / 1e6, 4),
    "median_step_overlap_ms": round(-sum(g for g in gaps if g < 0) / 1e6, 4),
    "families_ms": {k: {"launches": v[0], "ms": round(v[1], 4)}
                    for k, v in sorted(fams.items(), key=lambda kv: -kv[1][1])},
    "dispatches": [[fam(n), round((e - s) / 1e3, 2)] for n, s, e in med[1]],
}
json.dump(res, open(out, "w"), indent=1)
print(f"{len(steps)} steps: kernel {res['median_kernel_ms']} ms/step (union of intervals "
      f"{res['median_busy_union_ms']}), wall {res['median_wall_ms']} ms/step, "
      f"gaps {res['median_step_gap_ms']} ms, overlap {res['median_step_overlap_ms']} ms, "
      f"{len(med[1])} dispatches")
for k, v in list(res["families_ms"].items())[:15]:
    print(f"  {v['ms']:8.3f} ms  {v['launches']:4d}  {k[:100]}")
