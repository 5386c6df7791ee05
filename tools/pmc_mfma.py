"""Per-kernel MFMA utilisation from one rocprofv3 PMC pass
(--kernel-trace --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES
SQ_INSTS_MFMA GRBM_GUI_ACTIVE) of the bench (tools/profile_round.sh):

  mfma_busy_frac = SQ_VALU_MFMA_BUSY_CYCLES / (4 SIMDs x 256 CUs x cycles),
  cycles = GRBM_GUI_ACTIVE / 8 (rocprofv3 sums it over the 8 XCDs),
  clock  = cycles / kernel duration (the DVFS-held clock under this load),

MI355X_MICROARCH.md: SQ_VALU_MFMA_BUSY_CYCLES counts cycles (16 per
v_mfma_f32_16x16x32_bf16), GRBM_GUI_ACTIVE / 8 / wall = effective clock
(reads high on dispatches shorter than ~0.3 ms).

usage: python tools/pmc_mfma.py <results.db> <out.json>"""
import json
import re
import sqlite3
import sys

SIMDS = 4 * 256
COUNTERS = ("SQ_VALU_MFMA_BUSY_CYCLES", "SQ_BUSY_CYCLES", "SQ_WAVE_CYCLES", "SQ_INSTS_MFMA",
            "GRBM_GUI_ACTIVE")


def short(name):
    m = re.search(r"::(\w+)<([^(]*)>\(", name) or re.search(r"(\w+)\(", name)
    return m.group(0).rstrip("(") if m else name


c = sqlite3.connect(sys.argv[1])
cols = [r[1] for r in c.execute("pragma table_info(counters_collection)")]
rows = c.execute("select kernel_name, counter_name, value, dispatch_id from counters_collection").fetchall()
dur = {}
try:
    for did, s, e in c.execute("select dispatch_id, start, end from kernels"):
        dur[did] = e - s
except sqlite3.Error:
    pass
per = {}
for name, cn, v, did in rows:
    d = per.setdefault(name, {}).setdefault(did, {})
    d[cn] = d.get(cn, 0.0) + v
out = {}
for name, disp in per.items():
    n = len(disp)
    avg = {k: sum(d.get(k, 0.0) for d in disp.values()) / n for k in COUNTERS}
    ns = [dur[k] for k in disp if k in dur]
    cyc = avg["GRBM_GUI_ACTIVE"] / 8
    r = {"launches": n, **{k: round(v) for k, v in avg.items()}, "name": name}
    if cyc > 0:
        r["mfma_busy_frac"] = round(avg["SQ_VALU_MFMA_BUSY_CYCLES"] / (SIMDS * cyc), 4)
    if ns and cyc > 0:
        r["avg_ns"] = round(sum(ns) / len(ns))
        r["clock_ghz"] = round(cyc / (sum(ns) / len(ns)), 3)
    out[short(name)] = r
key = lambda kv: -kv[1].get("SQ_VALU_MFMA_BUSY_CYCLES", 0) * kv[1]["launches"]
json.dump(dict(sorted(out.items(), key=key)), open(sys.argv[2], "w"), indent=1)
for k, v in sorted(out.items(), key=key)[:16]:
    print(f"{v.get('mfma_busy_frac', 0):7.3f} mfma-busy  {v.get('clock_ghz', 0):5.2f} GHz  "
          f"{v.get('avg_ns', 0) / 1e3:8.1f} us  x{v['launches']:3d}  {k}")
