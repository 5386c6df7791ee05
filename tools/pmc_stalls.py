"""Per-kernel stall profile from one rocprofv3 --kernel-trace --pmc pass with
SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY
SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT
SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE (MI355X_MICROARCH.md 'rocprofv3 PMC slots'):
wave-cycle shares parked at waitcnt/barrier, issue-stalled, issuing;
MFMA-busy fraction; LDS bank-conflict share; effective clock.

usage: python tools/pmc_stalls.py <results.db> [out.json]"""
import json
import re
import sqlite3
import sys

SIMDS = 4 * 256
c = sqlite3.connect(sys.argv[1])
dur = {did: e - s for did, s, e in c.execute("select dispatch_id, start, end from kernels")}
per = {}
for name, cn, v, did in c.execute("select kernel_name, counter_name, value, dispatch_id "
                                  "from counters_collection"):
    d = per.setdefault(name, {}).setdefault(did, {})
    d[cn] = d.get(cn, 0.0) + v
out = {}
for name, disp in per.items():
    n = len(disp)
    keys = set().union(*[d.keys() for d in disp.values()])
    avg = {k: sum(d.get(k, 0.0) for d in disp.values()) / n for k in keys}
    ns = [dur[k] for k in disp if k in dur]
    r = {"launches": n, "avg_us": round(sum(ns) / len(ns) / 1e3, 1) if ns else None}
    wc = avg.get("SQ_WAVE_CYCLES", 0)
    if wc:
        for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_LDS"):
            if k in avg:
                r[k.replace("SQ_", "").lower() + "_share"] = round(avg[k] / wc, 3)
    cyc = avg.get("GRBM_GUI_ACTIVE", 0) / 8
    if cyc and "SQ_VALU_MFMA_BUSY_CYCLES" in avg:
        r["mfma_busy"] = round(avg["SQ_VALU_MFMA_BUSY_CYCLES"] / (SIMDS * cyc), 3)
    if ns and cyc:
        r["clock_ghz"] = round(cyc / (sum(ns) / len(ns)), 3)
    if avg.get("SQ_LDS_IDX_ACTIVE"):
        r["lds_conflict_share"] = round(avg.get("SQ_LDS_BANK_CONFLICT", 0) / avg["SQ_LDS_IDX_ACTIVE"], 3)
        r["lds_active_per_cu_cycle"] = round(avg["SQ_LDS_IDX_ACTIVE"] / (256 * cyc), 3) if cyc else None
    m = re.search(r"(\w+<[^(]*>)\(", name) or re.search(r"(\w+)\(", name)
    out[(m.group(1) if m else name)] = r
for k, v in out.items():
    print(k, json.dumps(v))
if len(sys.argv) > 2:
    json.dump(out, open(sys.argv[2], "w"), indent=1)
