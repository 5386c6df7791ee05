"""Per-kernel HBM traffic from two rocprofv3 PMC passes (FETCH_SIZE and
WRITE_SIZE collected in separate runs, --kernel-trace only), corrected as
MI355X_MICROARCH.md prescribes for gfx950: FETCH_SIZE reports 1/2 of the bytes
of wide coalesced reads -> x2; WRITE_SIZE exact for 16-B stores.  Units: the
counters are KiB per dispatch.

usage: python tools/pmc_traffic.py <fetch.db> <write.db> <out.json>"""
import json
import re
import sqlite3
import sys


def per_kernel(db, counter):
    c = sqlite3.connect(db)
    rows = c.execute("select kernel_name, value from counters_collection where counter_name = ?",
                     (counter,)).fetchall()
    agg = {}
    for name, v in rows:
        a = agg.setdefault(name, [0, 0.0])
        a[0] += 1
        a[1] += v
    return agg


def short(name):
    m = re.search(r"::(\w+)<([^(]*)>\(", name) or re.search(r"(\w+)\(", name)
    return m.group(0).rstrip("(") if m else name


f = per_kernel(sys.argv[1], "FETCH_SIZE")
w = per_kernel(sys.argv[2], "WRITE_SIZE")
out = {}
for name in set(f) | set(w):
    nf, kf = f.get(name, (0, 0.0))
    nw, kw = w.get(name, (0, 0.0))
    if not nf or not nw:
        continue
    fetch = kf / nf * 1024 * 2          # gfx950 correction
    write = kw / nw * 1024
    out[short(name)] = {"launches_per_pass": nf, "fetch_bytes_per_launch": round(fetch),
                        "write_bytes_per_launch": round(write),
                        "hbm_bytes_per_launch": round(fetch + write),
                        "fetch_size_kib_raw_avg": round(kf / nf, 3), "name": name}
json.dump(dict(sorted(out.items(), key=lambda kv: -kv[1]["hbm_bytes_per_launch"])),
          open(sys.argv[3], "w"), indent=1)
for k, v in sorted(out.items(), key=lambda kv: -kv[1]["hbm_bytes_per_launch"])[:12]:
    print(f"{v['hbm_bytes_per_launch'] / 1e6:10.1f} MB/launch  (fetch {v['fetch_bytes_per_launch'] / 1e6:8.1f}, "
          f"write {v['write_bytes_per_launch'] / 1e6:8.1f})  {k}")
