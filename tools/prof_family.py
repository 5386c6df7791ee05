"""kernel-stats CSV (tools/prof_summary.py) -> ms/step per kernel family
(template name without arguments).  usage: python tools/prof_family.py <csv> [top]"""
import csv
import re
import sys

fam = {}
for r in csv.DictReader(open(sys.argv[1])):
    n = re.sub(r"^void ", "", r["Name"])
    n = n.replace("(anonymous namespace)::", "")
    k = re.split(r"[<(]", n)[0]
    fam[k] = fam.get(k, 0.0) + float(r["MsPerStep"])
top = int(sys.argv[2]) if len(sys.argv) > 2 else 30
for k, v in sorted(fam.items(), key=lambda x: -x[1])[:top]:
    print(f"{v:7.3f}  {k}")
print(f"{sum(fam.values()):7.3f}  total")
