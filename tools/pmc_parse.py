"""Sum rocprofv3 --pmc counter_collection CSVs per counter (mean over the
dispatches of a kernel-name substring).  usage: pmc_parse.py DIR [substr]"""
import csv, collections, glob, sys
d = sys.argv[1]
sub = sys.argv[2] if len(sys.argv) > 2 else "stream3"
for f in sorted(glob.glob(f"{d}/**/*counter_collection.csv", recursive=True)):
    agg = collections.defaultdict(float)
    for r in csv.DictReader(open(f)):
        if sub in r["Kernel_Name"]:
            agg[(r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"])
    per = collections.defaultdict(list)
    for (_, cn), v in agg.items():
        per[cn].append(v)
    for cn, v in sorted(per.items()):
        print(f"{cn:28s} {sum(v) / len(v):16.1f}  (n={len(v)})")
