"""Per-kernel averages of rocprofv3 --pmc counter CSVs: python3 tools/sq_table.py DIR [kernel-substring...]"""
import csv
import glob
import sys
from collections import defaultdict

d = sys.argv[1]
pats = sys.argv[2:] or [""]
acc = defaultdict(lambda: defaultdict(list))
for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
    per = defaultdict(float)
    names = {}
    for r in csv.DictReader(open(f)):
        key = (r["Dispatch_Id"], r["Counter_Name"])
        per[key] += float(r["Counter_Value"])
        names[r["Dispatch_Id"]] = r["Kernel_Name"]
    for (disp, c), v in per.items():
        acc[names[disp]][c].append(v)
for k, cs in acc.items():
    if not any(p in k for p in pats):
        continue
    print(k[:90])
    for c in sorted(cs):
        vals = cs[c]
        print(f"   {c:28s} {sum(vals) / len(vals):16.4g}")
