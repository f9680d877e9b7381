"""Per-dispatch means of every PMC counter for kernels whose name contains a filter
(rocprofv3 --pmc csv under DIR): python tools/pmc_table.py DIR [filter]"""
import collections
import csv
import glob
import os
import sys

d, flt = sys.argv[1], (sys.argv[2] if len(sys.argv) > 2 else "")
rows = []
for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
    with open(f) as fh:
        rows += list(csv.DictReader(fh))
acc = collections.defaultdict(lambda: collections.defaultdict(float))
disp = collections.defaultdict(set)
for r in rows:
    k = r.get("Kernel_Name", "")
    if flt not in k:
        continue
    acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
    disp[k].add(r.get("Dispatch_Id"))
for k, c in acc.items():
    n = max(1, len(disp[k]))
    print(f"{os.path.basename(d)} {k[:70]} dispatches={n}")
    for name, v in sorted(c.items()):
        print(f"   {name:28s} {v / n:16.1f}")
