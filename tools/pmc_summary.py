"""Summarise rocprofv3 --pmc CSV passes per kernel: sum of each counter and
the kernel's total duration, plus per-dispatch averages."""
import collections
import csv
import glob
import os
import sys

root = sys.argv[1]
agg = collections.defaultdict(lambda: collections.defaultdict(float))
disp = collections.defaultdict(set)
dur = collections.defaultdict(dict)
for f in sorted(glob.glob(os.path.join(root, "p*", "**", "*counter_collection.csv"), recursive=True)):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0]
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
        key = (f, r["Dispatch_Id"])
        disp[(k, r["Counter_Name"])].add(key)
        try:
            dur[k][key] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        except (KeyError, ValueError):
            pass
for k, cs in agg.items():
    if k.startswith("__amd"):
        continue
    print(f"== {k}")
    for c, v in sorted(cs.items()):
        nd = len(disp[(k, c)])
        print(f"   {c:28s} total {v:16.4g}   per-dispatch {v / max(1, nd):14.4g}  ({nd} dispatches)")
