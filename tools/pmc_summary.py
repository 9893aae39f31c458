#!/usr/bin/env python3
"""Average PMC counters per kernel (per dispatch) from rocprofv3 counter_collection CSVs."""
import collections
import csv
import glob
import sys

agg = collections.defaultdict(lambda: collections.defaultdict(float))
disp = collections.defaultdict(set)
for d in sys.argv[1:]:
    for f in glob.glob(f"{d}/*counter_collection.csv"):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].split("(")[0][:100]
            agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
            disp[(k, r["Counter_Name"])].add(r["Dispatch_Id"])
for k, v in agg.items():
    if "niti" not in k:
        continue
    print(k)
    for c, x in sorted(v.items()):
        print(f"    {c:40s} {x / max(1, len(disp[(k, c)])):16.0f}")
