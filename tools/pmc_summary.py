#!/usr/bin/env python3
"""Summarise rocprofv3 PMC csv passes under a profile dir: per rc_* kernel, mean per dispatch."""
import collections
import csv
import glob
import json
import sys

d = sys.argv[1]
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in sorted(glob.glob(f"{d}/pmc*/run_counter_collection.csv")):
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in csv.DictReader(open(f)):
        if r["Kernel_Name"].startswith("rc_"):
            per[(r["Kernel_Name"], r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
    for (k, _), cs in per.items():
        for c, v in cs.items():
            agg[k][c].append(v)
out = {k: {c: sum(v) / len(v) for c, v in cs.items()} for k, cs in agg.items()}
print(json.dumps(out, indent=1))
