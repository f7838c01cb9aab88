"""Aggregate a rocprofv3 --pmc counter CSV per kernel-name prefix: sum of each counter over the dispatches whose
name contains the filter, and the dispatch count.  Usage: pmc_agg.py <dir> <name-substring>"""
import csv
import glob
import json
import sys
from collections import defaultdict

d, filt = sys.argv[1], sys.argv[2]
tot, disp = defaultdict(float), set()
for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if filt in r["Kernel_Name"]:
            tot[r["Counter_Name"]] += float(r["Counter_Value"])
            disp.add(r["Dispatch_Id"])
n = max(len(disp), 1)
print(json.dumps({"filter": filt, "dispatches": len(disp), "per_dispatch": {k: round(v / n, 1) for k, v in sorted(tot.items())}}))
