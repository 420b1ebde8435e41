#!/usr/bin/env python3
"""Sum rocprofv3 --pmc counter_collection.csv files per counter (per kernel
dispatch rows are summed; the number of dispatches is printed beside)."""
import collections
import csv
import glob
import sys

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc"
for f in sorted(glob.glob(f"{root}/**/*counter_collection.csv", recursive=True)):
    agg, disp = collections.defaultdict(float), collections.defaultdict(set)
    for r in csv.DictReader(open(f)):
        agg[r["Counter_Name"]] += float(r["Counter_Value"])
        disp[r["Counter_Name"]].add(r.get("Dispatch_Id", ""))
    print(f)
    for k in sorted(agg):
        print(f"  {k:28s} {agg[k]:20.1f}   dispatches={len(disp[k])}")
