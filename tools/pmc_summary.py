#!/usr/bin/env python3
"""Sum rocprofv3 --pmc counter_collection.csv files per (kernel, counter): the
per-dispatch rows of one kernel are summed; the dispatch count is printed
beside."""
import collections
import csv
import glob
import sys

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc"
for f in sorted(glob.glob(f"{root}/**/*counter_collection.csv", recursive=True)):
    agg, disp = collections.defaultdict(float), collections.defaultdict(set)
    for r in csv.DictReader(open(f)):
        k = (r.get("Kernel_Name", "?").split("(")[0][-40:], r["Counter_Name"])
        agg[k] += float(r["Counter_Value"])
        disp[k].add(r.get("Dispatch_Id", ""))
    print(f)
    for k in sorted(agg):
        print(f"  {k[0]:40s} {k[1]:24s} {agg[k]:20.1f}   dispatches={len(disp[k])}")
