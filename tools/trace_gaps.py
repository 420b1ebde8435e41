#!/usr/bin/env python3
"""Timeline of a rocprofv3 kernel + memory-copy trace: every dispatch/copy in
start order with its duration and the idle gap before it (ns -> us)."""
import csv
import glob
import sys

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/trace"
ev = []
for f in glob.glob(f"{root}/**/*kernel_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"][:60]))
for f in glob.glob(f"{root}/**/*memory_copy_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "copy " + r.get("Direction", "")))
ev.sort()
ev = [e for e in ev if "k_synth" not in e[2]]
prev_end = None
busy = 0
for s, e, n in ev:
    gap = (s - prev_end) / 1e3 if prev_end else 0.0
    print(f"{(s - ev[0][0]) / 1e3:10.1f} .. {(e - ev[0][0]) / 1e3:10.1f} us {(e - s) / 1e3:9.1f} us  gap {gap:9.1f} us  {n}")
    prev_end = max(prev_end or e, e)
    busy += e - s
if ev:
    span = ev[-1][1] - ev[0][0]
    print(f"span {span / 1e6:.3f} ms, busy {busy / 1e6:.3f} ms")
