#!/usr/bin/env python3
"""Per-dispatch HBM traffic of one kernel from rocprofv3 --pmc passes
(FETCH_SIZE, WRITE_SIZE in KiB summed over the XCDs) -> JSON for bench.py's
roofline.traffic.  gfx950 correction (MI355X_MICROARCH.md, HBM section):
FETCH_SIZE counts half the bytes of wide (16 B/lane) coalesced reads, so it
is doubled; WRITE_SIZE is taken as is (dword/byte stores: uncalibrated).

  pmc_to_json.py <pmc dir> <kernel substring> <images per dispatch> <out.json>
  pmc_to_json.py <pmc dir> <kernel substring> total:<images> <out.json>
      (mixed batches: every matching dispatch summed, divided by the images
      the run resampled)
"""
import collections
import csv
import glob
import hashlib
import json
import os
import sys


def source_hash():
    """sha256 of the library's kernel and host sources (bench.py checks it: a
    traffic figure measured on other sources is reported as stale)"""
    d = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "flyimg_amd", "csrc")
    h = hashlib.sha256()
    for f in sorted(os.listdir(d)):
        if f.endswith((".hip", ".cpp", ".h")):
            h.update(f.encode())
            h.update(open(os.path.join(d, f), "rb").read())
    return h.hexdigest()


root, kname, ipd_arg, out = sys.argv[1], sys.argv[2], sys.argv[3], sys.argv[4]
total_mode = ipd_arg.startswith("total:")
ipd = int(ipd_arg.split(":")[-1])
vals = collections.defaultdict(lambda: collections.defaultdict(float))
for f in glob.glob(f"{root}/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if kname not in r.get("Kernel_Name", ""):
            continue
        vals[r["Counter_Name"]][r.get("Dispatch_Id", "0")] += float(r["Counter_Value"])
res = {"kernel": kname, "images_per_dispatch": ipd, "source_sha256": source_hash()}
for c in ("FETCH_SIZE", "WRITE_SIZE"):
    d = vals.get(c, {})
    # bench.py re-runs a small verification batch after the timed loop: only
    # the full-batch dispatches (>= half the largest) are per-dispatch samples
    if d and total_mode:
        res[c.lower() + "_kib_total"] = sum(d.values())
        res["dispatches"] = len(d)
    elif d:
        top = max(d.values())
        d = {k: v for k, v in d.items() if v >= 0.5 * top}
        res[c.lower() + "_kib_per_dispatch"] = sum(d.values()) / len(d)
        res["dispatches"] = len(d)
if total_mode and "fetch_size_kib_total" in res and "write_size_kib_total" in res:
    b = 2 * res["fetch_size_kib_total"] * 1024 + res["write_size_kib_total"] * 1024
    res["images_per_dispatch"] = None
    res["images_total"] = ipd
    res["hbm_bytes_per_image"] = b / ipd
    res["correction"] = "2 x FETCH_SIZE (gfx950 wide-read half count) + WRITE_SIZE, summed over the run"
elif "fetch_size_kib_per_dispatch" in res and "write_size_kib_per_dispatch" in res:
    b = 2 * res["fetch_size_kib_per_dispatch"] * 1024 + res["write_size_kib_per_dispatch"] * 1024
    res["hbm_bytes_per_dispatch"] = b
    res["hbm_bytes_per_image"] = b / ipd
    res["correction"] = "2 x FETCH_SIZE (gfx950 wide-read half count) + WRITE_SIZE"
json.dump(res, open(out, "w"), indent=1)
print(json.dumps(res))
