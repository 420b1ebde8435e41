#!/usr/bin/env python3
"""Single-image request latency: the serving shape of the hot path
(ImageHandler::processImage -> one convert per request) --
ONE 1920x1080 host image, w_500,smc_1, through fi_process_batch (host buffers
in, host buffer out), 200 calls after a warmup.

Two passes:
  * wall: fi_process_batch wall time per call, timing events off -> p50 / p99
  * split: the same with the library's timed ranges on (fi_set_timing): per
    call the host source staging (pageable rows -> pinned, copy issue), the
    H2D copy (h2d_src, on the upload stream), the device batch (batch: first
    kernel .. last kernel), the D2H copy of the output (d2h_out), the host
    planning (host_plan) -- p50 of each.
Both for a pageable numpy source/destination and for pinned ones (fi_host_alloc).

  python tools/latency_bench.py [--calls 200] [--out profiles/r03/latency.json]
"""
import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from flyimg_amd import _lib as L  # noqa: E402
from flyimg_amd.processor import ImageProcessor, OptionsBag  # noqa: E402
from flyimg_amd.runtime import Context, _fill  # noqa: E402
from flyimg_amd.synth import synth_rgb  # noqa: E402

W, H, OPTS = 1920, 1080, "w_500,smc_1"
SPLIT = ("host_src_stage", "h2d_src", "host_plan", "batch", "resize", "sc_prep", "sc_score", "crop_apply", "d2h_out",
         "host_total")


def pct(v, q):
    return float(np.percentile(np.asarray(v), q))


def run(ctx, src, dst, op, calls, warmup, timing):
    tmpl = (L.FiImage * 1)()
    a = tmpl[0]
    a.src, a.src_h, a.src_w, a.src_stride, a.src_channels = src.ctypes.data, H, W, src.strides[0], 3
    _fill(a, op)
    L.check(L.lib().fi_plan(tmpl, 1))
    cap = a.out_w * a.out_h * max(a.out_channels, 1)
    assert dst.nbytes >= cap
    a.dst, a.dst_capacity = dst.ctypes.data, dst.nbytes
    arr = (L.FiImage * 1)()
    ctx.set_timing(timing)
    wall, split = [], {k: [] for k in SPLIT}
    lib = L.lib()
    for k in range(warmup + calls):
        ctypes.memmove(arr, tmpl, ctypes.sizeof(tmpl))
        before = {n: ctx.stats(n)[0] for n in SPLIT} if timing else None
        t0 = time.perf_counter()
        rc = lib.fi_process_batch(ctx.h, arr, 1)
        t1 = time.perf_counter()
        if rc != 0 or arr[0].status != 0:
            raise RuntimeError(f"fi_process_batch rc {rc} status {arr[0].status}")
        if k < warmup:
            continue
        wall.append((t1 - t0) * 1e3)
        if timing:
            for n in SPLIT:
                split[n].append(ctx.stats(n)[0] - before[n])
    ctx.set_timing(False)
    out = {"p50_ms": round(pct(wall, 50), 4), "p99_ms": round(pct(wall, 99), 4), "mean_ms": round(float(np.mean(wall)), 4),
           "min_ms": round(min(wall), 4), "calls": calls,
           "crop": [arr[0].out_w, arr[0].out_h]}
    if timing:
        out["split_p50_ms"] = {n: round(pct(v, 50), 4) for n, v in split.items()}
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--calls", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--out", default="")
    args = ap.parse_args()
    ctx = Context(0)
    op = ImageProcessor(OptionsBag(OPTS), W, H).to_op()
    res = {"workload": f"1 x {W}x{H} RGB8 host image, {OPTS}, fi_process_batch", "calls": args.calls}
    src_pg = np.ascontiguousarray(synth_rgb(W, H, 1234))
    dst_pg = np.zeros(W * H * 3, np.uint8)
    src_pin = ctx.host_array((H, W, 3))
    src_pin[...] = src_pg
    dst_pin = ctx.host_array((W * H * 3,))
    for name, s, d in (("pageable", src_pg, dst_pg), ("pinned", src_pin, dst_pin)):
        wall = run(ctx, s, d, op, args.calls, args.warmup, False)
        spl = run(ctx, s, d, op, args.calls, args.warmup, True)
        wall["split_p50_ms"] = spl["split_p50_ms"]
        wall["timed_pass_p50_ms"] = spl["p50_ms"]
        res[name] = wall
        print(name, json.dumps(wall), flush=True)
    ctx.close()
    if args.out:
        os.makedirs(os.path.dirname(args.out) or ".", exist_ok=True)
        with open(args.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
