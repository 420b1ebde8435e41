#!/usr/bin/env python3
"""Host planner cost of a workload, on the CPU (no GPU): fi_debug_host_plan
runs run_batch's planning stages over the workload's batches and reports the
per-stage milliseconds (images, smartcrop, workspace, vm + vr tiles, of which
vr, hv tiles, blob).

  python tools/plan_prof.py [cfg4|cfg2] [iters]
"""
import ctypes
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
from flyimg_amd import _lib as L  # noqa: E402
from flyimg_amd.processor import ImageProcessor, OptionsBag  # noqa: E402
from flyimg_amd.runtime import plan as fi_plan  # noqa: E402

STAGES = ("images", "smartcrop", "workspace", "vm+vr tiles", "  of which vr", "hv tiles", "blob")


def batches(workload):
    if workload == "cfg2":
        return [[(1920, 1080, "w_500,smc_1")] * 1024]
    items = bench.cfg4_list(65536)
    out, cur = [], []
    for W, H, k in items:
        cur.append((W, H, bench.CFG4_OPS[k]))
        if len(cur) == 1024:
            out.append(cur)
            cur = []
    if cur:
        out.append(cur)
    return out


def main():
    workload = sys.argv[1] if len(sys.argv) > 1 else "cfg4"
    iters = int(sys.argv[2]) if len(sys.argv) > 2 else 1
    lib = L.lib()
    lib.fi_debug_host_plan.argtypes = [ctypes.POINTER(L.FiImage), ctypes.c_int32, ctypes.c_int32,
                                       ctypes.POINTER(ctypes.c_double)]
    ops = {}
    tot = (ctypes.c_double * 7)()
    base = 1 << 36
    bl = batches(workload)
    arrs = []
    for b in bl:
        arr = (L.FiImage * len(b))()
        addr = base
        for i, (W, H, opts) in enumerate(b):
            if (W, H, opts) not in ops:
                op = ImageProcessor(OptionsBag(opts), W, H).to_op()
                ops[(W, H, opts)] = (op, fi_plan(W, H, op))
            op, (ow, oh, oc) = ops[(W, H, opts)]
            a = arr[i]
            stride = (W * 3 + 15) // 16 * 16
            a.src, a.src_w, a.src_h, a.src_stride, a.src_channels = addr, W, H, stride, 3
            addr += (stride * H + 255) // 256 * 256
            a.target_w, a.target_h, a.flags, a.gravity, a.rotate = op.target_w, op.target_h, op.flags, op.gravity, op.rotate
            a.smartcrop_w, a.smartcrop_h = op.smartcrop_w, op.smartcrop_h
            a.dst, a.dst_capacity = addr, ow * oh * oc
            addr += (ow * oh * oc + 255) // 256 * 256
        arrs.append(arr)
    warm = (ctypes.c_double * 7)()
    for arr in arrs:  # the first pass builds every table (a service's first minutes)
        L.check(lib.fi_debug_host_plan(arr, len(arr), 1, warm))
    lib.fi_debug_host_plan(None, 1, 0, None)  # FI_PLAN_PROF=1: section timers of the timed passes only
    t0 = time.perf_counter()
    for _ in range(iters):
        for arr in arrs:
            L.check(lib.fi_debug_host_plan(arr, len(arr), 1, tot))
    wall = time.perf_counter() - t0
    lib.fi_debug_host_plan(None, 0, 0, None)
    print(f"first pass (tables built): {sum(warm[k] for k in (0, 1, 2, 3, 5, 6)):.0f} ms")
    n = len(bl) * iters
    print(f"{workload}: {len(bl)} batches x {iters}: per step (all batches once) "
          + ", ".join(f"{s.strip()} {tot[k] / iters:.1f} ms" for k, s in enumerate(STAGES))
          + f"; total {sum(tot[k] for k in (0, 1, 2, 3, 5, 6)) / iters:.1f} ms ({wall:.2f} s wall, {n} plans)")


if __name__ == "__main__":
    main()
