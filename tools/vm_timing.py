#!/usr/bin/env python3
"""Per-phase cycle sums of k_rs_vm (FI_VM_VARIANT=9 stamps, s_memtime ticks)
on a full cfg2 batch: averaged over the workgroups of a few images.
phases: 0 tail of previous iteration (block phase of non-last pieces),
1 top barrier, 2 piece LDS write (incl. the wait for its loads), 3 A-fragment
and next-piece loads issue, 4 second barrier, 5 vertical MFMA issue, 6 block
phase, 7 stores of the previous block."""
import os
import sys

os.environ["FI_VM_VARIANT"] = "9"
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

from flyimg_amd import _lib as L  # noqa: E402
from flyimg_amd.processor import ImageProcessor, OptionsBag  # noqa: E402
from flyimg_amd.runtime import Context  # noqa: E402
from flyimg_amd.runtime import plan as fi_plan  # noqa: E402

W, H, n = 1920, 1080, int(os.environ.get("NIMG", "1024"))
op = ImageProcessor(OptionsBag("w_500"), W, H).to_op()
stride = W * 3
ow, oh, oc = fi_plan(W, H, op)
cap = ow * oh * oc
with Context(0) as ctx:
    pool = ctx.malloc(stride * H * n)
    dst = ctx.malloc(cap * n)
    for i in range(n):
        ctx.fill_synthetic(pool + i * stride * H, W, H, stride, 7 + i)
    arr = (L.FiImage * n)()
    for i in range(n):
        a = arr[i]
        a.src, a.src_w, a.src_h, a.src_stride, a.src_channels = pool + i * stride * H, W, H, stride, 3
        a.target_w, a.target_h, a.flags, a.gravity = op.target_w, op.target_h, op.flags, op.gravity
        a.dst, a.dst_capacity = dst + i * cap, cap
    for _ in range(3):
        L.check(ctx.process_device(arr, n))
    import ctypes
    NS = 12
    buf = np.zeros(4096 * (NS + 1), np.uint64)
    L.lib().fi_debug_vm_stamps.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int32]
    L.check(L.lib().fi_debug_vm_stamps(ctx.h, buf.ctypes.data, 4096))
    rows = [r for r in buf.reshape(4096, NS + 1) if 0 < r[NS] < 1000]
    a = np.array(rows, dtype=np.float64)
    tot = a[:, :NS].sum(axis=1)
    print(f"{len(a)} workgroups; pieces/WG {a[:, NS].mean():.1f}; total ticks/WG {tot.mean():.0f}")
    names = ["tail/prev", "barrier1", "piece write", "A+row issue", "barrier2", "V-MFMA issue", "H pass",
             "stores", "planes+drain", "plane barrier", "-", "-"]
    for k in range(NS):
        print(f"  {names[k]:14s} {a[:, k].mean():10.0f}  ({a[:, k].mean() / tot.mean() * 100:5.1f} %)  "
              f"per piece {a[:, k].mean() / a[:, NS].mean():8.0f}")
