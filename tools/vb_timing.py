#!/usr/bin/env python3
"""Per-phase cycle sums of k_rs_vb (FI_VB_VARIANT=9 stamps of wave 0,
s_memtime ticks) on a full cfg2 batch, averaged over the persistent
workgroups.  Phases: 0 top vmcnt wait, 1 top barrier, 2 item entry + stores
of the previous block, 3 B reads + vertical MFMA, 4 fold + planes, 5 planes
barrier, 6 A-record + group DMA issue, 7 horizontal pass, 8 cursor, 9 loop
tail."""
import ctypes
import os
import sys

os.environ["FI_VB_VARIANT"] = "9"
os.environ["FI_VB_RS"] = "1"
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

from flyimg_amd import _lib as L  # noqa: E402
from flyimg_amd.processor import ImageProcessor, OptionsBag  # noqa: E402
from flyimg_amd.runtime import Context  # noqa: E402
from flyimg_amd.runtime import plan as fi_plan  # noqa: E402

W, H = int(os.environ.get("W", "1920")), int(os.environ.get("H", "1080"))
n = int(os.environ.get("NIMG", "1024"))
op = ImageProcessor(OptionsBag(os.environ.get("OPTS", "w_500")), W, H).to_op()
stride = (W * 3 + 15) // 16 * 16
ow, oh, oc = fi_plan(W, H, op)
cap = ow * oh * oc
NS = 12
with Context(0) as ctx:
    pool = ctx.malloc(stride * H * n)
    dst = ctx.malloc(cap * n)
    for i in range(n):
        ctx.fill_synthetic(pool + i * stride * H, W, H, stride, 7 + i)
    arr = (L.FiImage * n)()
    for i in range(n):
        a = arr[i]
        a.src, a.src_w, a.src_h, a.src_stride, a.src_channels = pool + i * stride * H, W, H, stride, 3
        a.target_w, a.target_h, a.flags, a.gravity, a.rotate = op.target_w, op.target_h, op.flags, op.gravity, op.rotate
        a.dst, a.dst_capacity = dst + i * cap, cap
    for _ in range(3):
        L.check(ctx.process_device(arr, n))
    buf = np.zeros(1024 * NS, np.uint64)
    L.lib().fi_debug_vb_stamps.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int32]
    L.check(L.lib().fi_debug_vb_stamps(ctx.h, buf.ctypes.data, 1024))
    a = np.array([r for r in buf.reshape(1024, NS) if r[10] > 0], dtype=np.float64)
    tot = a[:, :10].sum(axis=1)
    print(f"{len(a)} workgroups; blocks/WG {a[:, 10].mean():.1f} (min {a[:, 10].min():.0f} max {a[:, 10].max():.0f}); "
          f"items/WG {a[:, 11].mean():.1f}; total ticks/WG {tot.mean():.0f} (max {tot.max():.0f})")
    names = ["top wait", "top barrier", "entry+stores", "B + V-MFMA", "fold+planes", "planes bar", "DMA issue",
             "horizontal", "cursor", "loop tail"]
    for k in range(10):
        print(f"  {names[k]:12s} {a[:, k].mean():12.0f}  ({a[:, k].mean() / tot.mean() * 100:5.1f} %)  "
              f"per block {a[:, k].mean() / a[:, 10].mean():8.0f}")
