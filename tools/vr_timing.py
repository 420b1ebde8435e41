#!/usr/bin/env python3
"""Per-phase cycle sums of k_rs_vr (FI_VR_VARIANT=9 stamps, s_memtime ticks)
on a full cfg2 batch, averaged over the persistent workgroups.
V waves 0-7: tile entry, vertical MFMA issue, block done (planes), barrier.
H waves 8-12: -, tile entry (fragment reload), horizontal pass, -, barrier.
L waves 14-15: A-fragment DMA issue, phase records + row DMA issue, vmcnt wait, barrier."""
import ctypes
import os
import sys

VR = True  # k_rs_vr (k_rs_vp was retired in round 3)
os.environ["FI_VR_VARIANT"] = os.environ.get("VP_STAMP_VARIANT", "9")
os.environ["FI_VR_RS"] = "1"
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

from flyimg_amd import _lib as L  # noqa: E402
from flyimg_amd.processor import ImageProcessor, OptionsBag  # noqa: E402
from flyimg_amd.runtime import Context  # noqa: E402
from flyimg_amd.runtime import plan as fi_plan  # noqa: E402

W, H, n = int(os.environ.get("VP_W", "1920")), int(os.environ.get("VP_H", "1080")), int(os.environ.get("NIMG", "1024"))
op = ImageProcessor(OptionsBag(os.environ.get("VP_OPTS", "w_500")), W, H).to_op()
stride = (W * 3 + 15) // 16 * 16
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
    NS = 16 * 6
    buf = np.zeros(256 * NS, np.uint64)
    fn = L.lib().fi_debug_vr_stamps
    fn.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int32]
    L.check(fn(ctx.h, buf.ctypes.data, 256))
    a = buf.reshape(256, 16, 6).astype(np.float64)
    a = a[a[:, 0, 5] > 0]
    ph = a[:, 0, 5].mean()
    nl = int(os.environ.get("VR_NL", "2"))  # the launch's loader waves (fi_api.cpp picks 4 for one-block strips)
    roles = {"V": (range(0, 8), ["tile entry", "V-MFMA issue", "planes", "barrier", "plane wait"]),
             "H": (range(8, 15 - nl), ["-", "tile entry", "horizontal", "-", "barrier"]),
             "L": (range(16 - nl, 16), ["A DMA", "records + row DMA", "vmcnt wait", "barrier"])}
    print(f"{len(a)} workgroups, phases/WG {ph:.0f}; per-phase ticks by wave (mean over workgroups)")
    for r, (waves, names) in roles.items():
        for w in waves:
            v = a[:, w, :len(names)].mean(axis=0) / ph
            work = sum(x for n, x in zip(names, v) if n not in ("barrier", "-", "plane wait"))
            print(f"  {r} wave {w:2d}: work {work:7.0f} | " + "  ".join(f"{n} {x:6.0f}" for n, x in zip(names, v)))
