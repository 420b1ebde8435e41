#!/usr/bin/env python3
"""k_rs_vr vs k_rs_vm: the persistent block-major resample must be
bit-identical to the streaming kernel (same weights, same integer algebra) on
every geometry class; cases k_rs_vr does not take print vr_images 0.

  python tools/vr_check.py            (GPU)
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from flyimg_amd import _lib as L  # noqa: E402
from flyimg_amd.processor import ImageProcessor, OptionsBag  # noqa: E402
from flyimg_amd.runtime import Context  # noqa: E402
from flyimg_amd.synth import synth_rgb  # noqa: E402


def ctx_with(env):
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        return Context(0)
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


CASES = [
    # (W, H, options, images)
    (1920, 1080, "w_500", 3),
    (1920, 1080, "w_500", 40),
    (3840, 2160, "w_512,h_512,c_1", 2),
    (6000, 4000, "w_400,h_400,c_1,r_90,clsp_Gray", 2),
    (3000, 2000, "w_300,h_250,c_1", 3),
    (1024, 768, "w_200,h_200,c_1,r_180", 2),
    (1200, 900, "w_300,r_270", 2),
    (800, 600, "w_250,clsp_Gray", 2),
    (2000, 1500, "w_640,h_480,c_1,mnchr_1", 1),
    (333, 517, "w_97", 4),
    (4000, 3000, "w_150", 2),
    (3840, 2160, "w_512,h_512,c_1", 300),
    (1920, 1080, "w_500", 300),
    (6000, 4000, "w_400,h_400,c_1,r_90,clsp_Gray", 24),
    (640, 480, "w_320", 7),
]

PATH = "path_vr"
vm = ctx_with({"FI_VR_RS": "0"})
vp = ctx_with({"FI_VR_RS": "1"})
bad = 0
for (W, H, opts, n) in CASES:
    op = ImageProcessor(OptionsBag(opts), W, H).to_op()
    srcs = [synth_rgb(W, H, 77 + k) for k in range(min(n, 4))]
    srcs = [srcs[k % len(srcs)] for k in range(n)]
    before = vp.stats(PATH)[1]
    oa, ra, rca = vm.process(srcs, [op] * n)
    ob, rb, rcb = vp.process(srcs, [op] * n)
    ran = vp.stats(PATH)[1] - before
    same = all(a is not None and b is not None and np.array_equal(a, b) for a, b in zip(oa, ob))
    diff = 0
    if not same:
        for a, b in zip(oa, ob):
            if a is not None and b is not None and a.shape == b.shape:
                diff = max(diff, int(np.abs(a.astype(int) - b.astype(int)).max()))
                nb = int((a != b).sum())
    print(f"{W}x{H} {opts} x{n}: rc {rca}/{rcb} vr_images {ran} identical {same}"
          + ("" if same else f" maxdiff {diff} ndiff {nb}"), flush=True)
    bad += (not same) or rca != 0 or rcb != 0
print("FAIL" if bad else "OK", bad)
sys.exit(1 if bad else 0)
