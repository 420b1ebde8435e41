#!/usr/bin/env python3
"""Smart-crop stage on flat images (every crop window ties, so every crop is
re-scored with smartcrop.py's exact sequential sums): 1024 x 1920x1080 of one
colour -> w_500,smc_1; prints the stage times (ms per batch)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import numpy as np

    from flyimg_amd import _lib as L
    from flyimg_amd.processor import ImageProcessor, OptionsBag
    from flyimg_amd.runtime import Context
    from flyimg_amd.runtime import plan as fi_plan

    W, H, n = 1920, 1080, int(sys.argv[1]) if len(sys.argv) > 1 else 1024
    ctx = Context(0)
    op = ImageProcessor(OptionsBag("w_500,smc_1"), W, H).to_op()
    img = np.empty((H, W, 3), np.uint8)
    img[...] = (201, 144, 120)  # skin-ish flat colour
    src = ctx.malloc(img.nbytes)
    ctx.h2d(src, img)
    ow, oh, oc = fi_plan(W, H, op)
    cap = ow * oh * oc
    dst = ctx.malloc(cap * n)
    arr = (L.FiImage * n)()
    for i in range(n):
        a = arr[i]
        a.src, a.src_w, a.src_h, a.src_stride, a.src_channels = src, W, H, W * 3, 3
        a.target_w, a.target_h, a.flags, a.gravity = op.target_w, op.target_h, op.flags, op.gravity
        a.smartcrop_w = a.smartcrop_h = 100
        a.dst, a.dst_capacity = dst + i * cap, cap
    L.check(ctx.process_device(arr, n))  # warm
    ctx.set_timing(True)
    ctx.reset_stats()
    for _ in range(3):
        L.check(ctx.process_device(arr, n))
    st = {k: round(ctx.stats(k)[0] / 3, 4) for k in ("resize", "sc_prep", "sc_score", "crop_apply")}
    print(json.dumps({"images": n, "candidates_per_image": arr[0].n_candidates, "ms_per_batch": st}))
    ctx.free(src)
    ctx.free(dst)
    ctx.close()


if __name__ == "__main__":
    main()
