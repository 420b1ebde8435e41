"""k_sc_score3 in the batch path: crop box / score / candidates of a cfg2
image against the oracle on the GPU-resized pixels (FI_SC_MFMA selects)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

from flyimg_amd import _lib as L  # noqa: E402
from flyimg_amd.processor import ImageProcessor, OptionsBag  # noqa: E402
from flyimg_amd.runtime import Context, Op  # noqa: E402
from flyimg_amd.synth import synth_rgb  # noqa: E402
from oracle import oracle as orc  # noqa: E402

W, H, opts = 1920, 1080, "w_500,smc_1"
src = synth_rgb(W, H, 0x5EED + W)
op = ImageProcessor(OptionsBag(opts), W, H).to_op()
op_noapply = Op(op.target_w, op.target_h, op.flags & ~L.FI_OP_SMARTCROP_APPLY, op.gravity, op.rotate, 100, 100)
with Context(0) as ctx:
    outs, recs, rc = ctx.process([src, src], [op_noapply, op])
    print("mfma images", ctx.stats("sc_score_mfma")[1], "valu", ctx.stats("sc_score_valu")[1])
    resized = outs[0]
    ref = orc.sc_crop(resized, 100, 100)
    for r in recs:
        print("gpu", (r.crop_x, r.crop_y, r.crop_w, r.crop_h), r.crop_score, r.n_candidates)
    t = ref["top_crop"]
    print("ref", (t["x"], t["y"], t["width"], t["height"]), t["score"]["total"])
    tots = sorted(((c["score"]["total"], i) for i, c in enumerate(ref["crops"])), reverse=True)[:4]
    print("ref best 4", tots)
    o = L.FiSmartcropOptions()
    L.lib().fi_smartcrop_default_options(o)
    o.exact_all = 0
    r = ctx.smartcrop_ex(resized, 100, 100, options=o)
    print("smartcrop_ex on resized: top", r["top_index"], r["crops"][r["top_index"]].total)
    for i, (c, g) in enumerate(zip(r["crops"], ref["crops"])):
        d = abs(c.total - g["score"]["total"])
        if d > 1e-12 * abs(g["score"]["total"]):
            print(" crop", i, c.total, g["score"]["total"])
