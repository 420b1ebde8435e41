"""k_sc_score3 check on one image: fast totals of every crop (bound-and-verify
path, exact_all=0) against the oracle's exact sequential totals."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

from flyimg_amd import _lib as L  # noqa: E402
from flyimg_amd.runtime import Context  # noqa: E402
from flyimg_amd.synth import synth_rgb  # noqa: E402
from oracle import oracle as orc  # noqa: E402

w, h = (int(v) for v in (sys.argv[1:3] if len(sys.argv) > 2 else (500, 281)))
src = synth_rgb(w, h, 0x5EED)
ref = orc.sc_crop(src, 100, 100)
with Context(0) as ctx:
    o = L.FiSmartcropOptions()
    L.lib().fi_smartcrop_default_options(o)
    o.exact_all = 0
    b = ctx.stats("sc_score_mfma")[1]
    r = ctx.smartcrop_ex(src, 100, 100, options=o)
    print("mfma images:", ctx.stats("sc_score_mfma")[1] - b, "top", r["top_index"], "ref top", ref["top_index"])
    worst = 0
    for i, (c, g) in enumerate(zip(r["crops"], ref["crops"])):
        ex = g["score"]
        rel = [abs(getattr(c, k) - ex[k]) / max(1e-300, abs(ex[k])) for k in ("detail", "skin", "saturation", "total")]
        worst = max(worst, max(rel))
        if i < 6 or max(rel) > 1e-9:
            print(i, c.x, c.y, c.exact, ["%.3e" % v for v in rel], c.total, ex["total"])
    print("worst rel", worst)
