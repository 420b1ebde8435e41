#!/usr/bin/env python3
"""Where does the resample path under test differ from the oracle?  Prints
the error pattern (rows / columns / channels) of one geometry."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from flyimg_amd import _lib as L  # noqa: E402
from flyimg_amd.runtime import Context, Op  # noqa: E402
from flyimg_amd.synth import synth_rgb  # noqa: E402
from oracle import oracle as orc  # noqa: E402

W, H, tw, th = (int(x) for x in (sys.argv[1:5] if len(sys.argv) > 4 else (1920, 1080, 500, 0)))
flags = L.FI_OP_THUMBNAIL | L.FI_GEOM_SHRINK_ONLY
oflags = orc.FLAG_THUMBNAIL | orc.FLAG_SHRINK
n = int(os.environ.get("NIMG", "1"))
src = synth_rgb(W, H, 1000 + W + H)
with Context(0) as ctx:
    outs, recs, rc = ctx.process([src] * n, [Op(tw, th, flags)] * n)
    print("rc", rc, "paths", {k: ctx.stats(k)[1] for k in ("path_vm", "path_fused", "path_mfma")})
ref = orc.im_convert(src, tw, th, oflags)
for k, o in enumerate(outs[:2]):
    d = np.abs(o.astype(int) - ref.astype(int))
    print(f"image {k}: max {d.max()} exact {(d == 0).mean():.5f}")
    bad = d > 1
    rows = np.where(bad.any(axis=(1, 2)))[0]
    cols = np.where(bad.any(axis=(0, 2)))[0]
    print("  bad rows", rows[:40], "... n", len(rows))
    print("  bad cols", cols[:60], "... n", len(cols))
    print("  bad per channel", bad.sum(axis=(0, 1)))
    if len(rows):
        r = rows[0]
        c = np.where(bad[r].any(axis=1))[0]
        print("  row", r, "cols", c[:20], "gpu", o[r, c[:4]].tolist(), "ref", ref[r, c[:4]].tolist())
