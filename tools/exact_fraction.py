#!/usr/bin/env python3
"""Exact fraction of the default resample (k_rs_vr; k_rs_vm carries the same
two-limb weights, so its bytes are the same) against the oracle's restatement
of ImageMagick's f64 resample, on each BASELINE geometry (synthetic images).
ADVICE r4 asked for the number next to the kernels: one JSON line per geometry
with max |diff|, the exact fraction and the table shifts the path used."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

from flyimg_amd.processor import ImageProcessor, OptionsBag  # noqa: E402
from flyimg_amd.runtime import Context  # noqa: E402
from flyimg_amd.synth import synth_rgb  # noqa: E402
from oracle import oracle as orc  # noqa: E402  (the checker)
from tests.test_gpu_parity import _oracle_flags  # noqa: E402

GEO = [("cfg1", 3000, 2000, "w_300,h_250,c_1"), ("cfg2", 1920, 1080, "w_500"),
       ("cfg3", 3840, 2160, "w_512,h_512,c_1"), ("cfg5", 6000, 4000, "w_400,h_400,c_1,r_90,clsp_Gray")]
out = []
for env in ({"FI_VR_RS": "1"}, {"FI_VR_RS": "0"}):
    os.environ.update(env)
    with Context(0) as ctx:
        for name, W, H, opts in GEO:
            op = ImageProcessor(OptionsBag(opts), W, H).to_op()
            tot_same, tot_n, dmax = 0, 0, 0
            for seed in (11, 12):
                src = synth_rgb(W, H, seed)
                got, recs, rc = ctx.process([src], [op])
                assert rc == 0 and recs[0].status == 0
                ref = orc.im_convert(src, op.target_w, op.target_h, _oracle_flags(op.flags), gravity=op.gravity,
                                     rotate=op.rotate)
                d = np.abs(got[0].astype(np.int16) - ref.astype(np.int16))
                tot_same += int((d == 0).sum())
                tot_n += d.size
                dmax = max(dmax, int(d.max()))
            r = {"geometry": name, "src": f"{W}x{H}", "options": opts, "kernel": "k_rs_vr" if env["FI_VR_RS"] == "1" else "k_rs_vm",
                 "max_abs_diff": dmax, "exact_fraction": round(tot_same / tot_n, 6), "values": tot_n}
            print(json.dumps(r), flush=True)
            out.append(r)
json.dump(out, open(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/exact_fraction.json", "w"), indent=1)
