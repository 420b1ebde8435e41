"""k_rs_vb vs k_rs_vm bitwise comparison on batches (both exact-integer paths
compute identical pixels), with the mismatch boxes per image; run twice to
tell a race from a deterministic indexing error."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from flyimg_amd import _lib as L  # noqa: E402
from flyimg_amd.processor import ImageProcessor, OptionsBag  # noqa: E402
from flyimg_amd.runtime import Context, Op  # noqa: E402
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
    (6000, 4000, "w_400,h_400,c_1,r_90,clsp_Gray,smc_1", 2),
    (6000, 4000, "w_400,h_400,c_1,r_90,clsp_Gray", 2),
    (6000, 4000, "w_400,h_400,c_1,clsp_Gray", 2),
    (6000, 4000, "w_400,h_400,c_1", 2),
    (6000, 4000, "w_400,h_400,c_1", 1),
    (3840, 2160, "w_512,h_512,c_1", 3),
]


def main():
    vb = ctx_with({"FI_VB_RS": "1"})
    vm = ctx_with({"FI_VB_RS": "0"})
    for W, H, opts, n in CASES:
        src = synth_rgb(W, H, 0x5EED + W)
        op = ImageProcessor(OptionsBag(opts), W, H).to_op()
        op = Op(op.target_w, op.target_h, op.flags & ~L.FI_OP_SMARTCROP_APPLY, op.gravity, op.rotate, 100, 100)
        ref, _, rc = vm.process([src] * n, [op] * n)
        assert rc == 0
        for rep in range(2):
            outs, _, rc = vb.process([src] * n, [op] * n)
            assert rc == 0, L.lib().fi_last_error()
            for i, (a, b) in enumerate(zip(outs, ref)):
                d = a.astype(np.int16) - b.astype(np.int16)
                bad = np.argwhere(d != 0)
                msg = f"{W}x{H} {opts} n={n} rep={rep} img={i} shape={a.shape}: {len(bad)} mismatches"
                if len(bad):
                    lo, hi = bad.min(0), bad.max(0)
                    rows = np.unique(bad[:, 0])
                    cols = np.unique(bad[:, 1])
                    msg += f" box {lo.tolist()}..{hi.tolist()} rows {rows[:12].tolist()} cols {cols[:12].tolist()}"
                    msg += f" maxabs {int(np.abs(d).max())}"
                print(msg, flush=True)
    vb.close()
    vm.close()


if __name__ == "__main__":
    main()
