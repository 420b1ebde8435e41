"""Production-size batches on the GPU (MI355X): one full cfg2 batch (1024
1920x1080 images -> w_500,smc_1) from a device-resident pool of 6.4 GB, so the
source offsets of the later images -- and the descriptor / tile / strip
offsets derived from them -- run past 2^32, through fi_process_batch_device
(the bench's path), spot-checked against the oracle: pixels within +-1 LSB,
smart-crop box bit-exact on the GPU-resized pixels, applied crop == that box.
Also the same batch on the k_rs_vm kernel (FI_VR_RS=0) is byte for byte
k_rs_vr's (the default): k_rs_vm carries k_rs_vr's two-limb weights scaled to
2^22 (fi_plan.cpp axis_q22)."""
import os

import numpy as np
import pytest

from flyimg_amd import _lib as L
from flyimg_amd.processor import ImageProcessor, OptionsBag
from flyimg_amd.runtime import Context
from flyimg_amd.runtime import plan as fi_plan
from oracle.verify import verify_batch, verify_sample

pytestmark = pytest.mark.gpu

W, H, N = 1920, 1080, 1024


def _ctx(env):
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


@pytest.fixture(scope="module")
def pool_ctx():
    ctx = _ctx({"FI_VR_RS": "1"})
    stride = (W * 3 + 15) // 16 * 16
    img = stride * H
    pool = ctx.malloc(img * N)
    for i in range(N):
        ctx.fill_synthetic(pool + i * img, W, H, stride, 0xB16 + i)
    yield ctx, pool, stride, img
    ctx.free(pool)
    ctx.close()


def _run(ctx, pool, stride, img, op):
    ow, oh, oc = fi_plan(W, H, op)
    cap = ow * oh * oc
    dst = ctx.malloc(cap * N)
    arr = (L.FiImage * N)()
    for i in range(N):
        a = arr[i]
        a.src, a.src_w, a.src_h, a.src_stride, a.src_channels = pool + i * img, W, H, stride, 3
        a.target_w, a.target_h, a.flags, a.gravity, a.rotate = op.target_w, op.target_h, op.flags, op.gravity, op.rotate
        a.smartcrop_w, a.smartcrop_h = op.smartcrop_w, op.smartcrop_h
        a.dst, a.dst_capacity = dst + i * cap, cap
    rc = ctx._lib.fi_process_batch_device(ctx.h, arr, N)
    return rc, arr, dst, cap


@pytest.mark.parametrize("opts", ["w_500,smc_1", "w_500"])
def test_full_cfg2_batch_past_4gb(pool_ctx, opts):
    ctx, pool, stride, img = pool_ctx
    assert img * N > (1 << 32)
    op = ImageProcessor(OptionsBag(opts), W, H).to_op()
    before = ctx.stats("path_vr")[1]
    rc, arr, dst, cap = _run(ctx, pool, stride, img, op)
    try:
        assert rc == 0 and all(arr[i].status == 0 for i in range(N))
        assert ctx.stats("path_vr")[1] == before + N  # the persistent block-major kernel ran the batch
        idxs = verify_sample(N, img)
        assert max(idxs) * img > (1 << 32)
        ok, tot, err = verify_batch(ctx, arr, idxs, lambda i: pool + i * img, lambda i: 0xB16 + i, W, H, stride, op,
                                    lambda i: dst + i * cap, cap)
        assert err is None and ok == tot, err
    finally:
        ctx.free(dst)


def test_full_cfg2_batch_vr_equals_vm(pool_ctx):
    """k_rs_vr and k_rs_vm (the same weights, three limbs at 2^22) on the whole
    1024-image resized batch: every byte equal."""
    ctx, pool, stride, img = pool_ctx
    op = ImageProcessor(OptionsBag("w_500"), W, H).to_op()
    rc, arr, dst, cap = _run(ctx, pool, stride, img, op)
    vm = _ctx({"FI_VR_RS": "0"})
    try:
        assert rc == 0
        rc2, arr2, dst2, cap2 = _run(vm, pool, stride, img, op)
        try:
            assert rc2 == 0 and vm.stats("path_vr")[1] == 0
            a = ctx.d2h(dst, cap * N)
            b = vm.d2h(dst2, cap * N)
            assert np.array_equal(a, b), int(np.count_nonzero(a != b))
        finally:
            vm.free(dst2)
    finally:
        vm.close()
        ctx.free(dst)
