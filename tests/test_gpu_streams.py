"""Stream ordering of the batch pipeline on the GPU (MI355X), through the C-ABI.

The crop apply of batch k runs on its own stream beside batch k+1's resample
(fi_api.cpp launch_batch); the RCCL record gather runs on a stream of its own
(fi_rccl_gather_start / _finish).  These tests pin what the header promises
across those streams:

* a device-ordered entry point (fi_pixelate_regions_device) called right after
  an asynchronous smart-crop batch sees the applied crop, as after fi_wait;
* a batch whose sources are the previous in-flight batch's outputs (a chained
  request) reads the applied pixels;
* a 1-rank gather started while two full-size batches are queued returns
  before they finish (it does not wait for the batch streams: VERDICT r5 item 2).
"""
import ctypes
import time

import numpy as np
import pytest

from flyimg_amd import _lib as L
from flyimg_amd.processor import ImageProcessor, OptionsBag
from flyimg_amd.runtime import Context
from flyimg_amd.runtime import plan as fi_plan

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    c = Context(0)
    yield c
    c.close()


def _batch(ctx, pool, W, H, stride, n, op, dst, cap):
    arr = (L.FiImage * n)()
    for i in range(n):
        a = arr[i]
        a.src, a.src_w, a.src_h, a.src_stride, a.src_channels = pool + i * stride * H, W, H, stride, 3
        a.target_w, a.target_h, a.flags, a.gravity = op.target_w, op.target_h, op.flags, op.gravity
        a.smartcrop_w, a.smartcrop_h = op.smartcrop_w, op.smartcrop_h
        a.dst, a.dst_capacity = dst + i * cap, cap
    return arr


def test_pixelate_device_after_async_apply_sees_the_crop(ctx):
    """fi_pixelate_regions_device on a dst of a batch just
    submitted (its apply still on the apply stream) gives the same bytes as the
    synchronous batch followed by the same call."""
    W, H, n = 1920, 1080, 64
    op = ImageProcessor(OptionsBag("w_500,smc_1"), W, H).to_op()
    assert op.flags & L.FI_OP_SMARTCROP_APPLY
    ow, oh, oc = fi_plan(W, H, op)
    cap = ow * oh * oc
    stride = W * 3
    pool = ctx.malloc(stride * H * n)
    dst = ctx.malloc(cap * n * 2)
    boxes = (ctypes.c_int32 * 8)(10, 10, 60, 60, 120, 30, 40, 40)
    try:
        for i in range(n):
            ctx.fill_synthetic(pool + i * stride * H, W, H, stride, 4100 + i)
        # reference: synchronous batch, then the face-blur of a 200 x 200 view of image 5's dst
        ref = _batch(ctx, pool, W, H, stride, n, op, dst, cap)
        L.check(ctx.process_device(ref, n))
        L.check(L.lib().fi_pixelate_regions_device(ctx.h, dst + 5 * cap, 200, 200, 600, 3, boxes, 2))
        want = ctx.d2h(dst, cap * n)
        # asynchronous: submit, then the face-blur at once (the apply may still run)
        got_arr = _batch(ctx, pool, W, H, stride, n, op, dst + cap * n, cap)
        L.check(ctx.submit_device(got_arr, n))
        L.check(L.lib().fi_pixelate_regions_device(ctx.h, dst + cap * n + 5 * cap, 200, 200, 600, 3, boxes, 2))
        L.check(ctx.wait(0))
        got = ctx.d2h(dst + cap * n, cap * n)
        for i in range(n):
            assert (got_arr[i].crop_w, got_arr[i].crop_h) == (ref[i].crop_w, ref[i].crop_h)
            m = ref[i].out_w * ref[i].out_h * oc
            assert np.array_equal(got[i * cap:i * cap + m], want[i * cap:i * cap + m]), i
    finally:
        ctx.free(pool)
        ctx.free(dst)


def test_chained_batch_reads_the_applied_crop(ctx):
    """Batch B resizes batch A's smart-cropped outputs, submitted while A is
    in flight: B waits for A's apply (its sources overlap A's dst) and equals
    the same chain run synchronously."""
    W, H, n = 1280, 720, 32
    opa = ImageProcessor(OptionsBag("w_600,smc_1"), W, H).to_op()
    owa, oha, oca = fi_plan(W, H, opa)
    capa = owa * oha * oca
    stride = W * 3
    pool = ctx.malloc(stride * H * n)
    da = ctx.malloc(capa * n * 2)
    try:
        for i in range(n):
            ctx.fill_synthetic(pool + i * stride * H, W, H, stride, 7100 + i)

        def chain(base_a, base_b, sync):
            a = _batch(ctx, pool, W, H, stride, n, opa, base_a, capa)
            if sync:
                L.check(ctx.process_device(a, n))
            else:
                L.check(ctx.submit_device(a, n))
            # B's source: the first 120 rows of 360 bytes of A's dst (inside
            # any crop of a 600 x 338 image: the box is at least 300 px square),
            # planned before A's crop size is known, as a chained request is
            opb = ImageProcessor(OptionsBag("w_60"), 120, 120).to_op()
            owb, ohb, ocb = fi_plan(120, 120, opb)
            capb = owb * ohb * ocb
            b = (L.FiImage * n)()
            for i in range(n):
                x = b[i]
                x.src, x.src_w, x.src_h, x.src_stride, x.src_channels = base_a + i * capa, 120, 120, 360, 3
                x.target_w, x.target_h, x.flags, x.gravity = opb.target_w, opb.target_h, opb.flags, opb.gravity
                x.dst, x.dst_capacity = base_b + i * capb, capb
            if sync:
                L.check(ctx.process_device(b, n))
            else:
                L.check(ctx.submit_device(b, n))
                L.check(ctx.wait(0))
            for i in range(n):
                assert a[i].status == 0 and min(a[i].crop_w, a[i].crop_h) >= 300, (a[i].crop_w, a[i].crop_h)
                assert b[i].status == 0
            return ctx.d2h(base_b, capb * n)

        db = ctx.malloc(60 * 60 * 3 * n * 2)
        try:
            want = chain(da, db, True)
            got = chain(da + capa * n, db + 60 * 60 * 3 * n, False)
            assert np.array_equal(got, want)
        finally:
            ctx.free(db)
    finally:
        ctx.free(pool)
        ctx.free(da)


def test_gather_returns_while_batches_run():
    """a 1-rank RCCL record gather started while two
    full-size cfg2 batches are queued completes before they do (its stream
    does not wait for the batch streams); the records come back unchanged."""
    ctx = Context(0)
    try:
        lib = L.lib()
        uid = ctypes.create_string_buffer(128)
        L.check(lib.fi_rccl_get_unique_id(uid))
        L.check(lib.fi_rccl_init(ctx.h, 0, 1, uid.raw))
        W, H, n = 1920, 1080, 1024
        op = ImageProcessor(OptionsBag("w_500,smc_1"), W, H).to_op()
        ow, oh, oc = fi_plan(W, H, op)
        cap = ow * oh * oc
        stride = (W * 3 + 15) // 16 * 16
        pool = ctx.malloc(stride * H * n)
        dst = ctx.malloc(cap * n * 2)
        try:
            for i in range(n):
                ctx.fill_synthetic(pool + i * stride * H, W, H, stride, 0x5EED + i)
            arrs = [_batch(ctx, pool, W, H, stride, n, op, dst + b * cap * n, cap) for b in (0, 1)]
            L.check(ctx.submit_device(arrs[0], n))  # warm (tables, skin/sat table)
            L.check(ctx.wait(0))
            for a in arrs:
                L.check(ctx.submit_device(a, n))
            assert ctx.query() >= 1
            recs = [(i, 0, 500, 281, i % 97, i % 13, 281, 281) for i in range(n)]
            send = (L.FiRecord * n)(*[L.FiRecord(*r) for r in recs])
            recv = (L.FiRecord * n)()
            t0 = time.perf_counter()
            L.check(lib.fi_rccl_gather_start(ctx.h, send, n, recv))
            L.check(lib.fi_rccl_gather_finish(ctx.h))
            t_gather = time.perf_counter() - t0
            running = ctx.query()
            L.check(ctx.wait(0))
            assert running >= 1, ("the gather waited for the batches", t_gather)
            assert [tuple(getattr(recv[i], f) for f, _ in L.FiRecord._fields_) for i in range(n)] == recs
            assert ctx.query() == 0
            assert all(arrs[1][i].status == 0 for i in range(n))
        finally:
            ctx.free(pool)
            ctx.free(dst)
    finally:
        ctx.close()


def test_record_gather_rccl_array_form():
    """RecordGather over RCCL (one rank) takes bench.py's cfg4 form -- an
    (n, 8) int32 block, copied into the fi_record send buffer in one move --
    and hands rank 0 the same rows back as an array; the tuple form still
    gives tuples."""
    from flyimg_amd.parallel import RecordGather

    ctx = Context(0)
    try:
        lib = L.lib()
        uid = ctypes.create_string_buffer(128)
        L.check(lib.fi_rccl_get_unique_id(uid))
        L.check(lib.fi_rccl_init(ctx.h, 0, 1, uid.raw))

        class One:
            rank, world = 0, 1

        g = RecordGather(One())
        g.ctx, g.backend = ctx, "rccl"  # the world > 1 backend, on this one rank's communicator
        recs = np.arange(300 * 8, dtype=np.int32).reshape(300, 8)
        got = g.gather(recs)
        assert isinstance(got, np.ndarray) and got.dtype == np.int32 and np.array_equal(got, recs)
        rows = [tuple(int(x) for x in r) for r in recs[:5]]
        assert g.gather(rows) == rows
    finally:
        ctx.close()
