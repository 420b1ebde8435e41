"""Host planner checks that need no GPU (fi_debug_host_plan: the batch planner
on the host, image pointers planned but never dereferenced)."""
import ctypes
import time

import bench
from flyimg_amd import _lib as L
from flyimg_amd.processor import ImageProcessor, OptionsBag
from flyimg_amd.runtime import plan as fi_plan


def _batch(items):
    arr = (L.FiImage * len(items))()
    addr = 1 << 36
    for i, (W, H, opts) in enumerate(items):
        op = ImageProcessor(OptionsBag(opts), W, H).to_op()
        ow, oh, oc = fi_plan(W, H, op)
        a = arr[i]
        stride = (W * 3 + 15) // 16 * 16
        a.src, a.src_w, a.src_h, a.src_stride, a.src_channels = addr, W, H, stride, 3
        addr += (stride * H + 255) // 256 * 256
        a.target_w, a.target_h, a.flags, a.gravity, a.rotate = op.target_w, op.target_h, op.flags, op.gravity, op.rotate
        a.smartcrop_w, a.smartcrop_h = op.smartcrop_w, op.smartcrop_h
        a.dst, a.dst_capacity = addr, ow * oh * oc
        addr += (ow * oh * oc + 255) // 256 * 256
    return arr


def test_mixed_batch_keeps_its_images_on_k_rs_vr():
    """A cfg4 batch (mixed sizes and ops, whole-image tiles): images whose
    block windows cannot share the ring at a tile seam leave the k_rs_vr
    launch one by one instead of failing it for every image (round 5's planner
    put 42 % of cfg4's vertical-first images on k_rs_vr, round 6's 99.8 %)."""
    lib = L.lib()
    items = [(W, H, bench.CFG4_OPS[k]) for W, H, k in bench.cfg4_list(65536)[:1024]]
    arr = _batch(items)
    ms = (ctypes.c_double * 7)()
    t0 = time.perf_counter()
    try:
        L.check(lib.fi_debug_host_plan(arr, len(arr), 1, ms))
        cnt = (ctypes.c_double * 7)()
        L.check(lib.fi_debug_host_plan(None, 2, 0, cnt))
    finally:
        lib.fi_debug_host_plan(None, 0, 0, None)
    vr, vf, launches = cnt[0], cnt[1], cnt[2]
    assert vf > 500, vf  # most cfg4 geometries are vertical-first
    assert vr >= 0.98 * vf, (vr, vf)
    assert 1 <= launches <= 2  # one launch per strip-width group
    assert time.perf_counter() - t0 < 120
