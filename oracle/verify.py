"""Checker for device-resident batches (TEST INFRASTRUCTURE, like the rest of
oracle/): compares images of a batch the GPU path produced with the CPU
oracle.  Used by bench.py after its timed loop (the headline batch itself) and
by tests/test_gpu_parity.py; never by the product path."""
from __future__ import annotations


def oracle_flags(op):
    """The oracle's im_convert flags for a runtime Op (test infrastructure)."""
    from flyimg_amd import _lib as L
    from oracle import oracle as orc

    flags = 0
    for f, o in ((L.FI_OP_THUMBNAIL, orc.FLAG_THUMBNAIL), (L.FI_GEOM_FILL, orc.FLAG_FILL),
                 (L.FI_GEOM_SHRINK_ONLY, orc.FLAG_SHRINK), (L.FI_OP_EXTENT, orc.FLAG_EXTENT),
                 (L.FI_OP_GRAY, orc.FLAG_GRAY), (L.FI_OP_ROTATE, orc.FLAG_ROTATE)):
        if op.flags & f:
            flags |= o
    return flags


def verify_sample(nimg, img_bytes):
    """Indices of the images bench.py checks after the timed loop: first,
    second, last, 13 spread over the batch and the first two whose pool offset
    lies past 2^32 (descriptor / tile offsets beyond 32 bits)."""
    import numpy as np

    idx = {0, 1, nimg - 1} | {int(v) for v in np.linspace(0, nimg - 1, 13)}
    k = (1 << 32) // img_bytes + 1
    idx |= {i for i in (k, k + 1) if i < nimg}
    return sorted(i for i in idx if 0 <= i < nimg)


def verify_batch(ctx, arr, idxs, src_ptr, seed_of, W, H, src_stride, op, dst_of, dst_cap):
    """Check images of the LAST timed batch against the oracle (test
    infrastructure, outside the timed region): resampled pixels within +-1 LSB
    of oracle im_convert; with smart-crop, the record's box bit-exact with the
    oracle's smartcrop restatement on the GPU-resized pixels (an untimed
    no-apply batch of the same device sources gives those pixels) and the
    applied output equal to that box of them.  Returns (ok, total, first error)."""
    import numpy as np

    from flyimg_amd import _lib as L
    from flyimg_amd.runtime import Op
    from flyimg_amd.synth import synth_rgb
    from oracle import oracle as orc

    flags = oracle_flags(op)
    smc = bool(op.flags & L.FI_OP_SMARTCROP)
    apply = bool(op.flags & L.FI_OP_SMARTCROP_APPLY)
    resized = {}
    if smc:
        no_apply = Op(op.target_w, op.target_h, op.flags & ~L.FI_OP_SMARTCROP_APPLY, op.gravity, op.rotate,
                      op.smartcrop_w, op.smartcrop_h)
        outs, recs, rc = ctx.process_device_views([(src_ptr(i), W, H, src_stride) for i in idxs],
                                                  [no_apply] * len(idxs))
        for i, o, r in zip(idxs, outs, recs):
            resized[i] = (o, (r.crop_x, r.crop_y, r.crop_w, r.crop_h), r.status)
    ok, err = 0, None
    for i in idxs:
        a = arr[i]
        try:
            assert a.status == 0, f"status {a.status}"
            src = synth_rgb(W, H, seed_of(i))
            ref = orc.im_convert(src, op.target_w, op.target_h, flags, rotate=op.rotate)
            out = ctx.d2h(dst_of(i), a.out_h * a.out_stride).reshape(a.out_h, a.out_stride)
            out = out[:, : a.out_w * a.out_channels].reshape(a.out_h, a.out_w, a.out_channels)
            out = out[:, :, 0] if a.out_channels == 1 else out
            if not smc:
                assert out.shape == ref.shape, (out.shape, ref.shape)
                d = int(np.abs(out.astype(np.int16) - ref.astype(np.int16)).max())
                assert d <= 1, f"max |gpu - oracle| = {d}"
            else:
                rz, box, st = resized[i]
                assert st == 0 and rz is not None, f"no-apply status {st}"
                assert rz.shape == ref.shape, (rz.shape, ref.shape)
                d = int(np.abs(rz.astype(np.int16) - ref.astype(np.int16)).max())
                assert d <= 1, f"max |gpu - oracle| = {d}"
                rgb = rz if rz.ndim == 3 else np.repeat(rz[:, :, None], 3, axis=2)
                t = orc.sc_crop(np.ascontiguousarray(rgb), op.smartcrop_w or 100, op.smartcrop_h or 100)["top_crop"]
                want = (t["x"], t["y"], t["width"], t["height"])
                got = (a.crop_x, a.crop_y, a.crop_w, a.crop_h)
                assert got == want == box, (got, want, box)
                if apply:
                    x, y, w, h = got
                    ow, oh = min(w + x, rz.shape[1] - x), min(h + y, rz.shape[0] - y)
                    assert np.array_equal(out, rz[y:y + oh, x:x + ow]), "applied crop differs"
            ok += 1
        except AssertionError as e:
            err = err or f"image {i}: {e}"
    return ok, len(idxs), err


def verify_mixed_batch(ctx, arr, views, ops, idxs, seeds, dst_of):
    """verify_batch for a batch of mixed geometries (cfg4).  The untimed re-run
    without the crop apply covers the WHOLE batch (views / ops of every image),
    so the library makes the same per-batch kernel choices as in the timed run
    (k_rs_vr takes a batch of <= FI_VR_MAX_CLASSES vertical tables; a single
    image would always take it) and the re-run pixels are the timed run's.
    Checked for images idxs: resampled pixels within +-1 LSB of the oracle;
    with smart-crop, the record's box bit-exact with the oracle's smartcrop on
    those pixels and the applied output equal to that box of them.  seeds[i]:
    the synth_rgb seed of image i.  Returns (ok, total, first error)."""
    import numpy as np

    from flyimg_amd import _lib as L
    from flyimg_amd.runtime import Op
    from flyimg_amd.synth import synth_rgb
    from oracle import oracle as orc

    no_apply = [Op(op.target_w, op.target_h, op.flags & ~L.FI_OP_SMARTCROP_APPLY, op.gravity, op.rotate,
                   op.smartcrop_w, op.smartcrop_h) for op in ops]
    outs, recs, rc = ctx.process_device_views(views, no_apply)
    ok, err = 0, None
    for i in idxs:
        a, op = arr[i], ops[i]
        try:
            assert rc == 0 and recs[i].status == 0 and outs[i] is not None, f"re-run status {rc}/{recs[i].status}"
            assert a.status == 0, f"status {a.status}"
            p, W, H, _ = views[i]
            src = synth_rgb(W, H, seeds[i])
            ref = orc.im_convert(src, op.target_w, op.target_h, oracle_flags(op), rotate=op.rotate)
            rz = outs[i]
            assert rz.shape == ref.shape, (rz.shape, ref.shape)
            d = int(np.abs(rz.astype(np.int16) - ref.astype(np.int16)).max())
            assert d <= 1, f"max |gpu - oracle| = {d}"
            out = ctx.d2h(dst_of(i), a.out_h * a.out_stride).reshape(a.out_h, a.out_stride)
            out = out[:, : a.out_w * a.out_channels].reshape(a.out_h, a.out_w, a.out_channels)
            out = out[:, :, 0] if a.out_channels == 1 else out
            if op.flags & L.FI_OP_SMARTCROP:
                rgb = rz if rz.ndim == 3 else np.repeat(rz[:, :, None], 3, axis=2)
                t = orc.sc_crop(np.ascontiguousarray(rgb), op.smartcrop_w or 100, op.smartcrop_h or 100)["top_crop"]
                want = (t["x"], t["y"], t["width"], t["height"])
                got = (a.crop_x, a.crop_y, a.crop_w, a.crop_h)
                assert got == want, (got, want)
                if op.flags & L.FI_OP_SMARTCROP_APPLY:
                    x, y, w, h = got
                    ow, oh = min(w + x, rz.shape[1] - x), min(h + y, rz.shape[0] - y)
                    assert np.array_equal(out, rz[y:y + oh, x:x + ow]), "applied crop differs"
            else:
                assert np.array_equal(out, rz), "timed output differs from the re-run"
            ok += 1
        except AssertionError as e:
            err = err or f"image {i}: {e}"
    return ok, len(idxs), err
