"""GPU JPEG decode (fi_jpeg.hip) against libjpeg-turbo through Pillow 12.2.0
(the host codec path's decoder, codec.decode_ex): bit-exact on every pixel
for 4:4:4 / 4:2:2 / 4:2:0 / gray streams, odd and tiny sizes, qualities,
optimised Huffman tables, restart intervals; unsupported streams come back
with FI_EUNSUPPORTED while the rest of the batch decodes."""
import io

import numpy as np
import pytest
from PIL import Image

from flyimg_amd import _lib as L
from flyimg_amd.runtime import Context, jpeg_info
from flyimg_amd.synth import synth_rgb

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    c = Context(0)
    yield c
    c.close()


def _enc(img, **kw):
    b = io.BytesIO()
    Image.fromarray(img).save(b, "JPEG", **kw)
    return b.getvalue()


def _ref(blob):
    return np.asarray(Image.open(io.BytesIO(blob)))


def _noise(w, h, seed):
    return np.random.default_rng(seed).integers(0, 256, (h, w, 3), dtype=np.uint8)


CASES = []
for ss in (0, 1, 2):
    for (w, h) in ((1, 1), (7, 9), (17, 33), (16, 16), (333, 211), (640, 481)):
        CASES.append((f"ss{ss}_{w}x{h}", w, h, dict(quality=90, subsampling=ss)))
CASES += [
    ("ss2_q50", 300, 200, dict(quality=50, subsampling=2)),
    ("ss2_q100", 300, 200, dict(quality=100, subsampling=2)),
    ("ss0_q100", 123, 77, dict(quality=100, subsampling=0)),
    ("ss2_optimize", 301, 199, dict(quality=85, subsampling=2, optimize=True)),
    ("ss2_restart_blocks", 250, 130, dict(quality=90, subsampling=2, restart_marker_blocks=5)),
    ("ss0_restart_rows", 97, 61, dict(quality=90, subsampling=0, restart_marker_rows=1)),
    ("ss1_restart_1", 65, 33, dict(quality=75, subsampling=1, restart_marker_blocks=1)),
    ("ss2_1920x1080", 1920, 1080, dict(quality=90, subsampling=2)),
]


@pytest.mark.parametrize("name,w,h,kw", CASES, ids=[c[0] for c in CASES])
def test_jpeg_decode_bit_exact(ctx, name, w, h, kw):
    blob = _enc(synth_rgb(w, h, 11 + w + h), **kw)
    assert jpeg_info(blob) == (w, h, 3)
    got = ctx.jpeg_decode_host([blob])[0]
    ref = _ref(blob)
    assert got is not None and got.shape == ref.shape
    assert np.array_equal(got, ref), f"{name}: {(got != ref).sum()} of {ref.size} values differ"


@pytest.mark.parametrize("ss", [0, 2])
def test_jpeg_decode_noise_bit_exact(ctx, ss):
    """Uniform noise: long AC runs, large coefficients, 0xFF stuffing everywhere."""
    blob = _enc(_noise(211, 157, ss), quality=97, subsampling=ss)
    got = ctx.jpeg_decode_host([blob])[0]
    assert np.array_equal(got, _ref(blob))


@pytest.mark.parametrize("w,h,q", [(1, 1, 90), (33, 17, 75), (500, 281, 90), (97, 61, 30)])
def test_jpeg_decode_gray_bit_exact(ctx, w, h, q):
    blob = _enc(synth_rgb(w, h, 3)[..., 1].copy(), quality=q)
    assert jpeg_info(blob) == (w, h, 1)
    got = ctx.jpeg_decode_host([blob])[0]
    ref = _ref(blob)
    assert got.shape == ref.shape and np.array_equal(got, ref)


def test_jpeg_decode_gray_as_rgb(ctx):
    """out_channels=3: a gray stream comes out with its luma in all three
    channels (Image.convert("RGB") of the decode), a YCbCr one unchanged."""
    blobs = [_enc(synth_rgb(57, 43, 6)[..., 2].copy(), quality=85), _enc(synth_rgb(57, 43, 7), quality=85)]
    ptrs = [ctx.malloc(57 * 43 * 3) for _ in blobs]
    try:
        assert ctx.jpeg_decode(blobs, ptrs, [57 * 3] * 2, channels=3) == [0, 0]
        got = [ctx.d2h(p, 57 * 43 * 3).reshape(43, 57, 3) for p in ptrs]
    finally:
        for p in ptrs:
            ctx.free(p)
    for g, b in zip(got, blobs):
        assert np.array_equal(g, np.asarray(Image.open(io.BytesIO(b)).convert("RGB")))


def test_jpeg_decode_batch_mixed_with_unsupported(ctx):
    """One call: several geometries and samplings; a progressive and a CMYK
    stream get FI_EUNSUPPORTED (host decode) and the others are exact."""
    blobs = [
        _enc(synth_rgb(120, 80, 1), quality=90, subsampling=2),
        _enc(synth_rgb(64, 64, 2), quality=90, progressive=True),
        _enc(synth_rgb(31, 45, 3), quality=80, subsampling=0),
        _enc_cmyk(synth_rgb(40, 30, 4)),
        _enc(synth_rgb(77, 55, 5)[..., 0].copy(), quality=60),
    ]
    outs = ctx.jpeg_decode_host(blobs)
    assert outs[1] is None and outs[3] is None
    for i in (0, 2, 4):
        assert np.array_equal(outs[i], _ref(blobs[i])), i


def _enc_cmyk(img):
    b = io.BytesIO()
    Image.fromarray(img).convert("CMYK").save(b, "JPEG", quality=90)
    return b.getvalue()


def test_jpeg_decode_status_codes(ctx):
    blobs = [_enc(synth_rgb(20, 20, 1), quality=90, progressive=True), b"\xff\xd8\xff\xd9garbage",
             _enc(synth_rgb(20, 20, 2), quality=90)]
    n = len(blobs)
    ptrs = [ctx.malloc(20 * 20 * 3) for _ in range(n)]
    try:
        st = ctx.jpeg_decode(blobs, ptrs, [60] * n)
    finally:
        for p in ptrs:
            ctx.free(p)
    assert st[0] == L.FI_EUNSUPPORTED and st[1] == L.FI_EINVAL and st[2] == L.FI_OK


def test_jpeg_decode_then_resize_matches_host_decode(ctx):
    """The decoded device image feeds the resample path: same output as
    decoding on the host and uploading (fi_process_batch)."""
    from flyimg_amd.processor import ImageProcessor, OptionsBag

    blob = _enc(synth_rgb(640, 360, 8), quality=90, subsampling=2)
    w, h, c = jpeg_info(blob)
    src = ctx.malloc(w * h * 3)
    try:
        assert ctx.jpeg_decode([blob], [src], [w * 3]) == [0]
        op = ImageProcessor(OptionsBag("w_200,smc_1"), w, h).to_op()
        dev_img = ctx.d2h(src, w * h * 3).reshape(h, w, 3)
    finally:
        ctx.free(src)
    outs_a, recs_a, rc_a = ctx.process([dev_img], [op])
    outs_b, recs_b, rc_b = ctx.process([_ref(blob)], [op])
    assert rc_a == rc_b == 0
    assert np.array_equal(outs_a[0], outs_b[0])


def test_codec_pipeline_gpu_decode_equals_host_decode(ctx):
    """CodecPipeline.process with the GPU decoder (baseline JPEGs decoded into
    device memory) returns byte-identical encoded outputs and the same records
    as the host-decode pipeline, on a mixed batch: 4:2:0 / 4:4:4 JPEGs, a gray
    JPEG (PseudoClass: Mitchell), an extract, a progressive JPEG, an
    EXIF-rotated JPEG and a PNG (the last four decode on the host)."""
    from flyimg_amd.codec import CodecPipeline, gpu_decodable

    rot = io.BytesIO()
    im = Image.fromarray(synth_rgb(300, 200, 9))
    ex = im.getexif()
    ex[0x0112] = 6
    im.save(rot, "JPEG", quality=90, exif=ex.tobytes())
    png = io.BytesIO()
    Image.fromarray(synth_rgb(320, 240, 10)).save(png, "PNG")
    blobs = [
        _enc(synth_rgb(1280, 720, 1), quality=90, subsampling=2),
        _enc(synth_rgb(999, 555, 2), quality=85, subsampling=0),
        _enc(synth_rgb(800, 600, 3), quality=90, subsampling=2),
        _enc(synth_rgb(640, 480, 4), quality=90, progressive=True),
        rot.getvalue(),
        png.getvalue(),
        _enc(synth_rgb(720, 480, 11)[..., 1].copy(), quality=90),
    ]
    opts = ["w_500,smc_1,q_90", "w_300,h_250,c_1", "e_1,p1x_100,p1y_50,p2x_700,p2y_450,w_200",
            "w_200,h_200,c_1", "w_150", "w_100,q_80", "w_300,h_200,c_1"]
    assert [gpu_decodable(b) is not None for b in blobs] == [True, True, True, False, False, False, True]
    res = {}
    for gd in (True, False):
        pipe = CodecPipeline(ctx, threads=4, gpu_decode=gd)
        try:
            res[gd] = pipe.process(blobs, opts)
        finally:
            pipe.close()
    (ea, ra), (eb, rb) = res[True], res[False]
    assert ea == eb
    key = ("out_w", "out_h", "crop_x", "crop_y", "crop_w", "crop_h", "status")
    assert [[getattr(r, k) for k in key] for r in ra] == [[getattr(r, k) for k in key] for r in rb]


def test_jpeg_decode_batch_beyond_2_32_pixels(ctx):
    """2100 1080p images (4.35 G pixels, 13 GB of output) in one call: the
    per-pixel and per-block kernels stride over the batch (a dispatch's
    work-item count is 32-bit), so images past 2^32 pixels decode too."""
    W, H, N = 1920, 1080, 2100
    blob = _enc(synth_rgb(W, H, 5), quality=90, subsampling=2)
    ref = _ref(blob)
    stride = W * 3
    base = ctx.malloc(stride * H * N)
    try:
        st = ctx.jpeg_decode([blob] * N, [base + i * stride * H for i in range(N)], [stride] * N)
        assert st == [0] * N
        for i in (0, 1000, 2069, N - 1):
            assert np.array_equal(ctx.d2h(base + i * stride * H, stride * H).reshape(H, W, 3), ref), i
    finally:
        ctx.free(base)
