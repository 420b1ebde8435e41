"""fi_jpeg_info (host-only header parse of the GPU JPEG decoder): the streams
it takes and the ones it leaves to the host decoder."""
import io

import pytest
from PIL import Image

from flyimg_amd.runtime import jpeg_info
from flyimg_amd.synth import synth_rgb


def _enc(img, mode=None, **kw):
    b = io.BytesIO()
    im = Image.fromarray(img)
    if mode:
        im = im.convert(mode)
    im.save(b, "JPEG", **kw)
    return b.getvalue()


@pytest.mark.parametrize("ss", [0, 1, 2])
def test_jpeg_info_ycbcr(ss):
    assert jpeg_info(_enc(synth_rgb(333, 211, 1), quality=90, subsampling=ss)) == (333, 211, 3)


def test_jpeg_info_gray_and_restart():
    assert jpeg_info(_enc(synth_rgb(31, 17, 2), mode="L", quality=75)) == (31, 17, 1)
    assert jpeg_info(_enc(synth_rgb(64, 48, 3), quality=90, restart_marker_blocks=2)) == (64, 48, 3)


@pytest.mark.parametrize("kw,mode", [(dict(progressive=True), None), (dict(), "CMYK")])
def test_jpeg_info_host_fallback(kw, mode):
    """Progressive and CMYK (Adobe transform) streams: None (the host decodes them)."""
    assert jpeg_info(_enc(synth_rgb(64, 48, 4), mode=mode, quality=90, **kw)) is None


def test_jpeg_info_malformed():
    for blob in (b"", b"\xff\xd8", b"\x89PNG\r\n\x1a\n" + b"\0" * 16, b"\xff\xd8\xff\xc0\x00\x11"):
        assert jpeg_info(blob) is None
    with open("tests/golden/smart_crop.jpg", "rb") as f:  # the reference fixture is progressive
        assert jpeg_info(f.read()) is None


def _dht(tc_th, bits, vals):
    body = bytes([tc_th]) + bytes(bits) + bytes(vals)
    return b"\xff\xc4" + (len(body) + 2).to_bytes(2, "big") + body


def test_jpeg_info_oversubscribed_huffman_table_in_child():
    """a DHT with 40 codes of length 1 used to write past the
    lookahead table before the over-subscription check.  It must be rejected
    (jdhuff.c JERR_BAD_HUFF_TABLE) and the parser must not crash: run in a child
    process so a crash fails the test instead of the runner."""
    import subprocess
    import sys

    good = _enc(synth_rgb(64, 48, 5), quality=90)
    k = good.index(b"\xff\xda")  # after the encoder's own DHTs: this table is the one in force
    bad = good[:k] + _dht(0x00, [40] + [0] * 15, range(40)) + good[k:]
    code = ("import sys; sys.path.insert(0, '.');"
            "from flyimg_amd.runtime import jpeg_info;"
            "print(jpeg_info(open(sys.argv[1], 'rb').read()))")
    import tempfile

    with tempfile.NamedTemporaryFile(suffix=".jpg", delete=False) as f:
        f.write(bad)
        path = f.name
    r = subprocess.run([sys.executable, "-c", code, path], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    assert r.stdout.strip() == "None"


@pytest.mark.parametrize("bits,vals,ok", [
    ([2] + [0] * 15, [0, 1], False),       # uses the all-ones code of length 1
    ([1] + [0] * 15, [0], True),
    ([0, 3] + [0] * 14, [0, 1, 2], True),
    ([0, 4] + [0] * 14, [0, 1, 2, 3], False),
    ([1] + [0] * 15, [16], False),         # DC symbol > 15
])
def test_jpeg_info_huffman_table_rules(bits, vals, ok):
    """libjpeg's table checks: codes of each length and the code after them fit
    that length (no all-ones code), DC symbols 0..15.  A later DHT of the same
    class/id replaces the encoder's table, so the stream is judged by it."""
    blob = _enc(synth_rgb(64, 48, 6), quality=90)
    # a DC table 0 redefinition right before SOS (after the encoder's own DHTs)
    k = blob.index(b"\xff\xda")
    blob = blob[:k] + _dht(0x00, bits, vals) + blob[k:]
    info = jpeg_info(blob)
    if ok:
        # a valid table that does not match the data still parses (decode would fail)
        assert info == (64, 48, 3)
    else:
        assert info is None


@pytest.mark.parametrize("cut", [0.5, 2 / 3, 0.95])
def test_jpeg_info_truncated_goes_to_host(cut):
    """a stream without EOI at the end of its scan is left to the host
    decoder (which reports the truncation) instead of decoding zero padding."""
    blob = _enc(synth_rgb(96, 64, 7), quality=90)
    assert jpeg_info(blob) == (96, 64, 3)
    assert jpeg_info(blob[: int(len(blob) * cut)]) is None
    assert jpeg_info(blob[:-2]) is None


def test_jpeg_info_rgb_colour_space_goes_to_host():
    """libjpeg decodes Adobe-transform-0 and 'R','G','B'-id streams as
    RGB; the GPU path converts YCbCr only, so both go to the host.  The Adobe
    marker normally precedes SOF."""
    rgb = _enc(synth_rgb(80, 64, 8), quality=90, keep_rgb=True)
    assert rgb.index(b"\xff\xee") < rgb.index(b"\xff\xc0")
    assert jpeg_info(rgb) is None
    # 'R','G','B' component ids with neither JFIF nor Adobe marker
    blob = bytearray(_enc(synth_rgb(80, 64, 9), quality=90))
    assert blob[2:4] == b"\xff\xe0"
    app0_len = int.from_bytes(blob[4:6], "big")
    del blob[2:4 + app0_len]
    assert jpeg_info(bytes(blob)) == (80, 64, 3)  # ids 1, 2, 3: YCbCr
    sof = blob.index(b"\xff\xc0")
    for c, cid in enumerate(b"RGB"):
        blob[sof + 10 + 3 * c] = cid
    sos = blob.index(b"\xff\xda")
    for c, cid in enumerate(b"RGB"):
        blob[sos + 5 + 2 * c] = cid
    assert jpeg_info(bytes(blob)) is None
