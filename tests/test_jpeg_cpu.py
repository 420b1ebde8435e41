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
