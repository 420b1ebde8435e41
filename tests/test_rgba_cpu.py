"""RGBA (IM matte) sources on the CPU side: the oracle's matte restatement
(resize.c matte branch) on cases with known answers, and the planner's
output channels / refusals through the C-ABI's fi_plan (no GPU)."""
import numpy as np

from flyimg_amd import _lib as L
from oracle import oracle as orc


def _src(W, H, seed, alpha):
    rng = np.random.default_rng(seed)
    a = rng.integers(0, 256, (H, W, 4), dtype=np.uint8)
    a[..., 3] = alpha
    return a


def test_oracle_matte_opaque_keeps_alpha():
    o = orc.im_convert(_src(300, 200, 1, 255), 100, 0, orc.FLAG_THUMBNAIL)
    assert o.shape == (67, 100, 4) and (o[..., 3] == 255).all()


def test_oracle_matte_transparent_is_black():
    # every tap has alpha 0: gamma = 0 -> PerceptibleReciprocal(0) * 0 = 0
    o = orc.im_convert(_src(300, 200, 2, 0), 100, 0, orc.FLAG_THUMBNAIL)
    assert (o == 0).all()


def test_oracle_matte_uniform_colour_is_alpha_independent():
    # alpha weighting: a constant colour stays constant whatever the alpha
    a = _src(240, 180, 3, 0)
    a[..., :3] = (200, 100, 50)
    a[..., 3] = np.random.default_rng(4).integers(1, 256, (180, 240))
    o = orc.im_convert(a, 80, 0, orc.FLAG_THUMBNAIL)
    assert (np.abs(o[..., :3].astype(int) - (200, 100, 50)) <= 1).all()


def test_oracle_matte_gray_alpha():
    o = orc.im_convert(_src(240, 180, 5, 128), 80, 0, orc.FLAG_THUMBNAIL | orc.FLAG_GRAY)
    assert o.shape == (60, 80, 2) and (np.abs(o[..., 1].astype(int) - 128) <= 1).all()


def _plan(W, H, C, flags, tw=100, th=0):
    img = L.FiImage()
    img.src, img.src_w, img.src_h, img.src_stride, img.src_channels = 1, W, H, W * C, C
    img.target_w, img.target_h, img.flags, img.gravity = tw, th, flags, 5
    img.smartcrop_w = img.smartcrop_h = 100
    L.lib().fi_plan(img, 1)
    return img


def test_plan_rgba_channels_and_refusals():
    assert _plan(400, 300, 4, L.FI_OP_THUMBNAIL).out_channels == 4
    assert _plan(400, 300, 4, L.FI_OP_THUMBNAIL | L.FI_OP_GRAY).out_channels == 2
    assert _plan(400, 300, 4, L.FI_OP_THUMBNAIL | L.FI_OP_SMARTCROP).status == L.FI_EUNSUPPORTED
    assert _plan(400, 300, 4, L.FI_OP_THUMBNAIL | L.FI_OP_MONOCHROME).status == L.FI_EUNSUPPORTED
    assert _plan(400, 300, 2, L.FI_OP_THUMBNAIL).status == L.FI_EUNSUPPORTED
