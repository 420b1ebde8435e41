"""CPU: pin the oracle (oracle/fi_oracle.c) against the golden vectors.

smartcrop.py half: bit-exact against vectors produced by the reference module
(tests/golden/make_golden.py).  ImageMagick half: geometry against the
reference's 68 ImageProcessorTest known answers; pixel values are parity
unpinned (ImageMagick absent) and are checked only for internal properties.
"""
import numpy as np
import pytest

from oracle import oracle as orc
from tests import _golden as G

SC = G.load("smartcrop_golden.json")


def _check_result(res, ref):
    assert len(res["crops"]) == len(ref["crops"])
    for c, r in zip(res["crops"], ref["crops"]):
        assert [c["x"], c["y"], c["width"], c["height"]] == r[:4]
        s = c["score"]
        assert [s["detail"].hex(), s["saturation"].hex(), s["skin"].hex(), s["total"].hex()] == r[4:]
    assert res["top_index"] == ref["top_index"]
    assert orc.sc_geometry_string(res) == ref["geometry"]
    assert list(res["analyse_size"]) == ref["analyse_size"]


@pytest.mark.parametrize("case", SC["cases"], ids=[c["name"] for c in SC["cases"]])
def test_smartcrop_oracle_matches_reference(case):
    arr = G.case_input(case)
    res = orc.sc_crop(arr, *case["target"])
    assert res["prescale"].hex() == case["prescale"]
    assert G.sha(res["prescaled"]) == case["prescaled_sha256"]
    assert G.sha(res["maps"]) == case["maps_sha256"]
    L, _, _, _ = orc.sc_maps(res["prescaled"])
    assert G.sha(L) == case["L_sha256"]
    _check_result(res, case)


def test_smartcrop_oracle_reference_fixture():
    """SmartCropProcessorTest.php:16-24: smart_crop.jpg -> 674x674 result."""
    g = SC["fixture"]
    arr = G.fixture_input()
    res = orc.sc_crop(arr, 100, 100)
    _check_result(res, g)
    t = res["top_crop"]
    assert f"{t['width']}x{t['height']}" == g["expected_result_dims"] == "674x674"


def test_smartcrop_oracle_nonsquare_target():
    g = SC["nonsquare_target"]
    from flyimg_amd.synth import synth_rgb

    arr = synth_rgb(g["w"], g["h"], g["seed"])
    res = orc.sc_crop(arr, *g["target"])
    _check_result(res, g)


def test_pillow_primitives_match_golden():
    P = G.load("pillow_golden.json")
    from flyimg_amd.synth import synth_rgb

    base = synth_rgb(257, 193, P["base_seed"])
    assert G.sha(base) == P["base_sha256"]
    for c in P["cases"]:
        if c["op"] == "reduce":
            out = orc.pil_reduce(base, c["fx"], c["fy"])
        elif c["op"] == "resample":
            out = orc.pil_resample(base, c["ow"], c["oh"], c["box"])
        else:
            src = synth_rgb(c["W"], c["H"], c["seed"])
            out = orc.pil_thumbnail(src, c["tx"], c["ty"])
        assert list(out.shape) == c["shape"], c
        assert G.sha(out) == c["sha256"], c


def test_luma_exhaustive_2pow24():
    """convert("L", Rec709) restatement over every RGB value."""
    P = G.load("pillow_golden.json")
    v = np.arange(1 << 24, dtype=np.uint32)
    rgb = np.stack([(v >> 16) & 255, (v >> 8) & 255, v & 255], -1).astype(np.uint8).reshape(4096, 4096, 3)
    L, _, _, _ = orc.sc_maps(rgb)
    assert G.sha(L) == P["luma_table_sha256"]


GEOM = G.load("im_geometry_cases.json")


@pytest.mark.parametrize("case", GEOM, ids=[f"{c['options']}@{c['fixture']}" for c in GEOM])
def test_im_geometry_known_answers(case):
    """Oracle's ParseMetaGeometry + extent + pns clamp vs ImageProcessorTest."""
    opts = dict(kv.split("_", 1) for kv in case["options"].split(","))
    W, H = case["src_w"], case["src_h"]
    w, h = int(opts.get("w", 0) or 0), int(opts.get("h", 0) or 0)
    crop = "c" in opts
    if w and h and crop:
        # updateTargetDimensions (pns=1 default): clamp to source dims
        w, h = min(w, W), min(h, H)
        ow, oh = orc.im_meta_geometry(W, H, w, h, fill=True)
        assert ow >= w and oh >= h
        ow, oh = w, h  # -extent WxH
    else:
        ow, oh = orc.im_meta_geometry(W, H, w, h, shrink_only=True)
    assert f"{ow}x{oh}" == case["expected"]


def test_im_convert_properties():
    """Parity-unpinned IM restatement: internal consistency only."""
    from flyimg_amd.synth import synth_rgb

    src = synth_rgb(300, 200, 99)
    # identity geometry is an exact copy (ResizeImage clone path)
    out = orc.im_convert(src, 300, 200, orc.FLAG_THUMBNAIL | orc.FLAG_SHRINK)
    assert np.array_equal(out, src)
    # constant image stays constant through Lanczos (normalised weights)
    flat = np.full((200, 300, 3), 77, np.uint8)
    out = orc.im_convert(flat, 120, 0, orc.FLAG_THUMBNAIL | orc.FLAG_SHRINK)
    assert out.shape == (80, 120, 3) and np.all(out == 77)
    # rotate 90 of a c_1 crop == np.rot90 clockwise of the unrotated crop
    a = orc.im_convert(src, 100, 90, orc.FLAG_THUMBNAIL | orc.FLAG_FILL | orc.FLAG_EXTENT)
    b = orc.im_convert(src, 100, 90, orc.FLAG_THUMBNAIL | orc.FLAG_FILL | orc.FLAG_EXTENT | orc.FLAG_ROTATE, rotate=90)
    assert a.shape == (90, 100, 3)
    assert np.array_equal(b, np.rot90(a, k=-1))
    g = orc.im_convert(src, 100, 90, orc.FLAG_THUMBNAIL | orc.FLAG_FILL | orc.FLAG_EXTENT | orc.FLAG_GRAY)
    assert g.shape == (90, 100)


def test_im_sample_pre_step_geometry():
    """ThumbnailImage takes the 5x sample pre-step on every BASELINE config."""
    for (W, H, rw, rh, fill) in [(3000, 2000, 300, 250, True), (1920, 1080, 500, 0, False),
                                 (3840, 2160, 512, 512, True), (6000, 4000, 400, 400, True)]:
        ow, oh = orc.im_meta_geometry(W, H, rw, rh, fill=fill, shrink_only=not fill)
        assert orc.lib().or_im_thumbnail_uses_sample(W, H, ow, oh) == 1
    assert orc.im_meta_geometry(1920, 1080, 500, 0, shrink_only=True) == (500, 281)
    assert orc.im_meta_geometry(3840, 2160, 512, 512, fill=True) == (910, 512)


def test_pseudoclass_flag_selects_mitchell():
    """FLAG_PSEUDOCLASS: ResizeImage's filter rule for PseudoClass sources
    (resize.c): the downscale equals the Mitchell result an enlargement-free
    matte-free image otherwise never gets, and differs from Lanczos."""
    import numpy as np

    from flyimg_amd.synth import synth_rgb
    from oracle import oracle as orc

    src = synth_rgb(320, 240, 9)
    base = orc.FLAG_THUMBNAIL | orc.FLAG_SHRINK
    m = orc.im_convert(src, 100, 0, base | orc.FLAG_PSEUDOCLASS)
    lz = orc.im_convert(src, 100, 0, base)
    assert m.shape == lz.shape == (75, 100, 3)
    assert np.abs(m.astype(int) - lz.astype(int)).max() > 1
    # an RGBA (matte) source already takes Mitchell: the flag changes nothing there
    rgba = np.dstack([src, np.full(src.shape[:2], 255, np.uint8)])
    a = orc.im_convert(rgba, 100, 0, base)
    b = orc.im_convert(rgba, 100, 0, base | orc.FLAG_PSEUDOCLASS)
    assert np.array_equal(a, b)
