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


def _scale_literal(q, ow, oh):
    """IM 6 ScaleImage (resize.c) in plain Python loops, opaque HWC, f64 --
    a second restatement the C oracle is checked against (small sizes)."""
    import numpy as np

    H, W, C = q.shape
    if ow == W and oh == H:
        return q.copy()
    out = np.zeros((oh, ow, C), np.uint16)
    xv = [[0.0] * C for _ in range(W)]
    yv = [[0.0] * C for _ in range(W)]
    clamp = lambda v: 0 if v <= 0.0 else 65535 if v >= 65535.0 else int(v + 0.5)  # noqa: E731
    nrows, nxt, i = 0, True, 0
    span_y, scale_y = 1.0, oh / H
    for y in range(oh):
        if oh == H:
            s = [[float(v) for v in q[i, x]] for x in range(W)]
            i += 1
        else:
            while scale_y < span_y:
                if nxt and nrows < H:
                    xv = [[float(v) for v in q[i, x]] for x in range(W)]
                    i += 1
                    nrows += 1
                for x in range(W):
                    for c in range(C):
                        yv[x][c] += scale_y * xv[x][c]
                span_y -= scale_y
                scale_y = oh / H
                nxt = True
            if nxt and nrows < H:
                xv = [[float(v) for v in q[i, x]] for x in range(W)]
                i += 1
                nrows += 1
                nxt = False
            s = [[yv[x][c] + span_y * xv[x][c] for c in range(C)] for x in range(W)]
            yv = [[0.0] * C for _ in range(W)]
            scale_y -= span_y
            if scale_y <= 0:
                scale_y = oh / H
                nxt = True
            span_y = 1.0
        if ow == W:
            out[y] = [[clamp(v) for v in px] for px in s]
            continue
        pixel = [0.0] * C
        nc, t, span_x = False, 0, 1.0
        sc = [[0.0] * C for _ in range(ow)]
        for x in range(W):
            scale_x = ow / W
            while scale_x >= span_x:
                if nc:
                    pixel = [0.0] * C
                    t += 1
                pixel = [pixel[c] + span_x * s[x][c] for c in range(C)]
                sc[t] = list(pixel)
                scale_x -= span_x
                span_x = 1.0
                nc = True
            if scale_x > 0:
                if nc:
                    pixel = [0.0] * C
                    nc = False
                    t += 1
                pixel = [pixel[c] + scale_x * s[x][c] for c in range(C)]
                span_x -= scale_x
        if span_x > 0:
            pixel = [pixel[c] + span_x * s[W - 1][c] for c in range(C)]
        if not nc and t < ow:
            sc[t] = list(pixel)
        out[y] = [[clamp(v) for v in px] for px in sc]
    return out


def test_scale_image_oracle_matches_literal_loops():
    """or_im_scale_q16 == a plain-Python restatement of ScaleImage on down,
    up and mixed scales; 1000% of a 10% image is pixel replication."""
    import numpy as np

    from oracle import oracle as orc

    rng = np.random.default_rng(7)
    for (W, H), (ow, oh) in [((57, 40), (6, 4)), ((23, 17), (2, 2)), ((6, 4), (60, 40)), ((31, 9), (7, 20)),
                             ((40, 40), (40, 13)), ((13, 40), (5, 40)), ((9, 9), (1, 1))]:
        q = (rng.integers(0, 256, (H, W, 3)) * 257).astype(np.uint16)
        assert np.array_equal(orc.im_scale_q16(q, ow, oh), _scale_literal(q, ow, oh)), (W, H, ow, oh)
    d = orc.im_scale_q16((rng.integers(0, 256, (40, 57, 3)) * 257).astype(np.uint16), 6, 4)
    assert np.array_equal(orc.im_scale_q16(d, 60, 40), np.repeat(np.repeat(d, 10, 0), 10, 1))


def test_pixelate_regions_oracle_semantics():
    """-region box -scale 10% -scale 1000%: only the box (and, when 10 x the
    10% size exceeds the box, up to that many pixels right / below it) changes;
    the box becomes 10x10 blocks; sizes follow ParseMetaGeometry's rounding."""
    import numpy as np

    from oracle import oracle as orc

    assert (orc.im_percent_size(57, 10.0), orc.im_percent_size(55, 10.0), orc.im_percent_size(54, 10.0)) == (6, 6, 5)
    rng = np.random.default_rng(3)
    img = rng.integers(0, 256, (100, 120, 3), dtype=np.uint8)
    out = orc.im_pixelate_regions(img, [(10, 20, 57, 40)])
    changed = np.argwhere((out != img).any(axis=2))
    assert changed[:, 0].min() >= 20 and changed[:, 0].max() < 20 + 40
    assert changed[:, 1].min() >= 10 and changed[:, 1].max() < 10 + 60  # 10% = 6 -> 60 px wide
    blk = out[20:60, 10:70]
    assert np.array_equal(blk, np.repeat(np.repeat(blk[::10, ::10], 10, 0), 10, 1))
    with pytest.raises(ValueError):
        orc.im_pixelate_regions(img, [(0, 0, 4, 40)])  # 10% of 4 px is empty
