"""-monochrome on the CPU: the oracle's deterministic
restatement (oracle/fi_oracle.c or_im_monochrome) against the literal
statement-by-statement restatement (tests/mono_literal.py), the Hilbert-curve
closed form against IM's recursive Riemersma walk, and the operator's
properties.  Parity with ImageMagick itself is unpinned (IM absent)."""
import numpy as np
import pytest

from oracle import oracle as orc
from tests import mono_literal as ml


@pytest.mark.parametrize("level", [1, 2, 3, 4, 5, 6])
def test_curve_closed_form_is_the_riemersma_walk(level):
    pts = ml.curve_positions(level)
    n = 1 << level
    assert len(pts) == n * n and len(set(pts)) == n * n
    assert [orc.hilbert_d2xy(level, d) for d in range(n * n)] == pts


@pytest.mark.parametrize("wh,level", [((1, 1), 1), ((2, 3), 2), ((400, 400), 9), ((512, 10), 10), ((300, 513), 10)])
def test_curve_level(wh, level):
    assert orc.mono_curve_level(*wh) == level


def _cases():
    rng = np.random.default_rng(20250112)
    out = []
    for t in range(36):
        h, w = (int(v) for v in rng.integers(1, 34, 2))
        kind = t % 4
        if kind == 0:
            g = rng.integers(0, 65536, (h, w))
        elif kind == 1:  # smooth field + noise (no exactly symmetric error ties)
            yy, xx = np.mgrid[0:h, 0:w]
            g = 30000 + 20000 * np.sin(xx / 5.0 + yy / 7.0) + rng.integers(-900, 900, (h, w))
        elif kind == 2:  # narrow range: NormalizeImage stretches it
            g = rng.integers(20000, 30000, (h, w))
        else:  # skewed histogram
            g = np.minimum(65535, (rng.random((h, w)) ** 3 * 70000).astype(np.int64))
        out.append((f"{kind}_{h}x{w}_{t}", np.clip(g, 0, 65535).astype(np.uint16)))
    return out


@pytest.mark.parametrize("name,g", _cases(), ids=[c[0] for c in _cases()])
def test_oracle_equals_literal_restatement(name, g):
    """Bit-exact against the literal restatement with the cluster sums held
    exactly (the oracle's documented reformulation; the quantize errors are
    still summed in IM's raster order there)."""
    a = orc.im_monochrome(g)
    b = ml.monochrome(g, exact_sums=True)
    assert np.array_equal(a, b), f"{name}: {(a != b).sum()} pixels differ"


def test_oracle_vs_raster_order_sums():
    """With IM's raster-order f64 colour sums, a cluster mean that lands on an
    exact .5 can round the other way (one documented case below); everything
    else is identical."""
    cases = _cases()
    same = sum(np.array_equal(orc.im_monochrome(g), ml.monochrome(g)) for _, g in cases)
    assert same >= len(cases) - 2, (same, len(cases))


def test_bilevel_input_passes_through():
    g = np.where(np.random.default_rng(3).random((20, 30)) > 0.5, 65535, 0).astype(np.uint16)
    assert np.array_equal(orc.im_monochrome(g), np.where(g > 0, 255, 0))


@pytest.mark.parametrize("v", [0, 1, 30000, 65534])
def test_uniform_image_is_one_colour(v):
    out = orc.im_monochrome(np.full((17, 23), v, np.uint16))
    assert len(np.unique(out)) == 1


def test_dither_preserves_the_mean():
    yy, xx = np.mgrid[0:120, 0:160]
    g = (65535 * (0.15 + 0.7 * xx / 159.0)).astype(np.uint16) + (yy % 3).astype(np.uint16)
    out = orc.im_monochrome(g)
    assert set(np.unique(out)) <= {0, 255}
    # NormalizeImage stretches [black, white] to [0, 65535]; the dither keeps the stretched mean
    lo, hi = np.percentile(g, [0.15, 99.95])
    s = np.clip((g.astype(np.float64) - lo) / (hi - lo), 0, 1)
    assert abs(out.mean() / 255 - s.mean()) < 0.03


def test_convert_monochrome_pipeline_and_rotate():
    rng = np.random.default_rng(9)
    src = rng.integers(0, 256, (90, 120, 3), dtype=np.uint8)
    F = orc.FLAG_THUMBNAIL | orc.FLAG_FILL | orc.FLAG_EXTENT | orc.FLAG_MONO
    a = orc.im_convert(src, 60, 50, F)
    assert a.shape == (50, 60) and set(np.unique(a)) <= {0, 255}
    r = orc.im_convert(src, 60, 50, F | orc.FLAG_ROTATE, rotate=90)
    assert np.array_equal(r, np.rot90(a, -1))
    # -colorspace Gray before -monochrome changes nothing (mono converts to GRAY itself)
    assert np.array_equal(orc.im_convert(src, 60, 50, F | orc.FLAG_GRAY), a)
