"""Face-blur pixelation (FaceDetectProcessor.php:67-73: mogrify -gravity
NorthWest -region WxH+X+Y -scale 10% -scale 1000%) pinned to the reference's
own fixture pair (FaceDetectProcessorTest.php:31-41): faces.jpg in,
face_fb.png out, through the data tests/golden/make_face_fb.py derived from
them (tests/golden/face_fb.json; faces.jpg is kept as tests/golden/faces.jpg).

Pinned: the block VALUES, not just the grid.  The detector's boxes are
56 x 56 @ (245,21), 51 x 51 @ (377,41), 55 x 55 @ (116,60) and 57 x 57 @
(467,76).  IM's 10 % image of a 56-px box has 6 columns, each the area
average of a 9.33-px window, and the 1000 % image (60 px) is composited at
the box origin unclipped, so the visible footprint (60 x 60, 50 x 50 for the
51-px box) is larger than the box.  The oracle's literal ScaleImage
(oracle/fi_oracle.c or_im_pixelate_regions) on Pillow's decode of faces.jpg
reproduces every block of face_fb.png within 1 LSB (max 0 / 1 / 1 / 1 per
box; the two decoders differ by <= 3 LSB outside the boxes).  The GPU kernel
is checked against the same values in tests/test_gpu_parity.py
(test_face_fb_fixture_blocks)."""
import json
import os

import numpy as np

from oracle import oracle as orc

HERE = os.path.dirname(os.path.abspath(__file__))
FB = json.load(open(os.path.join(HERE, "golden", "face_fb.json")))
DETECTOR = [(b["detector"]["x"], b["detector"]["y"], b["detector"]["w"], b["detector"]["h"]) for b in FB["boxes"]]


def faces_rgb():
    from PIL import Image

    return np.asarray(Image.open(os.path.join(HERE, "golden", "faces.jpg")).convert("RGB"))


def fixture_block_diff(out):
    """max |out - face_fb| over every block of every footprint"""
    worst = 0
    for b in FB["boxes"]:
        x, y = b["x"], b["y"]
        cols = [0] + b["col_edges"]
        rows = [0] + b["row_edges"]
        for i, r in enumerate(rows):
            for j, c in enumerate(cols):
                blk = out[y + r:y + (rows[i + 1] if i + 1 < len(rows) else b["h"]),
                          x + c:x + (cols[j + 1] if j + 1 < len(cols) else b["w"])].astype(int)
                worst = max(worst, int(np.abs(blk - np.array(b["blocks_rgb"][i][j])).max()))
    return worst


def _edges(block):
    """column / row indices where the block content changes (edge after index i -> i + 1)"""
    c = [int(i) + 1 for i in np.where((np.abs(np.diff(block.astype(int), axis=1)) > 0).reshape(block.shape[0], -1, block.shape[-1]).any(axis=(0, 2)))[0]]
    r = [int(i) + 1 for i in np.where((np.abs(np.diff(block.astype(int), axis=0)) > 0).reshape(-1, block.shape[1], block.shape[-1]).any(axis=(1, 2)))[0]]
    return c, r


def test_fixture_boxes_are_the_reference_geometry():
    W, H = FB["image"]
    assert (W, H) == (620, 349)
    assert FB["outside_max_abs_diff"] <= 3  # only the decoders differ outside the boxes
    assert [(d[2], d[3]) for d in DETECTOR] == [(56, 56), (51, 51), (55, 55), (57, 57)]
    for b, d in zip(FB["boxes"], DETECTOR):
        n_c = orc.im_percent_size(d[2], 10)
        n_r = orc.im_percent_size(d[3], 10)
        assert (d[0], d[1]) == (b["x"], b["y"])
        assert len(b["col_edges"]) == n_c - 1 and len(b["row_edges"]) == n_r - 1
        assert len(b["blocks_rgb"]) == n_r and len(b["blocks_rgb"][0]) == n_c
        # the footprint is the unclipped 1000 % image, not the detector box
        assert orc.im_percent_size(n_c, 1000) == b["w"] and orc.im_percent_size(n_r, 1000) == b["h"]


def test_oracle_block_grid_matches_face_fb():
    W, H = FB["image"]
    rng = np.random.default_rng(3)
    img = rng.integers(0, 256, (H, W, 3), dtype=np.uint8)  # every window mean distinct
    out = orc.im_pixelate_regions(img, DETECTOR)
    mask = np.ones((H, W), bool)
    for b in FB["boxes"]:
        x, y, w, h = b["x"], b["y"], b["w"], b["h"]
        mask[y:y + h, x:x + w] = False
        c, r = _edges(out[y:y + h, x:x + w])
        assert c == b["col_edges"] and r == b["row_edges"], (b["x"], c, r)
    assert np.array_equal(out[mask], img[mask])  # nothing outside the footprints changes


def test_oracle_reproduces_face_fb_blocks():
    """the pin: the oracle's ScaleImage on faces.jpg with the detector boxes
    gives every block of the reference's face_fb.png within 1 LSB"""
    src = faces_rgb()
    assert src.shape == (349, 620, 3)
    out = orc.im_pixelate_regions(src, DETECTOR)
    assert fixture_block_diff(out) <= 1
