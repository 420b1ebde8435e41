"""Derive face-blur (FaceDetectProcessor::blurFaces) data from the reference's
own fixture pair -- run in the build container, where /root/reference exists;
the GPU box never runs this.

  /root/reference/tests/testImages/faces.jpg    the input (copied as the
                                                fixture tests/golden/faces.jpg)
  /root/reference/tests/testImages/face_fb.png  'fb_1,o_png,rf_1' output
                                                (FaceDetectProcessorTest.php:31-41)

face_fb.png is faces.jpg after, per detected face, `mogrify -gravity NorthWest
-region WxH+X+Y -scale 10% -scale 1000%` (FaceDetectProcessor.php:67-73).
IM crops the w x h region, ScaleImage's it to im_percent_size(w, 10) columns
(area averages over w / n-px windows), scales that back up by 1000 % and
composites the result at the region origin, NOT clipped to the region: a
56-px box becomes a 6 x 6 block image of 60 x 60 px whose blocks average
9.33-px windows.  So the visible footprint is not the detector's box.

Recovered here, as data only:
  * the footprints: rectangles where face_fb.png is constant on 10 x 10 blocks
    anchored at their origin and equal to the decoded input (within the
    decoders' +-3 LSB) in a 2-px ring around them;
  * the DETECTOR box (x, y, w, h) behind each footprint: the box near the
    footprint origin whose pixelation (the oracle's literal ScaleImage,
    oracle/fi_oracle.c or_im_pixelate_regions) of Pillow's decode of faces.jpg
    reproduces the footprint's blocks best -- 56, 51, 55 and 57 px;
  * per footprint, the block grid (column / row edges) and every block's RGB;
  * the decode noise outside the footprints (face_fb vs Pillow's decode).

Writes tests/golden/face_fb.json.
"""
from __future__ import annotations

import json
import os
import sys

import numpy as np
from PIL import Image

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference/tests/testImages"


def footprints(fb, src):
    import scipy.ndimage as ndi

    mask = np.abs(fb - src).max(axis=2) > 3
    lab, n = ndi.label(ndi.binary_dilation(mask, iterations=3))
    out = []
    for k in range(1, n + 1):
        yy, xx = np.where(lab == k)
        # the dilation adds 3 px on each side; search the exact footprint around it
        x0, y0 = xx.min() + 3, yy.min() + 3
        w0 = xx.max() - xx.min() + 1 - 6
        best = None
        for x in range(x0 - 4, x0 + 5):
            for y in range(y0 - 4, y0 + 5):
                for w in range(w0 - 3, w0 + 4):
                    h = w
                    reg = fb[y:y + h, x:x + w]
                    err = sum(int(np.abs(reg[by:by + 10, bx:bx + 10] - reg[by, bx]).sum())
                              for by in range(0, h, 10) for bx in range(0, w, 10))
                    ring = np.abs(fb[y - 2:y + h + 2, x - 2:x + w + 2] - src[y - 2:y + h + 2, x - 2:x + w + 2]).max(axis=2)
                    ring[2:-2, 2:-2] = 0
                    score = err + 1000 * int((ring > 3).sum())
                    if best is None or score < best[0]:
                        best = (score, x, y, w, h)
        assert best[0] == 0, best
        out.append(best[1:])
    out.sort(key=lambda b: (b[1], b[0]))
    return out


def block_values(img, x, y, w, h):
    """the value of every 10 x 10 block of the footprint at (x, y)"""
    return np.array([[img[y + 10 * i, x + 10 * j] for j in range(w // 10)] for i in range(h // 10)], dtype=int)


def detector_box(fb, src_u8, fx, fy, fw, fh):
    """the detector box whose pixelation reproduces the footprint: its origin is
    the footprint's, its size s has im_percent_size(s, 10) = fw / 10 blocks"""
    from oracle import oracle as orc

    want = block_values(fb, fx, fy, fw, fh)
    best = None
    for w in range(fw - 14, fw + 5):
        for h in range(fh - 14, fh + 5):
            if orc.im_percent_size(w, 10) * 10 != fw or orc.im_percent_size(h, 10) * 10 != fh:
                continue
            out = orc.im_pixelate_regions(src_u8, [(fx, fy, w, h)]).astype(int)
            d = np.abs(block_values(out, fx, fy, fw, fh) - want)
            key = (float(d.mean()), int(d.max()), w, h)
            if best is None or key < best:
                best = key
    return best


def main():
    sys.path.insert(0, REPO)
    fb = np.asarray(Image.open(os.path.join(REF, "face_fb.png")).convert("RGB")).astype(int)
    src_u8 = np.asarray(Image.open(os.path.join(REF, "faces.jpg")).convert("RGB"))
    src = src_u8.astype(int)
    H, W = src.shape[:2]
    out = {"source": "derived from /root/reference/tests/testImages/face_fb.png and faces.jpg by "
                     "tests/golden/make_face_fb.py",
           "image": [W, H], "boxes": [], "outside_max_abs_diff": None}
    inside = np.zeros((H, W), bool)
    for (x, y, w, h) in footprints(fb, src):
        inside[y:y + h, x:x + w] = True
        reg = fb[y:y + h, x:x + w]
        col_edges = [int(c) + 1 for c in np.where((np.abs(np.diff(reg, axis=1)).max(axis=2) > 0).any(axis=0))[0]]
        row_edges = [int(r) + 1 for r in np.where((np.abs(np.diff(reg, axis=0)).max(axis=2) > 0).any(axis=1))[0]]
        cols = [0] + col_edges + [w]
        rows = [0] + row_edges + [h]
        blocks = [[[int(v) for v in reg[rows[i], cols[j]]] for j in range(len(cols) - 1)] for i in range(len(rows) - 1)]
        mean_d, max_d, dw, dh = detector_box(fb, src_u8, x, y, w, h)
        out["boxes"].append({"x": int(x), "y": int(y), "w": int(w), "h": int(h),
                             "detector": {"x": int(x), "y": int(y), "w": int(dw), "h": int(dh),
                                          "oracle_block_mean_abs_diff": round(mean_d, 4),
                                          "oracle_block_max_abs_diff": max_d},
                             "col_edges": col_edges, "row_edges": row_edges, "blocks_rgb": blocks})
    out["outside_max_abs_diff"] = int(np.abs(fb - src).max(axis=2)[~inside].max())
    with open(os.path.join(HERE, "face_fb.json"), "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps({k: v for k, v in out.items() if k != "boxes"}),
          [(b["detector"]["w"], b["detector"]["h"], b["detector"]["oracle_block_max_abs_diff"]) for b in out["boxes"]])


if __name__ == "__main__":
    main()
