"""Derive face-blur (FaceDetectProcessor::blurFaces) data from the reference's
own fixture pair -- run in the build container, where /root/reference exists;
the GPU box never runs this.

  /root/reference/tests/testImages/faces.jpg    the input
  /root/reference/tests/testImages/face_fb.png  'fb_1,o_png,rf_1' output
                                                (FaceDetectProcessorTest.php:31-41)

face_fb.png is faces.jpg after, per detected face, `mogrify -gravity NorthWest
-region WxH+X+Y -scale 10% -scale 1000%` (FaceDetectProcessor.php:67-73).
Recovered here, as data only (no image is copied):
  * the face boxes: the rectangles where face_fb.png is exactly constant on
    10x10 blocks anchored at the box origin and equal to the decoded input
    (within the decoders' +-3 LSB) in a 2-px ring around them;
  * per box, the block grid (column / row edges) and every block's RGB value;
  * the decode noise outside the boxes (face_fb vs Pillow's decode of faces.jpg).

Writes tests/golden/face_fb.json.
"""
from __future__ import annotations

import json
import os

import numpy as np
from PIL import Image

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference/tests/testImages"


def main():
    fb = np.asarray(Image.open(os.path.join(REF, "face_fb.png")).convert("RGB")).astype(int)
    src = np.asarray(Image.open(os.path.join(REF, "faces.jpg")).convert("RGB")).astype(int)
    H, W = src.shape[:2]
    # candidate regions: where the output departs from the decoded input by > 3 LSB
    import scipy.ndimage as ndi

    mask = np.abs(fb - src).max(axis=2) > 3
    lab, n = ndi.label(ndi.binary_dilation(mask, iterations=3))
    boxes = []
    for k in range(1, n + 1):
        yy, xx = np.where(lab == k)
        # the dilation adds 3 px on each side; search the exact box around it
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
        boxes.append(best[1:])
    boxes.sort(key=lambda b: (b[1], b[0]))
    out = {"source": "derived from /root/reference/tests/testImages/face_fb.png and faces.jpg by "
                     "tests/golden/make_face_fb.py",
           "image": [W, H], "boxes": [], "outside_max_abs_diff": None}
    inside = np.zeros((H, W), bool)
    for (x, y, w, h) in boxes:
        inside[y:y + h, x:x + w] = True
        reg = fb[y:y + h, x:x + w]
        col_edges = [int(c) + 1 for c in np.where((np.abs(np.diff(reg, axis=1)).max(axis=2) > 0).any(axis=0))[0]]
        row_edges = [int(r) + 1 for r in np.where((np.abs(np.diff(reg, axis=0)).max(axis=2) > 0).any(axis=1))[0]]
        cols = [0] + col_edges + [w]
        rows = [0] + row_edges + [h]
        blocks = [[[int(v) for v in reg[rows[i], cols[j]]] for j in range(len(cols) - 1)] for i in range(len(rows) - 1)]
        out["boxes"].append({"x": int(x), "y": int(y), "w": int(w), "h": int(h),
                             "col_edges": col_edges, "row_edges": row_edges, "blocks_rgb": blocks})
    out["outside_max_abs_diff"] = int(np.abs(fb - src).max(axis=2)[~inside].max())
    with open(os.path.join(HERE, "face_fb.json"), "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps({k: v for k, v in out.items() if k != "boxes"}), [b["x"] for b in out["boxes"]])


if __name__ == "__main__":
    main()
