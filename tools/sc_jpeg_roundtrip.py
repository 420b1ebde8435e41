#!/usr/bin/env python3
"""How often the FFI fused smart-crop box differs from the reference's.

The reference runs smartcrop.py on the JPEG file ImageMagick wrote
(SmartCropProcessor.php:24: `python smartcrop.py <output file>`); the fused
path (FI_OP_SMARTCROP) computes the box on the raw resized pixels before any
encode.  This tool measures the difference on the GPU path itself: for each
source it resizes (w_500, as cfg2), takes the box on the raw pixels and on the
same pixels after a JPEG round trip (Pillow, quality 90 -- flyimg's default
`q_90` -- with 4:4:4 sampling, ImageMagick's choice at quality >= 90, and also
4:2:0), and counts the images whose box changes.

It also checks the PHP shim's DEFAULT smc_1 path (HipSmartCropProcessor,
reference order): resize -> JPEG q90 4:2:0 (MozJPEG cjpeg's default sampling;
libjpeg-turbo through Pillow stands in for MozJPEG here) -> decode that file
-> fi_smartcrop; its box must equal the oracle's (pinned bit-exact to
smartcrop.py) on the same decoded bytes for every image ("ref_order_q90_420").

  python tools/sc_jpeg_roundtrip.py [--synthetic N] [--out file.json]

Sources: the reference's three photographs kept as fixtures under
tests/golden/ and N synthetic images (flyimg_amd.synth, four sizes)."""
import argparse
import io
import json
import os
import sys

import numpy as np
from PIL import Image

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from flyimg_amd.processor import ImageProcessor, OptionsBag  # noqa: E402
from flyimg_amd.runtime import Context  # noqa: E402
from flyimg_amd.synth import synth_rgb  # noqa: E402
from oracle import oracle as orc  # noqa: E402  (the checker)


def top_box(ctx, rgb):
    r = ctx.smartcrop_ex(rgb, 100, 100)
    c = r["crops"][r["top_index"]]
    return (c.x, c.y, c.width, c.height)


def iou(a, b):
    ax1, ay1, bx1, by1 = a[0] + a[2], a[1] + a[3], b[0] + b[2], b[1] + b[3]
    iw = max(0, min(ax1, bx1) - max(a[0], b[0]))
    ih = max(0, min(ay1, by1) - max(a[1], b[1]))
    inter = iw * ih
    return inter / float(a[2] * a[3] + b[2] * b[3] - inter)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--synthetic", type=int, default=200)
    ap.add_argument("--out", default="")
    args = ap.parse_args()
    sources = []
    for name in ("smart_crop.jpg", "extract-original.jpg", "extract-result.jpg"):
        sources.append(("fixture:" + name, np.asarray(Image.open(os.path.join(ROOT, "tests", "golden", name)).convert("RGB"))))
    sizes = [(1920, 1080), (3000, 2000), (1200, 900), (800, 600)]
    for k in range(args.synthetic):
        w, h = sizes[k % len(sizes)]
        sources.append((f"synthetic:{w}x{h}:{k}", synth_rgb(w, h, 1000 + k)))
    res = {"sources": len(sources), "options": "w_500, smartcrop 100x100 (SmartCropProcessor CLI defaults)",
           "variants": {}}
    per = []
    with Context(0) as ctx:
        for name, src in sources:
            h, w = src.shape[:2]
            op = ImageProcessor(OptionsBag("w_500"), w, h).to_op()
            outs, recs, rc = ctx.process([np.ascontiguousarray(src)], [op])
            if rc != 0 or recs[0].status != 0:
                raise SystemExit(f"{name}: resize failed ({rc})")
            resized = outs[0]
            raw = top_box(ctx, resized)
            row = {"source": name, "raw": raw}
            for tag, sub in (("q90_444", 0), ("q90_420", 2)):
                buf = io.BytesIO()
                Image.fromarray(resized).save(buf, "JPEG", quality=90, subsampling=sub)
                dec = np.asarray(Image.open(io.BytesIO(buf.getvalue())).convert("RGB"))
                row[tag] = top_box(ctx, dec)
                if tag == "q90_420":
                    t = orc.sc_crop(dec, 100, 100)["top_crop"]
                    row["ref_order_q90_420"] = (t["x"], t["y"], t["width"], t["height"])
            per.append(row)
    for tag in ("q90_444", "q90_420"):
        for group in ("fixture", "synthetic"):
            rows = [r for r in per if r["source"].startswith(group)]
            same = sum(1 for r in rows if tuple(r[tag]) == tuple(r["raw"]))
            ious = [iou(r["raw"], r[tag]) for r in rows]
            res["variants"][f"{tag}/{group}"] = {
                "images": len(rows), "same_box": same, "different_box": len(rows) - same,
                "mean_iou": round(float(np.mean(ious)), 4) if ious else None,
                "min_iou": round(float(np.min(ious)), 4) if ious else None}
    for group in ("fixture", "synthetic"):
        rows = [r for r in per if r["source"].startswith(group)]
        same = sum(1 for r in rows if tuple(r["q90_420"]) == tuple(r["ref_order_q90_420"]))
        res["variants"][f"ref_order_q90_420/{group}"] = {
            "images": len(rows), "gpu_box_equals_oracle_on_decoded_file": same,
            "encoder": "libjpeg-turbo (Pillow) q90 4:2:0 standing in for MozJPEG cjpeg -quality 90"}
    res["fixtures"] = [r for r in per if r["source"].startswith("fixture")]
    print(json.dumps(res, indent=1))
    if args.out:
        with open(args.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
