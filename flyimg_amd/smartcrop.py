"""Drop-in for the reference's python/smartcrop.py, backed by libflyimg_hip.

Same public names and argument meaning (SmartCrop(**kwargs).crop(image, width,
height, prescale, max_scale, min_scale, scale_step, step) -> dict with
"analyse_image", "crops", "top_crop"; CLI ``INPUT_FILE [--width --height]``
printing ``"%sx%s+%s+%s" % (w + x, h + y, x, y)``), reference
python/smartcrop.py:37-377.  The pixel work (prescale, maps, scoring, argmax)
runs on the GPU through ``fi_smartcrop_ex``; decode stays on the host (Pillow).

Differences from the reference, deliberate:
  * the CLI writes exactly one line to stdout and nothing to stderr on success
    (the reference's mode-conversion notice, smartcrop.py:358-362, lands in the
    PHP caller's output[0] through ``2>&1`` and corrupts the geometry);
  * ``analyse()`` (crop dims given directly, no prescale) is not exposed.
"""
from __future__ import annotations

import argparse
import ctypes
import sys

import numpy as np

from . import _lib as L

_ctx = None


def _context():
    global _ctx
    if _ctx is None:
        from .runtime import Context

        _ctx = Context(0)
    return _ctx


class SmartCrop(object):
    DEFAULT_SKIN_COLOR = [0.78, 0.57, 0.44]

    def __init__(self, detail_weight=0.2, edge_radius=0.4, edge_weight=-10, outside_importance=-0.5,
                 rule_of_thirds=True, saturation_bias=0.2, saturation_brightness_max=0.9,
                 saturation_brightness_min=0.05, saturation_threshold=0.4, saturation_weight=0.3,
                 score_down_sample=1, skin_bias=0.01, skin_brightness_max=1, skin_brightness_min=0.2,
                 skin_color=None, skin_threshold=0.8, skin_weight=1.8):
        p = L.FiSmartcropParams()
        p.detail_weight, p.edge_radius, p.edge_weight = detail_weight, edge_radius, edge_weight
        p.outside_importance, p.rule_of_thirds = outside_importance, int(bool(rule_of_thirds))
        p.saturation_bias = saturation_bias
        p.saturation_brightness_max, p.saturation_brightness_min = saturation_brightness_max, saturation_brightness_min
        p.saturation_threshold, p.saturation_weight = saturation_threshold, saturation_weight
        p.score_down_sample = int(score_down_sample)
        p.skin_bias, p.skin_brightness_max, p.skin_brightness_min = skin_bias, skin_brightness_max, skin_brightness_min
        color = skin_color or self.DEFAULT_SKIN_COLOR
        for i in range(3):
            p.skin_color[i] = color[i]
        p.skin_threshold, p.skin_weight = skin_threshold, skin_weight
        self.params = p

    def crop(self, image, width, height, prescale=True, max_scale=1, min_scale=0.9, scale_step=0.1, step=8,
             exact_scores=True):
        """smartcrop.py:137-191.  ``image`` is an RGB PIL image or an HxWx3
        uint8 array.  exact_scores=False returns the bounded fast-pass score
        for crops that cannot win (the top crop is exact either way)."""
        arr = np.asarray(image)
        if arr.ndim != 3 or arr.shape[2] != 3:
            # the reference unpacks image.split() into r, g, b (:17, :251)
            raise ValueError("smartcrop expects an RGB image")
        o = L.FiSmartcropOptions()
        o.prescale, o.max_scale, o.min_scale = int(bool(prescale)), max_scale, min_scale
        o.scale_step, o.step, o.exact_all = scale_step, int(step), int(bool(exact_scores))
        try:
            r = _context().smartcrop_ex(arr, int(width), int(height), self.params, o, want_images=True)
        except L.FiError as e:
            if e.code == L.FI_ENOCROP:
                raise ValueError(str(e)) from None
            raise
        crops = []
        for c in r["crops"]:
            crops.append({"x": c.x, "y": c.y, "width": c.width, "height": c.height,
                          "score": {"detail": c.detail, "saturation": c.saturation, "skin": c.skin,
                                    "total": c.total}})
        try:
            import PIL.Image

            analyse = PIL.Image.fromarray(np.ascontiguousarray(r["maps"]), "RGB")
        except ImportError:  # pragma: no cover
            analyse = r["maps"]
        return {"analyse_image": analyse, "crops": crops, "top_crop": crops[r["top_index"]]}


def parse_argument(argv=None):
    parser = argparse.ArgumentParser()
    parser.add_argument("inputfile", metavar="INPUT_FILE", help="Input image file")
    parser.add_argument("--width", dest="width", type=int, default=100, help="Crop width")
    parser.add_argument("--height", dest="height", type=int, default=100, help="Crop height")
    return parser.parse_args(argv)


def main(argv=None) -> int:
    """smartcrop.py:353-377 (target = 100 x int(height / width * 100))."""
    import PIL.Image

    options = parse_argument(argv)
    image = PIL.Image.open(options.inputfile)
    if image.mode not in ("RGB", "RGBA"):
        # the reference prints "<path> convert from mode='L' to mode='RGB' " here
        # (smartcrop.py:357-362, no newline); SmartCropProcessor.php:24-29 runs the
        # command with 2>&1 and reads output[0] as the -crop geometry, so the note
        # would corrupt it.  Deliberately not reproduced: nothing on stderr.
        new_image = PIL.Image.new("RGB", image.size)
        new_image.paste(image)
        image = new_image
    if image.mode == "RGBA":
        # the reference passes RGBA through and its analysis then fails
        # (``r, g, b = image.split()``, smartcrop.py:17 / :251)
        raise ValueError("too many values to unpack (expected 3)")
    arr = np.asarray(image)
    w, h = 100, int(options.height / options.width * 100)
    if h == 0:
        raise ZeroDivisionError("float division by zero")  # crop(): min(W / width, H / height)
    xywh = (ctypes.c_int32 * 4)()
    score = ctypes.c_double()
    arr = np.ascontiguousarray(arr)
    rc = L.lib().fi_smartcrop(_context().h, arr.ctypes.data, arr.shape[1], arr.shape[0], arr.strides[0], w, h,
                              ctypes.byref(SmartCrop().params), xywh, ctypes.byref(score))
    if rc == L.FI_ENOCROP:
        raise ValueError(L.lib().fi_last_error().decode())
    L.check(rc)
    x, y, cw, ch = xywh[0], xywh[1], xywh[2], xywh[3]
    sys.stdout.write("%sx%s+%s+%s\n" % (cw + x, ch + y, x, y))
    return 0


if __name__ == "__main__":
    sys.exit(main())
