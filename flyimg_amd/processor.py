"""Host-side mirror of flyimg's option model and ImageProcessor for the GPU path.

Same names, argument meaning and error behaviour as the reference:
  * ``OptionsBag``      -- src/Core/Entity/OptionsBag.php:40-172 with the keys and
                           defaults of config/parameters.yml:43-120;
  * ``ImageProcessor``  -- src/Core/Processor/ImageProcessor.php:49-315: builds the
                           same ``convert`` command string (for the ``im-command``
                           debug header, Response.php:58-64) and the equivalent
                           ``fi_image`` operator descriptor for libflyimg_hip;
  * ``SmartCropProcessor`` -- SmartCropProcessor.php:21-36 (geometry line, crop).
Errors surface as ``ExecFailedException`` (Processor.php:53-59).
"""
from __future__ import annotations

import shlex

from . import _lib as L
from .runtime import Op

# config/parameters.yml:43-80 (options_keys)
OPTIONS_KEYS = {
    "moz": "mozjpeg", "q": "quality", "o": "output", "unsh": "unsharp", "sh": "sharpen", "blr": "blur",
    "fc": "face-crop", "fcp": "face-crop-position", "fb": "face-blur", "w": "width", "h": "height",
    "c": "crop", "bg": "background", "st": "strip", "rz": "resize", "g": "gravity", "f": "filter",
    "r": "rotate", "sc": "scale", "sf": "sampling-factor", "rf": "refresh", "smc": "smart-crop",
    "ett": "extent", "par": "preserve-aspect-ratio", "pns": "preserve-natural-size",
    "webpl": "webp-lossless", "gf": "gif-frame", "e": "extract", "p1x": "extract-top-x",
    "p1y": "extract-top-y", "p2x": "extract-bottom-x", "p2y": "extract-bottom-y",
    "pg": "page_number", "tm": "time", "clsp": "colorspace", "mnchr": "monochrome", "dnst": "density",
}
# config/parameters.yml:82-120 (default_options)
DEFAULT_OPTIONS = {
    "mozjpeg": 1, "quality": 90, "output": "auto", "unsharp": None, "sharpen": None, "blur": None,
    "face-crop": 0, "face-crop-position": 0, "face-blur": 0, "width": None, "height": None, "crop": None,
    "background": None, "strip": 1, "resize": None, "gravity": "Center", "filter": "Lanczos", "rotate": None,
    "scale": None, "sampling-factor": "1x1", "refresh": False, "smart-crop": False, "extent": None,
    "preserve-aspect-ratio": 1, "preserve-natural-size": 1, "webp-lossless": 0, "gif-frame": 0,
    "extract": None, "extract-top-x": None, "extract-top-y": None, "extract-bottom-x": None,
    "extract-bottom-y": None, "page_number": 1, "time": "00:00:01", "colorspace": "sRGB",
    "monochrome": None, "density": None,
}


class ExecFailedException(RuntimeError):
    """Processor.php:53-59: a failed pixel operation."""


def im_parse_geometry(text: str):
    """ImageMagick ParseGeometry for the -unsharp / -sharpen / -blur arguments
    (geometry.c): ``rho[xsigma][+xi][+psi]`` -> (rho, sigma, xi, psi), None for
    a value that is absent (mogrify then applies its defaults: sigma 1, gain 1,
    threshold 0.05).  Separators 'x' / 'X' / ',' / '/' and signs '+' / '-'."""
    import re

    m = re.fullmatch(r"\s*([+-]?[0-9]*\.?[0-9]+(?:[eE][+-]?[0-9]+)?)?"
                     r"(?:[xX,/]([+-]?[0-9]*\.?[0-9]+(?:[eE][+-]?[0-9]+)?))?"
                     r"([+-][0-9]*\.?[0-9]+(?:[eE][+-]?[0-9]+)?)?"
                     r"([+-][0-9]*\.?[0-9]+(?:[eE][+-]?[0-9]+)?)?\s*", text)
    if not m or m.group(1) is None:
        raise ExecFailedException(f"invalid geometry {text!r}")
    vals = [float(x) if x is not None else None for x in m.groups()]
    return vals[0], vals[1], vals[2], vals[3]


def _empty(v) -> bool:
    """PHP empty(): null, '', '0', 0, false are empty."""
    return v is None or v is False or v == "" or v == "0" or v == 0


class OptionsBag:
    """OptionsBag.php:40-172."""

    def __init__(self, options: str, separator: str = ","):
        self.parsed = self._parse(options, separator or ",")
        self.collection = dict(self.parsed)

    @staticmethod
    def _parse(options: str, sep: str) -> dict:
        out = {}
        for opt in options.split(sep):
            parts = opt.split("_")
            key = parts[0]
            if key in OPTIONS_KEYS and OPTIONS_KEYS[key]:
                # PHP: $optArray[1] (a missing value is an undefined index -> null)
                out[OPTIONS_KEYS[key]] = parts[1] if len(parts) > 1 else None
        merged = dict(DEFAULT_OPTIONS)
        merged.update(out)
        return merged

    def get(self, key, default=None):
        return self.parsed.get(key, default)

    def has(self, key) -> bool:
        return key in self.parsed

    def remove(self, key):
        self.parsed.pop(key, None)

    def as_array(self) -> dict:
        return self.parsed

    def get_option(self, key):
        return self.collection.get(key, "")

    def set_option(self, key, value):
        self.collection[key] = str(value)
        return self

    def extract_key(self, key) -> str:
        """InputImage::extractKey (InputImage.php:108-117)."""
        value = ""
        if self.has(key):
            value = self.get(key)
            self.remove(key)
        return "" if value is None else value


class ImageProcessor:
    """ImageProcessor.php:21-316, restricted to the operators of the GPU path."""

    FORWARDED = ["background", "rotate", "unsharp", "sharpen", "blur", "filter"]

    def __init__(self, options: OptionsBag, src_w: int, src_h: int):
        self.options = options
        self.src_w, self.src_h = src_w, src_h  # ImageMetaInfo::dimensions() (identify)
        self.geometry = {}

    # --- ImageProcessor.php:240-259 ------------------------------------------
    def get_dimensions(self) -> str:
        if "dimensions" not in self.geometry:
            w, h = self.options.get_option("width"), self.options.get_option("height")
            d = ""
            if not _empty(w):
                d += shlex.quote(str(w)) if not str(w).isdigit() else f"'{w}'"
            if not _empty(h):
                d += "x" + (f"'{h}'" if str(h).isdigit() else shlex.quote(str(h)))
            self.geometry["dimensions"] = d
        return self.geometry["dimensions"]

    def get_resize_operator(self) -> str:  # :264-272
        return "-resize" if not _empty(self.options.get_option("resize")) else "-thumbnail"

    def update_target_dimensions(self):  # :277-295
        if _empty(self.options.get_option("preserve-natural-size")):
            return
        tw, th = self.options.get_option("width"), self.options.get_option("height")
        if not _empty(tw) and self.src_w < int(tw):
            self.options.set_option("width", self.src_w)
        if not _empty(th) and self.src_h < int(th):
            self.options.set_option("height", self.src_h)

    def calculate_size(self) -> str:  # :115-130
        w, h, c = (self.options.get_option(k) for k in ("width", "height", "crop"))
        if not _empty(w) and not _empty(h) and not _empty(c):
            return self.generate_crop_size()
        if not _empty(w) or not _empty(h):
            return self.generate_simple_size()
        return ""

    def generate_crop_size(self) -> str:  # :138-148
        self.update_target_dimensions()
        return " ".join([self.get_resize_operator(), self.get_dimensions() + "^",
                         "-gravity " + str(self.options.get_option("gravity")), "-extent " + self.get_dimensions()])

    def generate_simple_size(self) -> str:  # :154-162
        pns = not _empty(self.options.get_option("preserve-natural-size"))
        return " ".join([self.get_resize_operator(), self.get_dimensions() + ("'>'" if pns else "")])

    def generate_command(self, src_path="<src>", out_arg="<quality/output>") -> str:
        """The convert command string of generateCommand (:66-110)."""
        args = ["-auto-orient", src_path, self.calculate_size()]
        args.append("-colorspace " + shlex.quote(str(self.options.extract_key("colorspace"))))
        if not _empty(self.options.extract_key("monochrome")):
            args.append("-monochrome")
        fwd = []
        for o in self.FORWARDED:
            v = self.options.get_option(o)
            if not _empty(v):
                fwd.append(f"-{o} " + shlex.quote(str(v)))
        args.append(" ".join(fwd))
        if not _empty(self.options.extract_key("strip")):
            args.append("-strip")
        args.append(out_arg)
        return "/usr/bin/convert " + " ".join(args)

    # --- the fi_image descriptor -----------------------------------------------
    def to_op(self) -> Op:
        """Same decisions as generateCommand, as an fi_image operator set."""
        o = self.options
        op = Op()
        w, h, c = o.get_option("width"), o.get_option("height"), o.get_option("crop")
        resize = not _empty(o.get_option("resize"))
        op.flags = L.FI_OP_RESIZE if resize else L.FI_OP_THUMBNAIL
        if not _empty(w) and not _empty(h) and not _empty(c):
            self.update_target_dimensions()
            w, h = o.get_option("width"), o.get_option("height")
            op.target_w, op.target_h = int(w), int(h)
            op.flags |= L.FI_GEOM_FILL | L.FI_OP_EXTENT
            g = str(o.get_option("gravity"))
            code = {k.lower(): v for k, v in L.GRAVITY.items()}.get(g.lower())  # IM: case-insensitive
            if code is None:
                raise ExecFailedException(f"unsupported gravity {g!r}")
            op.gravity = code
        elif not _empty(w) or not _empty(h):
            op.target_w = int(w) if not _empty(w) else 0
            op.target_h = int(h) if not _empty(h) else 0
            if not _empty(o.get_option("preserve-natural-size")):
                op.flags |= L.FI_GEOM_SHRINK_ONLY
        clsp = str(o.get_option("colorspace"))
        if clsp.lower() == "gray":
            op.flags |= L.FI_OP_GRAY
        elif clsp.lower() not in ("srgb", "rgb", ""):
            raise ExecFailedException(f"colorspace {clsp!r} is not on the GPU path")
        if not _empty(o.get_option("monochrome")):
            op.flags |= L.FI_OP_MONOCHROME
        rot = o.get_option("rotate")
        if not _empty(rot):
            deg = int(float(rot))
            if deg % 90:
                raise ExecFailedException(f"-rotate {rot} (non-integral) is not on the GPU path")
            op.flags |= L.FI_OP_ROTATE
            op.rotate = deg
        if not _empty(o.get_option("background")):
            raise ExecFailedException("-background is not on the GPU path")
        # forwarded convolutions (:303-315), applied after -rotate in this order
        v = o.get_option("unsharp")
        if not _empty(v):
            g = im_parse_geometry(str(v))
            op.flags |= L.FI_OP_UNSHARP
            op.unsharp = (g[0], g[1] if g[1] is not None else 1.0, g[2] if g[2] is not None else 1.0,
                          g[3] if g[3] is not None else 0.05)
        for key, flag in (("sharpen", L.FI_OP_SHARPEN), ("blur", L.FI_OP_BLUR)):
            v = o.get_option(key)
            if not _empty(v):
                g = im_parse_geometry(str(v))
                op.flags |= flag
                setattr(op, key, (g[0], g[1] if g[1] is not None else 1.0))
        if not _empty(o.get_option("smart-crop")):
            # SmartCropProcessor runs smartcrop.py with its CLI defaults (100x100)
            op.flags |= L.FI_OP_SMARTCROP | L.FI_OP_SMARTCROP_APPLY
            op.smartcrop_w, op.smartcrop_h = 100, 100
        return op


class ExtractProcessor:
    """ExtractProcessor.php:21-40: ``convert <src> -crop WxH+X+Y <src>`` with
    W = p2x - p1x, H = p2y - p1y, run before ImageProcessor
    (ImageHandler.php:163-165), which then identifies the cropped file
    (ImageMetaInfo::info() is lazy, ImageMetaInfo.php:125-134).

    IM CropImage intersects the rectangle with the image.  No pixel work: the
    extracted source is a view (pointer + stride + dims) of the decoded one,
    which is what an fi_image source already is."""

    @staticmethod
    def rectangle(options: OptionsBag, src_w: int, src_h: int):
        """(x, y, w, h) of the extracted region, clipped to the image."""
        keys = ("extract-top-x", "extract-top-y", "extract-bottom-x", "extract-bottom-y")
        vals = [options.extract_key(k) for k in keys]
        try:
            x0, y0, x1, y1 = (int(str(v)) for v in vals)
        except ValueError:
            # PHP 8: arithmetic on a non-numeric string is a TypeError
            raise ExecFailedException(f"extract coordinates must be integers, got {vals}") from None
        gw, gh = x1 - x0, y1 - y0
        if gw <= 0 or gh <= 0 or x0 < 0 or y0 < 0:
            raise ExecFailedException(f"-crop {gw}x{gh}+{x0}+{y0}: not a positive rectangle")
        if x0 >= src_w or y0 >= src_h:
            raise ExecFailedException(f"-crop {gw}x{gh}+{x0}+{y0}: geometry does not contain image")
        return x0, y0, min(gw, src_w - x0), min(gh, src_h - y0)

    @staticmethod
    def extract(options: OptionsBag, image):
        """The extracted view of a decoded HWC image, or the image itself when
        ``e`` is not set."""
        if _empty(options.extract_key("extract")):
            return image
        x, y, w, h = ExtractProcessor.rectangle(options, image.shape[1], image.shape[0])
        return image[y:y + h, x:x + w]


class FaceDetectProcessor:
    """FaceDetectProcessor.php:45-74 blurFaces: every line ``"x y w h"`` of the
    facedetect output (face detection itself is out of scope: its output is
    the input here) becomes one ``mogrify -gravity NorthWest -region WxH+X+Y
    -scale 10% -scale 1000%`` on the output image -- fi_pixelate_regions, in
    place, boxes in the output's order; lines that do not split into four
    fields are skipped as the reference skips them."""

    @staticmethod
    def boxes(facedetect_output):
        out = []
        for line in facedetect_output:
            g = str(line).split(" ")
            if len(g) == 4:
                out.append(tuple(int(v) for v in g))
        return out

    @staticmethod
    def blur_faces(ctx, image, facedetect_output):
        boxes = FaceDetectProcessor.boxes(facedetect_output)
        if not boxes:
            return image
        rc = ctx.pixelate_regions(image, boxes)
        if rc != L.FI_OK:
            msg = L.lib().fi_last_error()
            raise ExecFailedException("Command failed.\nThe exit code: %d\n%s" % (rc, msg.decode() if msg else ""))
        return image


def process_new_image(ctx, options: str, image, pseudo_class: bool = False):
    """ImageHandler::processNewImage for the GPU path: ExtractProcessor ->
    ImageProcessor -> SmartCropProcessor on one decoded RGB8 image
    (``pseudo_class``: IM would have read a palette / gray PseudoClass image,
    codec.decode_ex).  Returns (pixels, record)."""
    bag = OptionsBag(options)
    image = ExtractProcessor.extract(bag, image)
    h, w = image.shape[:2]
    op = ImageProcessor(bag, w, h).to_op()
    if pseudo_class:
        op.flags |= L.FI_SRC_PSEUDOCLASS
    outs, recs, rc = ctx.process([image], [op])
    if recs[0].status != L.FI_OK:
        msg = L.lib().fi_last_error()
        raise ExecFailedException("Command failed.\nThe exit code: %d\n%s" % (recs[0].status, msg.decode() if msg else ""))
    return outs[0], recs[0]
