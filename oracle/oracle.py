"""ctypes binding of the CPU oracle (oracle/fi_oracle.c).

TEST INFRASTRUCTURE ONLY -- imported by tests/, ``__graft_entry__.smoke()`` and
``bench.py``'s ``cpu_baseline`` leg as the checker.  The product package
(``flyimg_amd``) never imports this module.

Parity status per half (see fi_oracle.c header):
  * smartcrop.py / Pillow / numpy arithmetic -- pinned by tests/golden/ vectors
    generated from the reference module (tests/golden/make_golden.py).
  * ImageMagick convert operators -- parity unpinned (IM absent); only output
    geometry pinned by the reference's ImageProcessorTest known answers.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "libfi_oracle.so")
_lib = None


class ScParams(ctypes.Structure):
    """Mirror of or_sc_params == SmartCrop.__init__ keyword defaults
    (reference python/smartcrop.py:41-77)."""

    _fields_ = [
        ("detail_weight", ctypes.c_double),
        ("edge_radius", ctypes.c_double),
        ("edge_weight", ctypes.c_double),
        ("outside_importance", ctypes.c_double),
        ("rule_of_thirds", ctypes.c_int),
        ("saturation_bias", ctypes.c_double),
        ("saturation_brightness_max", ctypes.c_double),
        ("saturation_brightness_min", ctypes.c_double),
        ("saturation_threshold", ctypes.c_double),
        ("saturation_weight", ctypes.c_double),
        ("score_down_sample", ctypes.c_int),
        ("skin_bias", ctypes.c_double),
        ("skin_brightness_max", ctypes.c_double),
        ("skin_brightness_min", ctypes.c_double),
        ("skin_color", ctypes.c_double * 3),
        ("skin_threshold", ctypes.c_double),
        ("skin_weight", ctypes.c_double),
    ]


class ScCrop(ctypes.Structure):
    _fields_ = [
        ("x", ctypes.c_int32),
        ("y", ctypes.c_int32),
        ("width", ctypes.c_int32),
        ("height", ctypes.c_int32),
        ("fx", ctypes.c_double),
        ("fy", ctypes.c_double),
        ("fw", ctypes.c_double),
        ("fh", ctypes.c_double),
        ("detail", ctypes.c_double),
        ("saturation", ctypes.c_double),
        ("skin", ctypes.c_double),
        ("total", ctypes.c_double),
    ]


def build() -> str:
    """Compile libfi_oracle.so with the committed Makefile (gcc)."""
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH) or os.path.getmtime(_LIB_PATH) < os.path.getmtime(
            os.path.join(_HERE, "fi_oracle.c")
        ):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        P = ctypes.POINTER
        u8p = P(ctypes.c_uint8)
        i = ctypes.c_int
        L.or_im_meta_geometry.argtypes = [i, i, i, i, i, i, P(i), P(i)]
        L.or_im_resize_u8_to_q16.argtypes = [u8p, i, i, i, i, i, i, i, i, P(ctypes.c_uint16)]
        L.or_im_convert.argtypes = [u8p, i, i, i, i, i, ctypes.c_uint, i, i, u8p, i, P(i), P(i), P(i)]
        L.or_im_convert_c.argtypes = [u8p, i, i, i, i, i, i, ctypes.c_uint, i, i, u8p, i, P(i), P(i), P(i)]
        L.or_im_convert_ex.argtypes = [u8p, i, i, i, i, i, i, ctypes.c_uint, i, i, P(ctypes.c_double), ctypes.c_uint,
                                       u8p, i, P(i), P(i), P(i)]
        L.or_im_convolve_ops.argtypes = [P(ctypes.c_uint16), i, i, i, P(ctypes.c_double), ctypes.c_uint]
        L.or_im_blur_kernel.argtypes = [ctypes.c_double, ctypes.c_double, P(ctypes.c_double), i]
        L.or_im_sharpen_kernel.argtypes = [ctypes.c_double, ctypes.c_double, P(ctypes.c_double), i]
        L.or_im_kernel_width_1d.argtypes = [ctypes.c_double, ctypes.c_double]
        L.or_im_kernel_width_2d.argtypes = [ctypes.c_double, ctypes.c_double]
        L.or_im_gravity_offset.argtypes = [i, i, i, i, i, P(i), P(i)]
        L.or_im_gravity_offset.restype = None
        L.or_im_sample_index.argtypes = [ctypes.c_long] * 3
        L.or_im_sample_index.restype = ctypes.c_long
        L.or_im_thumbnail_uses_sample.argtypes = [i, i, i, i]
        L.or_pil_reduce.argtypes = [u8p, i, i, i, i, i, u8p]
        L.or_pil_resample.argtypes = [u8p, i, i, i, i, i] + [ctypes.c_float] * 4 + [u8p]
        L.or_pil_thumbnail_size.argtypes = [i, i, i, i, P(i), P(i)]
        L.or_pil_thumbnail.argtypes = [u8p, i, i, i, i, i, u8p, P(i), P(i)]
        L.or_sc_default_params.argtypes = [P(ScParams)]
        L.or_sc_default_params.restype = None
        L.or_sc_maps.argtypes = [P(ScParams), u8p, i, i, i, u8p, u8p, u8p, u8p]
        L.or_sc_crops.argtypes = [i, i, i, i, ctypes.c_double, ctypes.c_double, ctypes.c_double, i, P(ScCrop), i]
        L.or_sc_crop.argtypes = [
            P(ScParams), u8p, i, i, i, i, i, i,
            ctypes.c_double, ctypes.c_double, ctypes.c_double, i,
            P(ScCrop), i, P(i), P(i), P(i), P(ctypes.c_double), u8p, u8p,
        ]
        L.or_sc_max_crops.argtypes = [i, i, i]
        u16p = P(ctypes.c_uint16)
        L.or_im_monochrome.argtypes = [u16p, i, i, u8p]
        L.or_hilbert_d2xy.argtypes = [i, ctypes.c_long, P(i), P(i)]
        L.or_hilbert_d2xy.restype = None
        L.or_mono_curve_level.argtypes = [i, i]
        L.or_mono_quant_info.argtypes = [P(ctypes.c_uint64), P(i), u16p, u16p]
        assert L.or_sizeof_crop() == ctypes.sizeof(ScCrop)
        assert L.or_sizeof_params() == ctypes.sizeof(ScParams)
        _lib = L
    return _lib


def _u8(a: np.ndarray):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8))


def default_params(**overrides) -> ScParams:
    p = ScParams()
    lib().or_sc_default_params(ctypes.byref(p))
    for k, v in overrides.items():
        if k == "skin_color":
            for j in range(3):
                p.skin_color[j] = v[j]
        else:
            setattr(p, k, v)
    return p


# --------------------------------------------------------------------------
# ImageMagick restatement
# --------------------------------------------------------------------------
def im_meta_geometry(W, H, tw, th, fill=False, shrink_only=False):
    ow, oh = ctypes.c_int(), ctypes.c_int()
    rc = lib().or_im_meta_geometry(W, H, tw or 0, th or 0, int(fill), int(shrink_only), ctypes.byref(ow), ctypes.byref(oh))
    if rc:
        raise ValueError(f"or_im_meta_geometry rc={rc}")
    return ow.value, oh.value


def im_gravity_offset(W, H, ew, eh, gravity=5):
    x, y = ctypes.c_int(), ctypes.c_int()
    lib().or_im_gravity_offset(W, H, ew, eh, gravity, ctypes.byref(x), ctypes.byref(y))
    return x.value, y.value


FLAG_THUMBNAIL, FLAG_FILL, FLAG_SHRINK, FLAG_EXTENT, FLAG_GRAY, FLAG_ROTATE = 1, 2, 4, 8, 16, 32
FLAG_MONO = 64  # -monochrome (B7); implies gray
FLAG_PSEUDOCLASS = 128  # PseudoClass source (palette / gray): ResizeImage's Mitchell rule (resize.c)
CONV_UNSHARP, CONV_SHARPEN, CONV_BLUR = 1, 2, 4  # forwarded convolutions (ImageProcessor.php:303-315)


def im_monochrome(gray_q16: np.ndarray) -> np.ndarray:
    """-monochrome of a Q16 gray image (B7 restatement, parity unpinned) -> 0/255 u8."""
    g = np.ascontiguousarray(gray_q16, dtype=np.uint16)
    h, w = g.shape
    out = np.zeros((h, w), np.uint8)
    rc = lib().or_im_monochrome(g.ctypes.data_as(ctypes.POINTER(ctypes.c_uint16)), w, h, _u8(out))
    if rc:
        raise ValueError(f"or_im_monochrome rc={rc}")
    return out


def hilbert_d2xy(level: int, d: int):
    x, y = ctypes.c_int(), ctypes.c_int()
    lib().or_hilbert_d2xy(level, d, ctypes.byref(x), ctypes.byref(y))
    return x.value, y.value


def mono_curve_level(w: int, h: int) -> int:
    return lib().or_mono_curve_level(w, h)


def mono_quant_info(hist: np.ndarray):
    """(ncol, cluster means, bilevel colours) of a stretched Q16 histogram."""
    H = np.ascontiguousarray(hist, dtype=np.uint64)
    assert H.size == 65536
    n = ctypes.c_int()
    m = np.zeros(2, np.uint16)
    b = np.zeros(2, np.uint16)
    P = ctypes.POINTER
    lib().or_mono_quant_info(H.ctypes.data_as(P(ctypes.c_uint64)), ctypes.byref(n),
                             m.ctypes.data_as(P(ctypes.c_uint16)), b.ctypes.data_as(P(ctypes.c_uint16)))
    return n.value, m[: min(n.value, 2)].tolist(), b[: min(n.value, 2)].tolist()


def im_convert(src: np.ndarray, rw=0, rh=0, flags=FLAG_THUMBNAIL, gravity=5, rotate=0, conv=None,
               conv_ops=0) -> np.ndarray:
    """convert <src> <resize op> [-gravity g -extent WxH] [-colorspace Gray] [-monochrome] [-rotate r].
    RGBA sources (H x W x 4) take IM's matte path: Mitchell, alpha-weighted passes,
    RGBA out (gray + alpha after -colorspace Gray).  conv = (unsharp radius, sigma,
    gain, threshold, sharpen radius, sigma, blur radius, sigma), conv_ops = CONV_*
    bits: the forwarded -unsharp / -sharpen / -blur after -rotate."""
    src = np.ascontiguousarray(src, dtype=np.uint8)
    H, W = src.shape[:2]
    C = src.shape[2] if src.ndim == 3 else 1  # 3 = RGB, 4 = RGBA (IM matte image)
    tw, th = W, H
    if rw or rh:
        tw, th = im_meta_geometry(W, H, rw, rh, bool(flags & FLAG_FILL), bool(flags & FLAG_SHRINK))
    cap = 4 * (max(tw, rw or 0) * max(th, rh or 0) + 16)  # output bound (an int32 on the C side)
    out = np.zeros(cap, np.uint8)
    ow, oh, oc = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
    cv = (ctypes.c_double * 8)(*(list(conv) + [0.0] * 8)[:8]) if conv is not None else (ctypes.c_double * 8)()
    rc = lib().or_im_convert_ex(_u8(src), W, H, C, W * C, rw, rh, flags, gravity, rotate, cv, conv_ops, _u8(out),
                                cap, ctypes.byref(ow), ctypes.byref(oh), ctypes.byref(oc))
    if rc:
        raise ValueError(f"or_im_convert rc={rc}")
    o = out[: ow.value * oh.value * oc.value].reshape(oh.value, ow.value, oc.value)
    return o[:, :, 0] if oc.value == 1 else o


def im_convolve_q16(q16: np.ndarray, conv, ops: int) -> np.ndarray:
    """or_im_convolve_ops (-unsharp / -sharpen / -blur on a Q16 HWC image) -> 8-bit."""
    q = np.ascontiguousarray(q16, dtype=np.uint16).copy()
    h, w = q.shape[:2]
    ch = q.shape[2] if q.ndim == 3 else 1
    cv = (ctypes.c_double * 8)(*conv)
    rc = lib().or_im_convolve_ops(q.ctypes.data_as(ctypes.POINTER(ctypes.c_uint16)), w, h, ch, cv, ops)
    if rc:
        raise ValueError(f"or_im_convolve_ops rc={rc}")
    return (((q.astype(np.uint32) + 128) - ((q.astype(np.uint32) + 128) >> 8)) >> 8).astype(np.uint8)


def im_scale_q16(q16: np.ndarray, ow: int, oh: int) -> np.ndarray:
    """or_im_scale_q16: IM 6 ScaleImage of an opaque Q16 HWC image."""
    q = np.ascontiguousarray(q16, dtype=np.uint16)
    h, w = q.shape[:2]
    c = q.shape[2] if q.ndim == 3 else 1
    out = np.zeros((oh, ow, c), np.uint16)
    P = ctypes.POINTER(ctypes.c_uint16)
    rc = lib().or_im_scale_q16(q.ctypes.data_as(P), w, h, c, ow, oh, out.ctypes.data_as(P))
    if rc:
        raise ValueError(f"or_im_scale_q16 rc={rc}")
    return out if q.ndim == 3 else out[:, :, 0]


def im_percent_size(size: int, percent: float) -> int:
    return int(lib().or_im_percent_size(int(size), ctypes.c_double(percent)))


def im_pixelate_regions(img: np.ndarray, boxes) -> np.ndarray:
    """or_im_pixelate_regions: the face-blur mogrify per box, on a copy."""
    out = np.ascontiguousarray(img, dtype=np.uint8).copy()
    h, w = out.shape[:2]
    c = out.shape[2] if out.ndim == 3 else 1
    flat = [int(v) for b in boxes for v in b]
    arr = (ctypes.c_int * max(len(flat), 1))(*flat)
    rc = lib().or_im_pixelate_regions(_u8(out), w, h, w * c, c, arr, len(flat) // 4)
    if rc:
        raise ValueError(f"or_im_pixelate_regions rc={rc}")
    return out


def im_resize_q16(src: np.ndarray, ow: int, oh: int, thumbnail=True) -> np.ndarray:
    src = np.ascontiguousarray(src, dtype=np.uint8)
    H, W, C = src.shape
    out = np.zeros((oh, ow, C), np.uint16)
    rc = lib().or_im_resize_u8_to_q16(_u8(src), W, H, C, W * C, ow, oh, int(thumbnail), 0,
                                      out.ctypes.data_as(ctypes.POINTER(ctypes.c_uint16)))
    if rc:
        raise ValueError(f"or_im_resize_u8_to_q16 rc={rc}")
    return out


# --------------------------------------------------------------------------
# Pillow restatement
# --------------------------------------------------------------------------
def pil_reduce(src: np.ndarray, fx: int, fy: int) -> np.ndarray:
    src = np.ascontiguousarray(src, dtype=np.uint8)
    H, W = src.shape[:2]
    out = np.zeros(((H + fy - 1) // fy, (W + fx - 1) // fx, 3), np.uint8)
    rc = lib().or_pil_reduce(_u8(src), W, H, W * 3, fx, fy, _u8(out))
    if rc:
        raise ValueError(rc)
    return out


def pil_resample(src: np.ndarray, ow: int, oh: int, box=None) -> np.ndarray:
    src = np.ascontiguousarray(src, dtype=np.uint8)
    H, W = src.shape[:2]
    box = box or (0, 0, W, H)
    out = np.zeros((oh, ow, 3), np.uint8)
    rc = lib().or_pil_resample(_u8(src), W, H, W * 3, ow, oh, *[float(b) for b in box], _u8(out))
    if rc:
        raise ValueError(rc)
    return out


def pil_thumbnail(src: np.ndarray, x: int, y: int) -> np.ndarray:
    src = np.ascontiguousarray(src, dtype=np.uint8)
    H, W = src.shape[:2]
    out = np.zeros((max(H, 1), max(W, 1), 3), np.uint8)
    ow, oh = ctypes.c_int(), ctypes.c_int()
    rc = lib().or_pil_thumbnail(_u8(src), W, H, W * 3, x, y, _u8(out), ctypes.byref(ow), ctypes.byref(oh))
    if rc:
        raise ValueError(rc)
    return out.reshape(-1)[: ow.value * oh.value * 3].reshape(oh.value, ow.value, 3)


# --------------------------------------------------------------------------
# smartcrop.py restatement
# --------------------------------------------------------------------------
def sc_maps(rgb: np.ndarray, params: ScParams | None = None):
    """Returns (L, edge, skin, sat) uint8 maps of an RGB image (analyse())."""
    rgb = np.ascontiguousarray(rgb, dtype=np.uint8)
    H, W = rgb.shape[:2]
    maps = [np.zeros((H, W), np.uint8) for _ in range(4)]
    lib().or_sc_maps(ctypes.byref(params) if params else None, _u8(rgb), W, H, W * 3, *[_u8(m) for m in maps])
    return tuple(maps)


def sc_crop(rgb: np.ndarray, width: int = 100, height: int = 100, prescale=True, max_scale=1.0,
            min_scale=0.9, scale_step=0.1, step=8, params: ScParams | None = None):
    """SmartCrop().crop() -> dict like the reference (crops, top_crop) plus the
    analysed maps, prescaled image and prescale factor."""
    rgb = np.ascontiguousarray(rgb, dtype=np.uint8)
    H, W = rgb.shape[:2]
    L = lib()
    cap = L.or_sc_max_crops(W, H, step) + 16
    crops = (ScCrop * cap)()
    top, aw, ah = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
    pre = ctypes.c_double()
    maps = np.zeros(W * H * 3 + 3, np.uint8)
    prescaled = np.zeros(W * H * 3 + 3, np.uint8)
    n = L.or_sc_crop(ctypes.byref(params) if params else None, _u8(rgb), W, H, W * 3, width, height,
                     int(prescale), max_scale, min_scale, scale_step, step, crops, cap,
                     ctypes.byref(top), ctypes.byref(aw), ctypes.byref(ah), ctypes.byref(pre),
                     _u8(maps), _u8(prescaled))
    if n == -2:
        raise ValueError("smartcrop: no crops")
    if n < 0:
        raise RuntimeError(f"or_sc_crop rc={n}")
    out = []
    for c in crops[:n]:
        out.append({
            "x": c.x, "y": c.y, "width": c.width, "height": c.height,
            "fx": c.fx, "fy": c.fy, "fw": c.fw, "fh": c.fh,
            "score": {"detail": c.detail, "saturation": c.saturation, "skin": c.skin, "total": c.total},
        })
    na = aw.value * ah.value * 3
    return {
        "crops": out,
        "top_index": top.value,
        "top_crop": out[top.value],
        "analyse_size": (aw.value, ah.value),
        "maps": maps[:na].reshape(ah.value, aw.value, 3),
        "prescaled": prescaled[:na].reshape(ah.value, aw.value, 3),
        "prescale": pre.value,
    }


def sc_geometry_string(result) -> str:
    """smartcrop.py main() output line (smartcrop.py:372-377)."""
    t = result["top_crop"]
    return "%sx%s+%s+%s" % (t["width"] + t["x"], t["height"] + t["y"], t["x"], t["y"])
