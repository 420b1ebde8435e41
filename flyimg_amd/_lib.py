"""ctypes binding of libflyimg_hip.so (include/flyimg_hip.h).

The shared library is built in-tree (``make -C flyimg_amd`` or
``__graft_entry__.build()``) and loaded from this directory.  There is no CPU
fallback: if the library is missing or cannot be loaded, ``lib()`` raises.
"""
from __future__ import annotations

import ctypes
import os
import re

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("FI_LIB_PATH") or os.path.join(HERE, "libflyimg_hip.so")  # override: A/B of two builds
HEADER = os.path.join(os.path.dirname(HERE), "include", "flyimg_hip.h")

FI_OK = 0
FI_EINVAL = -1
FI_ENOCROP = -2
FI_ENOMEM = -3
FI_EDEVICE = -4
FI_EUNSUPPORTED = -5
FI_ECAPACITY = -6

FI_OP_THUMBNAIL = 1 << 0
FI_OP_RESIZE = 1 << 1
FI_GEOM_FILL = 1 << 2
FI_GEOM_SHRINK_ONLY = 1 << 3
FI_OP_EXTENT = 1 << 4
FI_OP_GRAY = 1 << 5
FI_OP_MONOCHROME = 1 << 6
FI_OP_ROTATE = 1 << 7
FI_OP_SMARTCROP = 1 << 8
FI_OP_SMARTCROP_APPLY = 1 << 9
FI_OP_UNSHARP = 1 << 10
FI_OP_SHARPEN = 1 << 11
FI_OP_BLUR = 1 << 12
FI_SRC_PSEUDOCLASS = 1 << 13  # IM PseudoClass source (palette / gray): Mitchell (resize.c)

GRAVITY = {
    "NorthWest": 1, "North": 2, "NorthEast": 3, "West": 4, "Center": 5,
    "East": 6, "SouthWest": 7, "South": 8, "SouthEast": 9,
}


class FiImage(ctypes.Structure):
    _fields_ = [
        ("src", ctypes.c_void_p),
        ("src_w", ctypes.c_int32), ("src_h", ctypes.c_int32),
        ("src_stride", ctypes.c_int32), ("src_channels", ctypes.c_int32),
        ("target_w", ctypes.c_int32), ("target_h", ctypes.c_int32),
        ("flags", ctypes.c_uint32), ("gravity", ctypes.c_int32), ("rotate", ctypes.c_int32),
        ("smartcrop_w", ctypes.c_int32), ("smartcrop_h", ctypes.c_int32),
        ("dst", ctypes.c_void_p), ("dst_capacity", ctypes.c_int64),
        ("out_w", ctypes.c_int32), ("out_h", ctypes.c_int32),
        ("out_channels", ctypes.c_int32), ("out_stride", ctypes.c_int32),
        ("crop_x", ctypes.c_int32), ("crop_y", ctypes.c_int32),
        ("crop_w", ctypes.c_int32), ("crop_h", ctypes.c_int32),
        ("crop_score", ctypes.c_double),
        ("status", ctypes.c_int32), ("n_candidates", ctypes.c_int32),
        ("unsharp", ctypes.c_double * 4), ("sharpen", ctypes.c_double * 2), ("blur", ctypes.c_double * 2),
    ]


class FiSmartcropParams(ctypes.Structure):
    _fields_ = [
        ("detail_weight", ctypes.c_double), ("edge_radius", ctypes.c_double),
        ("edge_weight", ctypes.c_double), ("outside_importance", ctypes.c_double),
        ("rule_of_thirds", ctypes.c_int32),
        ("saturation_bias", ctypes.c_double), ("saturation_brightness_max", ctypes.c_double),
        ("saturation_brightness_min", ctypes.c_double), ("saturation_threshold", ctypes.c_double),
        ("saturation_weight", ctypes.c_double), ("score_down_sample", ctypes.c_int32),
        ("skin_bias", ctypes.c_double), ("skin_brightness_max", ctypes.c_double),
        ("skin_brightness_min", ctypes.c_double), ("skin_color", ctypes.c_double * 3),
        ("skin_threshold", ctypes.c_double), ("skin_weight", ctypes.c_double),
    ]


class FiSmartcropOptions(ctypes.Structure):
    _fields_ = [
        ("prescale", ctypes.c_int32), ("max_scale", ctypes.c_double), ("min_scale", ctypes.c_double),
        ("scale_step", ctypes.c_double), ("step", ctypes.c_int32), ("exact_all", ctypes.c_int32),
    ]


class FiCropScore(ctypes.Structure):
    _fields_ = [
        ("x", ctypes.c_int32), ("y", ctypes.c_int32), ("width", ctypes.c_int32), ("height", ctypes.c_int32),
        ("fx", ctypes.c_double), ("fy", ctypes.c_double), ("fw", ctypes.c_double), ("fh", ctypes.c_double),
        ("detail", ctypes.c_double), ("saturation", ctypes.c_double), ("skin", ctypes.c_double),
        ("total", ctypes.c_double), ("exact", ctypes.c_int32), ("pad", ctypes.c_int32),
    ]


class FiRecord(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int32) for n in
                ("image", "status", "out_w", "out_h", "crop_x", "crop_y", "crop_w", "crop_h")]


def struct_view(arr):
    """A ctypes array of a Structure as a numpy structured array over the same
    memory (scalar and fixed-array fields at their ctypes offsets), so a batch's
    fields are read or written column-wise instead of one attribute at a time."""
    import numpy as np

    st = arr._type_
    kinds = {ctypes.c_int32: "<i4", ctypes.c_uint32: "<u4", ctypes.c_int64: "<i8", ctypes.c_double: "<f8",
             ctypes.c_void_p: "<u8"}
    names, formats, offsets = [], [], []
    for name, ty in st._fields_:
        if ty in kinds:
            fmt = kinds[ty]
        else:  # ctypes.c_double * k
            fmt = (kinds[ty._type_], (ty._length_,))
        names.append(name)
        formats.append(fmt)
        offsets.append(getattr(st, name).offset)
    dt = np.dtype({"names": names, "formats": formats, "offsets": offsets, "itemsize": ctypes.sizeof(st)})
    return np.frombuffer((ctypes.c_char * ctypes.sizeof(arr)).from_buffer(arr), dtype=dt, count=len(arr))


class FiError(RuntimeError):
    """A non-zero status from libflyimg_hip (Processor.php:53-59's
    ExecFailedException analogue)."""

    def __init__(self, code: int, msg: str):
        super().__init__(f"flyimg_hip error {code}: {msg}")
        self.code = code


_lib = None


def header_functions() -> list[str]:
    """Every function the C-ABI header declares."""
    with open(HEADER) as f:
        text = f.read()
    return sorted(set(re.findall(r"\b(fi_[a-z0-9_]+)\s*\(", text)))


def lib():
    """Load libflyimg_hip.so (raises if it is missing: no fallback path)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"{LIB_PATH} is not built; run `make -C {HERE}` (hipcc, gfx950)")
    L = ctypes.CDLL(LIB_PATH)
    P = ctypes.POINTER
    i32, i64, u64, vp = ctypes.c_int32, ctypes.c_int64, ctypes.c_uint64, ctypes.c_void_p
    L.fi_abi_version.restype = i32
    L.fi_last_error.restype = ctypes.c_char_p
    L.fi_device_count.argtypes = [P(i32)]
    L.fi_create.argtypes = [P(vp), i32]
    L.fi_destroy.argtypes = [vp]
    L.fi_destroy.restype = None
    L.fi_plan.argtypes = [P(FiImage), i32]
    L.fi_plan_bytes.argtypes = [P(FiImage), i32, P(i64)]
    L.fi_pixelate_regions.argtypes = [vp, vp, i32, i32, i32, i32, P(i32), i32]
    L.fi_pixelate_regions_device.argtypes = [vp, vp, i32, i32, i32, i32, P(i32), i32]
    L.fi_process_batch.argtypes = [vp, P(FiImage), i32]
    L.fi_submit_batch.argtypes = [vp, P(FiImage), i32]
    L.fi_host_alloc.argtypes = [vp, ctypes.c_size_t]
    L.fi_host_alloc.restype = vp
    L.fi_host_free.argtypes = [vp, vp]
    L.fi_process_batch_device.argtypes = [vp, P(FiImage), i32]
    L.fi_submit_batch_device.argtypes = [vp, P(FiImage), i32]
    L.fi_wait.argtypes = [vp, i32]
    L.fi_smartcrop_default_params.argtypes = [P(FiSmartcropParams)]
    L.fi_smartcrop_default_params.restype = None
    L.fi_smartcrop_default_options.argtypes = [P(FiSmartcropOptions)]
    L.fi_smartcrop_default_options.restype = None
    L.fi_smartcrop.argtypes = [vp, vp, i32, i32, i32, i32, i32, P(FiSmartcropParams), P(i32), P(ctypes.c_double)]
    L.fi_smartcrop_ex.argtypes = [vp, vp, i32, i32, i32, i32, i32, P(FiSmartcropParams), P(FiSmartcropOptions),
                                  P(FiCropScore), i32, P(i32), P(i32), P(i32), P(ctypes.c_double), vp, vp, i64]
    L.fi_device_malloc.argtypes = [vp, P(vp), u64]
    L.fi_device_free.argtypes = [vp, vp]
    L.fi_memcpy_h2d.argtypes = [vp, vp, vp, u64]
    L.fi_memcpy_d2h.argtypes = [vp, vp, vp, u64]
    L.fi_fill_synthetic.argtypes = [vp, vp, i32, i32, i32, ctypes.c_uint32]
    L.fi_set_timing.argtypes = [vp, i32]
    L.fi_reset_stats.argtypes = [vp]
    L.fi_kernel_stats.argtypes = [vp, ctypes.c_char_p, P(ctypes.c_double), P(i64), P(ctypes.c_double)]
    L.fi_rccl_get_unique_id.argtypes = [ctypes.c_char_p]
    L.fi_rccl_init.argtypes = [vp, i32, i32, ctypes.c_char_p]
    L.fi_rccl_gather_records.argtypes = [vp, P(FiRecord), i32, P(FiRecord)]
    L.fi_rccl_gather_start.argtypes = [vp, P(FiRecord), i32, P(FiRecord)]
    L.fi_rccl_gather_finish.argtypes = [vp]
    L.fi_query.argtypes = [vp, P(i32)]
    L.fi_debug_monochrome.argtypes = [vp, vp, i32, i32, i32, vp, i32]
    L.fi_debug_convolve.argtypes = [vp, vp, i32, i32, i32, vp, ctypes.c_uint32, vp]
    L.fi_debug_skinsat.argtypes = [vp, vp, vp]
    L.fi_debug_host_plan.argtypes = [ctypes.POINTER(FiImage), i32, i32, ctypes.POINTER(ctypes.c_double)]
    L.fi_jpeg_info.argtypes = [ctypes.c_char_p, ctypes.c_size_t, P(i32), P(i32), P(i32)]
    L.fi_jpeg_decode_device.argtypes = [vp, vp, vp, i32, vp, vp, i32, vp]
    _lib = L
    return L


def check(rc: int) -> int:
    if rc != FI_OK:
        msg = lib().fi_last_error()
        raise FiError(rc, msg.decode() if msg else "")
    return rc
