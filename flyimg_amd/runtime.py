"""Host-side runtime over the C-ABI: one ``Context`` per process per GPU.

Thin, allocation-light wrappers: numpy arrays in, numpy arrays out for the
host path (``fi_process_batch``), raw device pointers for device-resident
batches (``fi_process_batch_device``, used by bench.py).
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass

import numpy as np

from . import _lib as L


@dataclass
class Op:
    """One image's operator list -- the fields of fi_image a caller sets.
    Mirrors the convert argv ImageProcessor::generateCommand builds
    (ImageProcessor.php:66-110)."""

    target_w: int = 0
    target_h: int = 0
    flags: int = L.FI_OP_THUMBNAIL
    gravity: int = L.GRAVITY["Center"]
    rotate: int = 0
    smartcrop_w: int = 0
    smartcrop_h: int = 0
    # forwarded -unsharp / -sharpen / -blur (FI_OP_UNSHARP / SHARPEN / BLUR)
    unsharp: tuple = (0.0, 1.0, 1.0, 0.05)
    sharpen: tuple = (0.0, 1.0)
    blur: tuple = (0.0, 1.0)


def _fill(img: L.FiImage, op: Op):
    img.target_w, img.target_h = op.target_w, op.target_h
    img.flags, img.gravity, img.rotate = op.flags, op.gravity, op.rotate
    img.smartcrop_w, img.smartcrop_h = op.smartcrop_w, op.smartcrop_h
    for k in range(4):
        img.unsharp[k] = op.unsharp[k]
    for k in range(2):
        img.sharpen[k] = op.sharpen[k]
        img.blur[k] = op.blur[k]


def plan(width: int, height: int, op: Op):
    """fi_plan for one image: (out_w, out_h, out_channels) before smart-crop apply."""
    img = L.FiImage()
    img.src_w, img.src_h, img.src_stride, img.src_channels = width, height, width * 3, 3
    _fill(img, op)
    L.check(L.lib().fi_plan(ctypes.byref(img), 1))
    return img.out_w, img.out_h, img.out_channels


def plan_bytes(sizes_ops):
    """fi_plan_bytes: SURVEY 8(e) B_img (algorithmic HBM bytes) of each
    (width, height, Op); -1 where the image does not plan."""
    n = len(sizes_ops)
    arr = (L.FiImage * max(n, 1))()
    for i, (w, h, op) in enumerate(sizes_ops):
        a = arr[i]
        a.src_w, a.src_h, a.src_stride, a.src_channels = w, h, w * 3, 3
        _fill(a, op)
    out = (ctypes.c_int64 * max(n, 1))()
    L.lib().fi_plan_bytes(arr, n, out)  # per-image -1 on failure; the caller decides
    return [int(out[i]) for i in range(n)]


def jpeg_info(blob: bytes):
    """(width, height, channels) of a JPEG the GPU decoder handles, else None
    (fi_jpeg_info: progressive, CMYK, 4:1:1, ... decode on the host)."""
    w, h, c = ctypes.c_int32(), ctypes.c_int32(), ctypes.c_int32()
    rc = L.lib().fi_jpeg_info(blob, len(blob), ctypes.byref(w), ctypes.byref(h), ctypes.byref(c))
    return (w.value, h.value, c.value) if rc == L.FI_OK else None


class Context:
    def __init__(self, device: int = 0):
        self._lib = L.lib()
        h = ctypes.c_void_p()
        L.check(self._lib.fi_create(ctypes.byref(h), device))
        self.h = h
        self.device = device

    def close(self):
        if self.h:
            for ptr in list(getattr(self, "_pinned", {})):
                self._lib.fi_host_free(self.h, ptr)
        self._pinned = {}
        if self.h:
            self._lib.fi_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    # ---- host batches ----------------------------------------------------
    def pixelate_regions(self, image: np.ndarray, boxes) -> int:
        """fi_pixelate_regions: the face-blur mogrify (-region box -scale 10%
        -scale 1000%) of each (x, y, w, h) box in order, in place on an 8-bit HWC
        (or HW gray) numpy image.  Returns the C-ABI status (boxes before a
        rejected one are applied, as consecutive mogrify runs would be)."""
        assert image.dtype == np.uint8 and image.flags["C_CONTIGUOUS"]
        h, w = image.shape[:2]
        ch = image.shape[2] if image.ndim == 3 else 1
        flat = [int(v) for b in boxes for v in b]
        arr = (ctypes.c_int32 * max(len(flat), 1))(*flat)
        return self._lib.fi_pixelate_regions(self.h, image.ctypes.data, w, h, image.strides[0], ch, arr,
                                             len(flat) // 4)

    def process(self, images: list[np.ndarray], ops: list[Op]):
        """Run a batch of RGB8 HWC numpy images; returns (outputs, fi_image records)."""
        n = len(images)
        arr = (L.FiImage * n)()
        outs = []
        keep = []
        for i, (src, op) in enumerate(zip(images, ops)):
            src = np.ascontiguousarray(src, dtype=np.uint8)
            keep.append(src)
            img = arr[i]
            img.src = src.ctypes.data
            img.src_h, img.src_w = src.shape[:2]
            img.src_stride = src.strides[0]
            img.src_channels = src.shape[2] if src.ndim == 3 else 1
            _fill(img, op)
        L.lib().fi_plan(arr, n)  # per-image status decides below
        for i in range(n):
            cap = max(arr[i].out_w * arr[i].out_h * max(arr[i].out_channels, 1), 1)
            buf = np.zeros(cap, np.uint8)
            outs.append(buf)
            arr[i].dst = buf.ctypes.data
            arr[i].dst_capacity = cap
        rc = self._lib.fi_process_batch(self.h, arr, n)
        results = []
        for i in range(n):
            a = arr[i]
            if a.status == L.FI_OK:
                o = outs[i][: a.out_h * a.out_stride].reshape(a.out_h, a.out_w, a.out_channels)
                results.append(o[:, :, 0] if a.out_channels == 1 else o)
            else:
                results.append(None)
        return results, arr, rc

    # ---- pinned host buffers + asynchronous host batches ----------------------
    def host_array(self, shape, dtype=np.uint8) -> np.ndarray:
        """A numpy array over pinned host memory (fi_host_alloc): sources and
        outputs there are copied by DMA directly, overlapping earlier batches.
        Freed with the context (or ``host_free``)."""
        nbytes = int(np.prod(shape)) * np.dtype(dtype).itemsize
        ptr = self._lib.fi_host_alloc(self.h, max(nbytes, 1))
        if not ptr:
            raise MemoryError(L.lib().fi_last_error().decode())
        buf = (ctypes.c_uint8 * max(nbytes, 1)).from_address(ptr)
        arr = np.frombuffer(buf, dtype=np.uint8, count=nbytes).view(dtype).reshape(shape)
        self._pinned = getattr(self, "_pinned", {})
        self._pinned[ptr] = arr
        return arr

    def host_free(self, arr: np.ndarray):
        ptr = arr.ctypes.data
        if ptr in getattr(self, "_pinned", {}):
            del self._pinned[ptr]
            L.check(self._lib.fi_host_free(self.h, ptr))

    def submit(self, images: list[np.ndarray], ops: list[Op], outs: list[np.ndarray] | None = None):
        """fi_submit_batch: queue a batch of host images; returns (FiImage array,
        output buffers) whose contents are final after ``wait()``.  Buffers from
        ``host_array`` go by DMA directly; others through the library's pinned
        staging.  ``images`` / ``outs`` must stay alive until then."""
        n = len(images)
        arr = (L.FiImage * n)()
        for i, (src, op) in enumerate(zip(images, ops)):
            img = arr[i]
            img.src = src.ctypes.data
            img.src_h, img.src_w = src.shape[:2]
            img.src_stride = src.strides[0]
            img.src_channels = src.shape[2] if src.ndim == 3 else 1
            _fill(img, op)
        L.lib().fi_plan(arr, n)
        if outs is None:
            outs = [np.zeros(max(arr[i].out_w * arr[i].out_h * max(arr[i].out_channels, 1), 1), np.uint8)
                    for i in range(n)]
        for i in range(n):
            arr[i].dst = outs[i].ctypes.data
            arr[i].dst_capacity = outs[i].nbytes
        L.check(self._lib.fi_submit_batch(self.h, arr, n))
        return arr, outs

    @staticmethod
    def views(arr, outs):
        """Per image: the HWC (or HW) output view of a finished batch, or None."""
        res = []
        for i in range(len(outs)):
            a = arr[i]
            if a.status != L.FI_OK:
                res.append(None)
                continue
            o = outs[i].reshape(-1)[: a.out_h * a.out_stride].reshape(a.out_h, a.out_w, a.out_channels)
            res.append(o[:, :, 0] if a.out_channels == 1 else o)
        return res

    # ---- smartcrop (smartcrop.py SmartCrop().crop) ---------------------------
    def smartcrop_ex(self, rgb: np.ndarray, width: int, height: int, params=None, options=None,
                     want_images: bool = False):
        rgb = np.ascontiguousarray(rgb, dtype=np.uint8)
        h, w = rgb.shape[:2]
        step, nsc = 8, 2
        if options is not None:  # crops() positions per scale x scales
            step = max(int(options.step), 1)
            nsc = int((options.max_scale - options.min_scale) / max(options.scale_step, 1e-9) + 1.5) + 1
        cap = nsc * ((w + step - 1) // step + 1) * ((h + step - 1) // step + 1) + 16
        crops = (L.FiCropScore * cap)()
        n, top = ctypes.c_int32(), ctypes.c_int32()
        awh = (ctypes.c_int32 * 2)()
        pre = ctypes.c_double()
        ocap = w * h * 3
        pbuf = np.zeros(ocap, np.uint8) if want_images else None
        mbuf = np.zeros(ocap, np.uint8) if want_images else None
        rc = self._lib.fi_smartcrop_ex(
            self.h, rgb.ctypes.data, w, h, rgb.strides[0], width, height,
            ctypes.byref(params) if params is not None else None,
            ctypes.byref(options) if options is not None else None,
            crops, cap, ctypes.byref(n), ctypes.byref(top), awh, ctypes.byref(pre),
            pbuf.ctypes.data if want_images else None, mbuf.ctypes.data if want_images else None, ocap)
        L.check(rc)
        out = {"n": n.value, "top_index": top.value, "analyse_size": (awh[0], awh[1]),
               "prescale": pre.value, "crops": [crops[k] for k in range(n.value)]}
        if want_images:
            na = awh[0] * awh[1] * 3
            out["prescaled"] = pbuf[:na].reshape(awh[1], awh[0], 3)
            out["maps"] = mbuf[:na].reshape(awh[1], awh[0], 3)
        return out

    # ---- device memory -------------------------------------------------------
    def malloc(self, nbytes: int) -> int:
        p = ctypes.c_void_p()
        L.check(self._lib.fi_device_malloc(self.h, ctypes.byref(p), nbytes))
        return p.value

    def free(self, ptr: int):
        L.check(self._lib.fi_device_free(self.h, ptr))

    def h2d(self, dptr: int, arr: np.ndarray):
        arr = np.ascontiguousarray(arr)
        L.check(self._lib.fi_memcpy_h2d(self.h, dptr, arr.ctypes.data, arr.nbytes))

    def d2h(self, dptr: int, nbytes: int) -> np.ndarray:
        out = np.empty(nbytes, np.uint8)
        L.check(self._lib.fi_memcpy_d2h(self.h, out.ctypes.data, dptr, nbytes))
        return out

    def jpeg_decode(self, blobs: list[bytes], dptrs: list[int], strides: list[int], channels: int = 0) -> list[int]:
        """fi_jpeg_decode_device: decodes baseline JPEG byte strings into the
        device buffers ``dptrs`` (HWC rows of ``strides`` bytes; channels as
        jpeg_info says, or 3 for every image with ``channels=3``: gray
        replicated); returns the per-image status (0 = decoded,
        FI_EUNSUPPORTED = decode that one on the host)."""
        n = len(blobs)
        bufs = [ctypes.c_char_p(b) for b in blobs]  # the bytes objects' own storage, no copy
        data = (ctypes.c_void_p * n)(*[ctypes.cast(b, ctypes.c_void_p).value for b in bufs])
        lens = (ctypes.c_size_t * n)(*[len(b) for b in blobs])
        dst = (ctypes.c_void_p * n)(*dptrs)
        st = (ctypes.c_int64 * n)(*strides)
        status = (ctypes.c_int32 * n)()
        rc = self._lib.fi_jpeg_decode_device(self.h, data, lens, n, dst, st, channels, status)
        if rc not in (L.FI_OK, L.FI_EUNSUPPORTED, L.FI_EINVAL):
            L.check(rc)
        return list(status)

    def jpeg_decode_host(self, blobs: list[bytes]) -> list[np.ndarray | None]:
        """jpeg_decode into scratch device buffers, copied back (tests / tools):
        HWC uint8 arrays (H, W, 3) or (H, W) for gray; None where the GPU
        decoder returned a non-zero status."""
        infos = [jpeg_info(b) for b in blobs]
        sizes = [(i[0] * i[1] * i[2]) if i else 1 for i in infos]
        ptrs = [self.malloc(max(sz, 1)) for sz in sizes]
        try:
            status = self.jpeg_decode(blobs, ptrs, [(i[0] * i[2]) if i else 1 for i in infos])
            out = []
            for info, p, sz, s in zip(infos, ptrs, sizes, status):
                if s != 0 or not info:
                    out.append(None)
                    continue
                w, h, c = info
                a = self.d2h(p, sz)
                out.append(a.reshape(h, w, 3) if c == 3 else a.reshape(h, w))
            return out
        finally:
            for p in ptrs:
                self.free(p)

    def process_device_views(self, views, ops: list[Op]):
        """fi_process_batch_device on device-resident RGB8 sources given as
        (device pointer, width, height, stride) views (e.g. fi_jpeg_decode_device
        targets, extract offsets applied); outputs land in a scratch device
        buffer and come back as host arrays: (outputs, fi_image records, rc)
        like ``process``."""
        n = len(views)
        arr = (L.FiImage * max(n, 1))()
        for i, ((p, w, h, st), op) in enumerate(zip(views, ops)):
            a = arr[i]
            a.src, a.src_w, a.src_h, a.src_stride, a.src_channels = p, w, h, st, 3
            _fill(a, op)
        L.lib().fi_plan(arr, n)
        caps = [max(arr[i].out_w * arr[i].out_h * max(arr[i].out_channels, 1), 1) for i in range(n)]
        offs = np.concatenate([[0], np.cumsum([(c + 255) // 256 * 256 for c in caps])]).astype(np.int64)
        base = self.malloc(int(offs[-1]) if n else 256)
        try:
            for i in range(n):
                arr[i].dst, arr[i].dst_capacity = base + int(offs[i]), caps[i]
            rc = self._lib.fi_process_batch_device(self.h, arr, n)
            results = []
            for i in range(n):
                a = arr[i]
                if a.status == L.FI_OK:
                    o = self.d2h(base + int(offs[i]), a.out_h * a.out_stride)
                    o = o.reshape(a.out_h, a.out_stride)[:, : a.out_w * a.out_channels]
                    o = o.reshape(a.out_h, a.out_w, a.out_channels)
                    results.append(o[:, :, 0] if a.out_channels == 1 else o)
                else:
                    results.append(None)
        finally:
            self.free(base)
        return results, [arr[i] for i in range(n)], rc

    def fill_synthetic(self, dptr: int, w: int, h: int, stride: int, seed: int):
        L.check(self._lib.fi_fill_synthetic(self.h, dptr, w, h, stride, seed & 0xFFFFFFFF))

    def process_device(self, arr, n: int) -> int:
        """fi_process_batch_device on a prepared FiImage array (device pointers)."""
        return self._lib.fi_process_batch_device(self.h, arr, n)

    def submit_device(self, arr, n: int) -> int:
        """fi_submit_batch_device: plan + upload + launch, returns before the GPU
        finishes; ``arr`` must stay alive until ``wait()``."""
        return self._lib.fi_submit_batch_device(self.h, arr, n)

    def wait(self, keep: int = 0) -> int:
        """fi_wait: finalize submitted batches (oldest first) until at most
        ``keep`` remain in flight, filling their records."""
        return self._lib.fi_wait(self.h, keep)

    def query(self) -> int:
        """fi_query: how many submitted batches are still running on the GPU
        (does not block)."""
        n = ctypes.c_int32()
        L.check(self._lib.fi_query(self.h, ctypes.byref(n)))
        return n.value

    # ---- timing ----------------------------------------------------------------
    def set_timing(self, on):
        """True / 1: every stage timed; 2: the resample stage only; False / 0: off."""
        L.check(self._lib.fi_set_timing(self.h, int(on)))

    def reset_stats(self):
        L.check(self._lib.fi_reset_stats(self.h))

    def stats(self, name: str):
        ms, n, b = ctypes.c_double(), ctypes.c_int64(), ctypes.c_double()
        L.check(self._lib.fi_kernel_stats(self.h, name.encode(), ctypes.byref(ms), ctypes.byref(n), ctypes.byref(b)))
        return ms.value, n.value, b.value

    def monochrome_q16(self, gray: np.ndarray, rot: int = 0) -> np.ndarray:
        """Test hook: the -monochrome kernels on a Q16 gray image (fi_debug_monochrome)."""
        g = np.ascontiguousarray(gray, dtype=np.uint16)
        h, w = g.shape
        oh, ow = (w, h) if rot in (90, 270) else (h, w)
        out = np.zeros((oh, ow), np.uint8)
        L.check(self._lib.fi_debug_monochrome(self.h, g.ctypes.data, w, h, rot, out.ctypes.data, ow))
        return out

    def convolve_q16(self, q16: np.ndarray, conv, ops: int) -> np.ndarray:
        """Test hook: the forwarded convolution kernels on a Q16 HWC image
        (fi_debug_convolve); conv = unsharp[4] + sharpen[2] + blur[2]."""
        q = np.ascontiguousarray(q16, dtype=np.uint16)
        h, w = q.shape[:2]
        ch = q.shape[2] if q.ndim == 3 else 1
        cv = (ctypes.c_double * 8)(*conv)
        out = np.zeros(q.shape, np.uint8)
        L.check(self._lib.fi_debug_convolve(self.h, q.ctypes.data, w, h, ch, cv, ops, out.ctypes.data))
        return out


def device_count() -> int:
    n = ctypes.c_int32()
    L.check(L.lib().fi_device_count(ctypes.byref(n)))
    return n.value
