"""Host codec pipeline around the GPU path:
ImageHandler::processNewImage end to end for a batch of encoded images.

  decode   Pillow (libjpeg-turbo / libpng) on a thread pool -- the decoders
           release the GIL -- with ``-auto-orient`` (ImageProcessor.php:78)
           applied from the EXIF orientation, then ExtractProcessor's view;
  process  ONE fi_process_batch for the whole batch (ImageProcessor +
           SmartCropProcessor on the MI355X);
  encode   on the thread pool: JPEG at ``q_`` (default 90) -- flyimg pipes
           TGA into MozJPEG's cjpeg when it is executable and otherwise lets
           ImageMagick write the JPEG with ``-quality`` (calculateQuality,
           ImageProcessor.php:195-217); neither ``cjpeg`` nor ``convert`` is
           in this image, so the encoder is libjpeg-turbo at the same quality
           (IM's own JPEG coder is libjpeg as well).  Images with alpha are
           written as PNG.

Gray (L), bilevel and palette sources are expanded to RGB / RGBA before the
GPU (IM would keep a gray JPEG gray: the channels are equal either way), and
flagged FI_SRC_PSEUDOCLASS: IM's readers give them a colormap (1-component
JPEG, palette / 8-bit gray PNG, GIF), so ResizeImage filters them with
Mitchell instead of Lanczos (resize.c).
"""
from __future__ import annotations

import io
from concurrent.futures import ThreadPoolExecutor

import numpy as np

from . import _lib as L
from .processor import ExecFailedException, ExtractProcessor, ImageProcessor, OptionsBag, _empty


# Pillow modes whose IM reading is a PseudoClass image: bilevel, 8-bit gray and
# palette (16-bit gray "I;16" / "I" stays DirectClass, depth > 8)
PSEUDOCLASS_MODES = ("1", "L", "P")


def decode_ex(blob: bytes):
    """Encoded bytes -> (HWC uint8 RGB, or RGBA when the file has alpha, EXIF
    orientation applied (-auto-orient); True when IM would read a PseudoClass
    image)."""
    from PIL import Image, ImageOps

    im = Image.open(io.BytesIO(blob))
    im = ImageOps.exif_transpose(im)
    pseudo = im.mode in PSEUDOCLASS_MODES
    alpha = im.mode in ("RGBA", "LA", "PA") or (im.mode == "P" and "transparency" in im.info)
    im = im.convert("RGBA" if alpha else "RGB")
    return np.asarray(im), pseudo


def decode(blob: bytes) -> np.ndarray:
    """decode_ex without the class flag."""
    return decode_ex(blob)[0]


def encode(pixels: np.ndarray, quality: int = 90) -> bytes:
    from PIL import Image

    buf = io.BytesIO()
    ch = pixels.shape[2] if pixels.ndim == 3 else 1
    if ch in (2, 4):  # alpha survives: PNG
        Image.fromarray(pixels, "LA" if ch == 2 else "RGBA").save(buf, "PNG")
    else:
        # IM 6 coders/jpeg.c: without -sampling-factor, quality >= 90 writes 1x1
        # (4:4:4) chroma and lower qualities 2x2 (4:2:0).  (MozJPEG's cjpeg, the
        # reference's path when it is installed, always uses 2x2.)
        Image.fromarray(pixels, "L" if ch == 1 else "RGB").save(
            buf, "JPEG", quality=int(quality), subsampling=0 if int(quality) >= 90 else 2)
    return buf.getvalue()


class _PinnedSlot:
    """One in-flight batch's pinned host memory (fi_host_alloc): the decoded
    sources and the GPU outputs, sliced per image (256-B aligned), grown on
    demand.  Two slots: batch k+1 decodes into one while batch k's DMA and
    kernels use the other."""

    def __init__(self, ctx):
        self.ctx, self.src, self.dst = ctx, None, None

    def _grow(self, which, nbytes):
        cur = getattr(self, which)
        if cur is None or cur.nbytes < nbytes:
            if cur is not None:
                self.ctx.host_free(cur)
            setattr(self, which, self.ctx.host_array((max(nbytes, 1 << 20),)))
        return getattr(self, which)

    @staticmethod
    def _slices(buf, sizes):
        out, off = [], 0
        for n in sizes:
            out.append(buf[off:off + n])
            off += (n + 255) // 256 * 256
        return out

    def sources(self, shapes):
        sizes = [int(np.prod(s)) for s in shapes]
        buf = self._grow("src", sum((n + 255) // 256 * 256 for n in sizes))
        return [v.reshape(s) for v, s in zip(self._slices(buf, sizes), shapes)]

    def outputs(self, sizes):
        buf = self._grow("dst", sum((n + 255) // 256 * 256 for n in sizes))
        return self._slices(buf, sizes)


def gpu_decodable(blob: bytes):
    """(width, height, source channels) when the GPU decoder
    (fi_jpeg_decode_device, RGB output) produces exactly what decode_ex would:
    a baseline gray or YCbCr JPEG (fi_jpeg_info) with no EXIF rotation to
    apply; None otherwise (progressive, CMYK, PNG, ...).  A gray (1-component)
    JPEG is an IM PseudoClass source, as decode_ex flags it."""
    from PIL import Image

    from .runtime import jpeg_info

    info = jpeg_info(blob)
    if not info:
        return None
    try:
        orientation = Image.open(io.BytesIO(blob)).getexif().get(0x0112, 1)  # headers only
    except Exception:  # noqa: BLE001 - unreadable EXIF: let the host path decide
        return None
    return info if orientation in (0, 1) else None


class CodecPipeline:
    """Batches of encoded images through decode -> GPU -> encode.  With
    ``gpu_decode`` (default) baseline gray / YCbCr JPEGs are decoded on the MI355X
    straight into device memory (bit-exact with the host decoder) and only
    the other sources take the host decoder."""

    def __init__(self, ctx, threads: int = 16, gpu_decode: bool = True):
        self.ctx = ctx
        self.pool = ThreadPoolExecutor(max_workers=max(1, threads))
        self.gpu_decode = gpu_decode

    def close(self):
        self.pool.shutdown()

    @staticmethod
    def _quality(bag):
        q = bag.get_option("quality")
        return int(q) if not _empty(q) else 90

    def _host_batch(self, blobs, bags):
        decoded = list(self.pool.map(decode_ex, blobs))
        srcs, ops = [], []
        for (img, pseudo), bag in zip(decoded, bags):
            img = ExtractProcessor.extract(bag, img)
            h, w = img.shape[:2]
            op = ImageProcessor(bag, w, h).to_op()
            if pseudo:
                op.flags |= L.FI_SRC_PSEUDOCLASS
            ops.append(op)
            srcs.append(np.ascontiguousarray(img))
        outs, recs, _ = self.ctx.process(srcs, ops)
        return outs, list(recs)

    def _gpu_batch(self, blobs, bags, dims):
        """GPU decode into one device pool (16-B aligned rows for the streaming
        resample kernels), one device batch.
        Returns (outputs, records, indices the GPU decoder turned down)."""
        strides = [(w * 3 + 15) // 16 * 16 for w, _, _ in dims]
        offs = np.concatenate([[0], np.cumsum([(s * h + 255) // 256 * 256 for s, (_, h, _) in zip(strides, dims)])])
        base = self.ctx.malloc(int(offs[-1]))
        try:
            ptrs = [base + int(o) for o in offs[:-1]]
            status = self.ctx.jpeg_decode(blobs, ptrs, strides, channels=3)
            views, ops, keep = [], [], []
            for i, (bag, (w, h, c), p, st) in enumerate(zip(bags, dims, ptrs, strides)):
                if status[i] != L.FI_OK:
                    continue
                views.append((p, w, h, st))
                op = ImageProcessor(bag, w, h).to_op()
                if c == 1:  # 1-component JPEG: IM PseudoClass (Mitchell), as decode_ex flags it
                    op.flags |= L.FI_SRC_PSEUDOCLASS
                ops.append(op)
                keep.append(i)
            outs, recs, _ = self.ctx.process_device_views(views, ops)
        finally:
            self.ctx.free(base)
        full_o, full_r = [None] * len(blobs), [None] * len(blobs)
        for k, i in enumerate(keep):
            full_o[i], full_r[i] = outs[k], recs[k]
        return full_o, full_r, [i for i in range(len(blobs)) if status[i] != L.FI_OK]

    def process(self, blobs: list[bytes], options: list[str]):
        """Returns (encoded outputs, fi_image records); a failed image raises
        ExecFailedException as Processor::execute does."""
        bags = [OptionsBag(o) for o in options]
        n = len(blobs)
        outs, recs = [None] * n, [None] * n
        # extract (e_1) views start at any byte: the host path copies them to an
        # aligned array, so they decode there and take the same kernels
        # (bag.get: extract_key would consume the option, as InputImage::extractKey does)
        dims = [gpu_decodable(b) if self.gpu_decode and _empty(bag.get("extract")) else None
                for b, bag in zip(blobs, bags)]
        host = [i for i in range(n) if dims[i] is None]
        gpu = [i for i in range(n) if dims[i] is not None]
        if gpu:
            o, r, back = self._gpu_batch([blobs[i] for i in gpu], [bags[i] for i in gpu], [dims[i] for i in gpu])
            for k, i in enumerate(gpu):
                outs[i], recs[i] = o[k], r[k]
            host += [gpu[k] for k in back]
        if host:
            o, r = self._host_batch([blobs[i] for i in host], [bags[i] for i in host])
            for k, i in enumerate(host):
                outs[i], recs[i] = o[k], r[k]
        for i, r in enumerate(recs):
            if r.status != L.FI_OK:
                msg = L.lib().fi_last_error()
                raise ExecFailedException("Command failed.\nThe exit code: %d\n%s" % (
                    r.status, msg.decode() if msg else f"image {i}"))
        encoded = list(self.pool.map(lambda a: encode(a[0], a[1]), zip(outs, [self._quality(b) for b in bags])))
        return encoded, recs

    def _prepare(self, slot, blobs, options):
        """Decode (thread pool) straight into the slot's pinned sources; ops."""
        decoded = list(self.pool.map(decode_ex, blobs))
        views, ops, quality = [], [], []
        for (img, pseudo), opts in zip(decoded, options):
            bag = OptionsBag(opts)
            img = ExtractProcessor.extract(bag, img)
            h, w = img.shape[:2]
            q = bag.get_option("quality")
            quality.append(int(q) if not _empty(q) else 90)
            op = ImageProcessor(bag, w, h).to_op()
            if pseudo:
                op.flags |= L.FI_SRC_PSEUDOCLASS
            ops.append(op)
            views.append(img)
        pins = slot.sources([v.shape for v in views])
        list(self.pool.map(lambda a: np.copyto(a[0], a[1]), zip(pins, views)))
        return pins, ops, quality

    def process_batches(self, batches):
        """Pipelined form of ``process`` over an iterable of (blobs, options)
        batches: batch k+1 is decoded into pinned memory and submitted
        (fi_submit_batch) while batch k's DMA and kernels run, and batch k is
        encoded while batch k+1 runs.  Yields (encoded outputs, records) per
        batch, in order; the ``stats`` attribute holds the host time spent
        decoding, blocked on the GPU, and encoding."""
        from .runtime import plan as fi_plan

        slots = [_PinnedSlot(self.ctx), _PinnedSlot(self.ctx)]
        self.stats = {"s_decode": 0.0, "s_gpu_wait": 0.0, "s_encode": 0.0}
        import time

        prev = None
        for k, (blobs, options) in enumerate(batches):
            t0 = time.perf_counter()
            slot = slots[k % 2]
            srcs, ops, quality = self._prepare(slot, blobs, options)
            sizes = []
            for src, op in zip(srcs, ops):
                ow, oh, oc = fi_plan(src.shape[1], src.shape[0], op)
                sizes.append(max(ow * oh * oc, 1))
            outs = slot.outputs(sizes)
            arr, outs = self.ctx.submit(srcs, ops, outs)
            t1 = time.perf_counter()
            self.stats["s_decode"] += t1 - t0
            if prev is not None:
                yield self._finish(prev, keep=1)
            prev = (arr, outs, quality, srcs)
        if prev is not None:
            yield self._finish(prev, keep=0)

    def _finish(self, batch, keep):
        import time

        arr, outs, quality, _ = batch
        t0 = time.perf_counter()
        self.ctx.wait(keep)  # that batch is final (its failures are in its records)
        t1 = time.perf_counter()
        for i in range(len(outs)):
            if arr[i].status != L.FI_OK:
                msg = L.lib().fi_last_error()
                raise ExecFailedException("Command failed.\nThe exit code: %d\n%s" % (
                    arr[i].status, msg.decode() if msg else f"image {i}"))
        views = self.ctx.views(arr, outs)
        encoded = list(self.pool.map(lambda a: encode(np.ascontiguousarray(a[0]), a[1]), zip(views, quality)))
        self.stats["s_gpu_wait"] += t1 - t0
        self.stats["s_encode"] += time.perf_counter() - t1
        return encoded, arr
