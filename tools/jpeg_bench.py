#!/usr/bin/env python3
"""GPU JPEG decode throughput (fi_jpeg_decode_device) vs Pillow's
libjpeg-turbo on the host threads, on synthetic 1920x1080 q90 4:2:0 JPEGs
(the cfg2 source size); prints one JSON line.  The GPU figure is the wall
time of the C-ABI call: header parse + H2D of the compressed bytes + the
three kernels, into a device-resident pool."""
import io
import json
import os
import sys
import time
from concurrent.futures import ThreadPoolExecutor

import numpy as np
from PIL import Image

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from flyimg_amd.runtime import Context, jpeg_info  # noqa: E402
from flyimg_amd.synth import synth_rgb  # noqa: E402

N = int(os.environ.get("NIMG", "256"))
W, H = int(os.environ.get("JW", "1920")), int(os.environ.get("JH", "1080"))
REPS = int(os.environ.get("REPS", "5"))
THREADS = int(os.environ.get("THREADS", "16"))


def enc(i):
    b = io.BytesIO()
    Image.fromarray(synth_rgb(W, H, 100 + i)).save(b, "JPEG", quality=90, subsampling=2)
    return b.getvalue()


pool = ThreadPoolExecutor(THREADS)
uniq = list(pool.map(enc, range(min(N, 32))))
blobs = [uniq[i % len(uniq)] for i in range(N)]
assert all(jpeg_info(b) == (W, H, 3) for b in uniq)
mb = sum(len(b) for b in blobs) / 1e6

t0 = time.perf_counter()
for _ in range(2):
    host = list(pool.map(lambda b: np.asarray(Image.open(io.BytesIO(b))), blobs))
host_s = (time.perf_counter() - t0) / 2

with Context(0) as ctx:
    stride = W * 3
    base = ctx.malloc(stride * H * N)
    ptrs = [base + i * stride * H for i in range(N)]
    st = ctx.jpeg_decode(blobs, ptrs, [stride] * N)  # warm-up (allocations)
    assert st == [0] * N, st
    ts = []
    for _ in range(REPS):
        t0 = time.perf_counter()
        ctx.jpeg_decode(blobs, ptrs, [stride] * N)
        ts.append(time.perf_counter() - t0)
    gpu_s = float(np.median(ts))
    # spot-check the decoded pool against the host decode
    for i in (0, N // 2, N - 1):
        got = ctx.d2h(ptrs[i], stride * H).reshape(H, W, 3)
        assert np.array_equal(got, host[i]), i
    ctx.free(base)

print(json.dumps({
    "images": N, "size": f"{W}x{H}", "jpeg": "q90 4:2:0 (Pillow)", "compressed_MB": round(mb, 1),
    "gpu_decode_s": round(gpu_s, 4), "gpu_images_per_s": round(N / gpu_s, 1),
    "gpu_input_Mpix_per_s": round(N * W * H / gpu_s / 1e6, 1),
    "host_decode_s": round(host_s, 4), "host_threads": THREADS, "host_images_per_s": round(N / host_s, 1),
    "bit_exact_spot_check": True,
}))
