#!/usr/bin/env python3
"""End-to-end throughput of the host codec pipeline (flyimg_amd/codec.py):
JPEG 1920x1080 q90 in -> decode (threads) -> GPU w_500,smc_1 -> JPEG q90 out,
batches of --batch images, first serially (decode, fi_process_batch with
pageable buffers, encode), then pipelined (CodecPipeline.process_batches:
decode into pinned slots, fi_submit_batch, encode of batch k during batch
k+1), then with the JPEGs decoded on the GPU (CodecPipeline gpu_decode).
Prints one JSON line with the stage splits; gpu_path_share = host time
blocked on the GPU path / wall."""
import argparse
import io
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--images", type=int, default=256)
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--threads", type=int, default=16)
    ap.add_argument("--options", default="w_500,smc_1,q_90")
    a = ap.parse_args()
    import numpy as np
    from PIL import Image

    from flyimg_amd import codec
    from flyimg_amd.runtime import Context
    from flyimg_amd.synth import synth_rgb

    blobs = []
    for i in range(8):
        b = io.BytesIO()
        Image.fromarray(synth_rgb(1920, 1080, 100 + i)).save(b, "JPEG", quality=90)
        blobs.append(b.getvalue())
    ctx = Context(0)
    pipe = codec.CodecPipeline(ctx, a.threads, gpu_decode=False)
    pipe.process(blobs[:2], [a.options] * 2)  # warm
    t_dec = t_gpu = t_enc = 0.0
    t0 = time.perf_counter()
    done = 0
    while done < a.images:
        n = min(a.batch, a.images - done)
        batch = [blobs[(done + k) % len(blobs)] for k in range(n)]
        s0 = time.perf_counter()
        px = list(pipe.pool.map(codec.decode, batch))
        s1 = time.perf_counter()
        from flyimg_amd.processor import ImageProcessor, OptionsBag
        ops = [ImageProcessor(OptionsBag(a.options), 1920, 1080).to_op()] * n
        outs, recs, rc = ctx.process([np.ascontiguousarray(p) for p in px], ops)
        s2 = time.perf_counter()
        list(pipe.pool.map(lambda o: codec.encode(o, 90), outs))
        s3 = time.perf_counter()
        t_dec += s1 - s0
        t_gpu += s2 - s1
        t_enc += s3 - s2
        done += n
    el = time.perf_counter() - t0
    serial = {"images": done, "images_per_s": round(done / el, 1),
              "input_mpix_per_s": round(done * 1920 * 1080 / 1e6 / el, 1), "wall_s": round(el, 3),
              "s_decode": round(t_dec, 3), "s_gpu_host_path": round(t_gpu, 3), "s_encode": round(t_enc, 3),
              "gpu_path_share": round(t_gpu / el, 4)}
    # pipelined: decode of batch k+1 into pinned memory + async submit overlap
    # batch k's DMA / kernels; batch k is encoded while k+1 runs
    batches = []
    done = 0
    while done < a.images:
        n = min(a.batch, a.images - done)
        batches.append(([blobs[(done + k) % len(blobs)] for k in range(n)], [a.options] * n))
        done += n
    for _ in pipe.process_batches(batches[:2]):  # warm the pinned slots
        pass
    t0 = time.perf_counter()
    got = sum(len(enc) for enc, _ in pipe.process_batches(batches))
    el = time.perf_counter() - t0
    st = pipe.stats
    piped = {"images": got, "images_per_s": round(got / el, 1), "input_mpix_per_s": round(got * 1920 * 1080 / 1e6 / el, 1),
             "wall_s": round(el, 3), "s_decode": round(st["s_decode"], 3), "s_gpu_wait": round(st["s_gpu_wait"], 3),
             "s_encode": round(st["s_encode"], 3), "gpu_path_share": round(st["s_gpu_wait"] / el, 4)}
    # GPU decode: CodecPipeline.process decodes the (baseline YCbCr) JPEGs on
    # the MI355X into device memory (fi_jpeg_decode_device), one device batch,
    # host threads only encode the outputs
    gpipe = codec.CodecPipeline(ctx, a.threads, gpu_decode=True)
    gpipe.process(blobs[:2], [a.options] * 2)  # warm
    t0 = time.perf_counter()
    done = 0
    while done < a.images:
        n = min(a.batch, a.images - done)
        gpipe.process([blobs[(done + k) % len(blobs)] for k in range(n)], [a.options] * n)
        done += n
    el = time.perf_counter() - t0
    gdec = {"images": done, "images_per_s": round(done / el, 1),
            "input_mpix_per_s": round(done * 1920 * 1080 / 1e6 / el, 1), "wall_s": round(el, 3)}
    gpipe.close()
    print(json.dumps({"batch": a.batch, "threads": a.threads, "options": a.options, "serial": serial,
                      "pipelined": piped, "gpu_decode": gdec}))
    pipe.close()
    ctx.close()


if __name__ == "__main__":
    main()
