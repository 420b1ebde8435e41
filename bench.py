#!/usr/bin/env python3
"""flyimg hot-path benchmark on MI355X (contract: see README / DESIGN.md).

  python bench.py [--gpus N] [--steps K] [--warmup W] [--workload cfg2]

Ranks: under torch.distributed.run (WORLD_SIZE set) each process is one rank
and WORLD_SIZE must equal --gpus; without a launcher, --gpus N > 1 starts N
rank processes itself (launch_ranks) and relays rank 0's line.

One step = one batch (fi_submit_batch_device; batch k+1 is planned on the
host while batch k runs, every batch is finalized inside the timed region) over the rank's device-resident
batch of synthetic RGB8 images (inputs already in HBM when timing starts):
ImageMagick-semantics resample -> smartcrop (prescale, maps, scoring, argmax)
-> crop apply, plus -- for N > 1 -- the RCCL gather of the per-image result
records to rank 0.  Default workload = BASELINE.json configs[1] (cfg2:
1024 x 1920x1080 -> w_500,smc_1 per GPU, weak scaling).

value = input Mpix of all ranks / max-over-ranks wall time of the K steps.
Rank 0 prints ONE JSON line.  No torch import: the control plane is
flyimg_amd.parallel (file rendezvous), RCCL is called by libflyimg_hip.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

METRIC = "input Mpix/s resize+smartcrop at 1/2/4/8 MI355X; % of HBM roofline"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md: 8.0 TB/s)

WORKLOADS = {
    # name: (W, H, images per GPU, options, BASELINE config text)
    "cfg2": (1920, 1080, 1024, "w_500,smc_1", "configs[1]: batch of 1024 1920x1080 RGB -> w_500,smc_1 smart-crop"),
    "cfg3": (3840, 2160, 4096, "w_512,h_512,c_1", "configs[2]: batch of 4096 3840x2160 RGB -> 512x512 Lanczos thumbnails c_1"),
    "cfg5": (6000, 4000, 1024, "w_400,h_400,c_1,r_90,clsp_Gray,smc_1", "configs[4]: 6000x4000 batch -> w_400,h_400,c_1,r_90,clsp_Gray,smc_1"),
    "cfg1": (3000, 2000, 1024, "w_300,h_250,c_1", "configs[0] geometry on the GPU: 3000x2000 -> w_300,h_250,c_1"),
    # cfg4 is a mixed list, not one geometry (see cfg4_list / run_cfg4)
    "cfg4": (0, 0, 65536, "mixed", "configs[3]: 65536 mixed-size images (0.5-24 MP), multiple output sizes, "
                                    "sharded across GPUs"),
}

CFG4_OPS = ["w_300,h_250,c_1", "w_500,smc_1", "w_512,h_512,c_1", "h_300", "w_400,h_400,c_1"]
CFG4_ASPECTS = [4 / 3, 3 / 2, 16 / 9, 1.0, 2 / 3, 9 / 16]
CFG4_MP_CLASSES = 64


def cfg4_list(n=65536, seed=20250112):
    """megapixels log-uniform in [0.5, 24] (64 log-spaced
    classes, like the finite set of camera resolutions a service sees), aspect
    from {4:3, 3:2, 16:9, 1:1, 2:3, 9:16}, ops cycling through the cfg1 / cfg2 /
    cfg3 ops, h_300 and w_400,h_400,c_1.  Returns [(W, H, op_index)]."""
    import numpy as np

    rng = np.random.default_rng(seed)
    mps = np.exp(np.linspace(np.log(0.5), np.log(24.0), CFG4_MP_CLASSES))
    out = []
    ks = rng.integers(0, CFG4_MP_CLASSES, n)
    asp = rng.integers(0, len(CFG4_ASPECTS), n)
    for i in range(n):
        a = CFG4_ASPECTS[int(asp[i])]
        W = max(16, int(round((float(mps[ks[i]]) * 1e6 * a) ** 0.5)))
        H = max(16, int(round(W / a)))
        out.append((W, H, i % len(CFG4_OPS)))
    return out


KERNEL_OF_PATH = {
    "path_vm": "k_rs_vm (streaming exact-integer MFMA, vertical first)",
    "path_vr": "k_rs_vr (persistent block-major exact-integer MFMA, vertical first)",
    "path_hv": "k_rs_hv (streaming exact-integer MFMA, horizontal first)",
    "path_generic_v": "k_rs_v_u8 + k_rs_h_final (two-pass)",
    "path_generic_h": "k_rs_h_u8 + k_rs_v_final (two-pass)",
    "path_copy": "k_rs_copy",
}
# smartcrop prescale + maps kernel per image (counts kept by the library)
SC_KERNEL_OF_PATH = {
    "sc_path_cx": "k_sc_hx + k_sc_vx (prescale + maps, co-resident beside the next batch's resample)",
    "sc_path_fd": "k_sc_fd (prescale + maps, source rows by LDS-DMA)",
    "sc_path_fz": "k_sc_fz (prescale + maps, register-staged source rows)",
}


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def cpu_baseline(W, H, options, budget_s=8.0, threads=None, max_images=None):
    """The oracle restatement (oracle/fi_oracle.c) on the host cores: the same
    per-image work (IM resample -> smartcrop -> crop) on synthetic images of the
    same shape, one image per thread at a time (ctypes releases the GIL, the C
    code has no shared state), for about ``budget_s`` seconds of wall time
    (or until ``max_images`` images are done).
    ImageMagick itself runs its OpenMP loops over the host cores, so the
    baseline uses as many threads as this process' CPU share allows (16 on
    a one-GPU box; ``nproc`` shows the whole machine there)."""
    import threading

    import numpy as np

    from flyimg_amd.processor import ImageProcessor, OptionsBag
    from flyimg_amd.synth import synth_rgb
    from oracle import oracle as orc

    op = ImageProcessor(OptionsBag(options), W, H).to_op()
    from flyimg_amd import _lib as L

    from oracle.verify import oracle_flags

    flags = oracle_flags(op)
    smc = bool(op.flags & L.FI_OP_SMARTCROP)
    if threads is None:
        try:
            share = len(os.sched_getaffinity(0))
        except AttributeError:  # pragma: no cover
            share = os.cpu_count() or 1
        threads = max(1, min(16, share, int(os.environ.get("OMP_NUM_THREADS", "16") or 16)))
    srcs = [synth_rgb(W, H, 0x5EED + i) for i in range(2)]
    counts = [0] * threads

    def one(k):
        src = srcs[k % 2]
        out = orc.im_convert(src, op.target_w, op.target_h, flags, rotate=op.rotate)
        if smc:
            rgb = out if out.ndim == 3 else np.repeat(out[:, :, None], 3, axis=2)
            r = orc.sc_crop(rgb, 100, 100)
            t = r["top_crop"]
            _ = out[t["y"]:t["y"] + t["height"] + t["y"], t["x"]:t["x"] + t["width"] + t["x"]].copy()

    one(0)  # warm the oracle library
    t0 = time.perf_counter()
    deadline = t0 + budget_s

    lock = threading.Lock()
    started = [0]

    def worker(i):
        k = i
        while time.perf_counter() < deadline:
            with lock:
                if max_images is not None and started[0] >= max_images:
                    return
                started[0] += 1
            one(k)
            counts[i] += 1
            k += threads

    ts = [threading.Thread(target=worker, args=(i,)) for i in range(threads)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    wall = time.perf_counter() - t0
    n = sum(counts)
    mpix = n * W * H / 1e6
    return {"value": round(mpix / wall, 4), "unit": "Mpix/s", "cores": threads, "kind": "port",
            "images": n, "wall_s": round(wall, 3),
            "sample": f"{n} images {W}x{H} '{options}' through oracle/fi_oracle.c (IM restatement + smartcrop "
                      f"restatement + crop), {threads} threads, {wall:.1f} s wall; ImageMagick convert and "
                      f"python smartcrop.py are not installed on the GPU box"}


def cfg4_cpu_baseline(items, n_sample=8, threads=None):
    """The oracle on the first ``n_sample`` images of the cfg4 list, each
    image's class timed on its own (``cpu_baseline`` with max_images =
    threads, so every thread does one image): Mpix / summed measured wall."""
    mpix = wall = 0.0
    cores = 0
    done = 0
    for W, H, k in items[:n_sample]:
        r = cpu_baseline(W, H, CFG4_OPS[k], budget_s=30.0, threads=threads, max_images=threads or 16)
        mpix += r["images"] * W * H / 1e6
        wall += r["wall_s"]
        cores = max(cores, r["cores"])
        done += r["images"]
    return {"value": round(mpix / wall, 4) if wall > 0 else None, "unit": "Mpix/s", "cores": cores,
            "kind": "port", "images": done, "wall_s": round(wall, 3),
            "sample": f"{done} images of the first {n_sample} cfg4 (size, op) classes through oracle/fi_oracle.c, "
                      f"{cores} threads (one image per thread per class), {wall:.1f} s measured wall"}


def source_hash():
    """sha256 of the library's sources, as tools/pmc_to_json.py records it"""
    import hashlib

    d = os.path.join(REPO, "flyimg_amd", "csrc")
    h = hashlib.sha256()
    for f in sorted(os.listdir(d)):
        if f.endswith((".hip", ".cpp", ".h")):
            h.update(f.encode())
            h.update(open(os.path.join(d, f), "rb").read())
    return h.hexdigest()


def launch_ranks(n: int) -> int:
    """``bench.py --gpus N`` without an external launcher: start N rank
    processes of this same command (RANK / LOCAL_RANK / WORLD_SIZE, a private
    rendezvous id, MASTER_ADDR 127.0.0.1), relay rank 0's JSON line, and fail
    when any rank fails.  Runs before this process loads the library or
    touches a GPU; the ranks are children, not an exec of this process."""
    import subprocess
    import uuid

    rdzv = f"bench{os.getpid()}_{uuid.uuid4().hex[:8]}"
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=os.environ.get("MASTER_PORT", "29500"), FI_RDZV_ID=rdzv)
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env,
                                      stdout=subprocess.PIPE if r == 0 else subprocess.DEVNULL, text=True))
    log(f"launched {n} ranks (rendezvous {rdzv})")
    import threading

    out0 = []
    reader = threading.Thread(target=lambda: out0.append(procs[0].stdout.read()))
    reader.start()
    # a rank that fails leaves the others waiting in the rendezvous: stop them
    while any(p.poll() is None for p in procs):
        if any(p.poll() not in (None, 0) for p in procs):
            for p in procs:
                if p.poll() is None:
                    p.terminate()
            for p in procs:
                try:
                    p.wait(timeout=30)
                except subprocess.TimeoutExpired:
                    p.kill()
            break
        time.sleep(0.2)
    reader.join()
    rcs = [p.wait() for p in procs]
    lines = [ln for ln in "".join(out0).splitlines() if ln.startswith("{")]
    if any(rcs) or len(lines) != 1:
        log(f"error: rank exit codes {rcs}, {len(lines)} JSON lines from rank 0")
        return 1
    print(lines[0], flush=True)
    return 0


# batches in flight per context: the library's slots (fi_api.cpp kSlots)
PIPE_DEPTH = 3


def run_batches(ctx, arrs, nimg, k0, count, on_done):
    """Batches k0 .. k0+count-1 of one rank, pipelined len(arrs) deep (the
    library's slots): submit batch k (fi_submit_batch_device: planned and
    uploaded while earlier batches run), then finalize batch k-D+1
    (fi_wait(D-1)) and hand its records to on_done.  With the smartcrop stage
    beside the next resample, batch k's stage ends after batch k+1's resample,
    so batch k+2 must be queued before batch k is waited for (D = 3).
    Nothing here waits on another rank: the result gather is the caller's, once
    after the last batch (RCCL on the library's gather stream), so no rank
    blocks its next batch on a collective.  Returns after every batch is
    finalized."""
    from flyimg_amd import _lib as L

    if count <= 0:
        return
    D = len(arrs)
    done = k0
    for k in range(k0, k0 + count):
        L.check(ctx.submit_device(arrs[k % D], nimg))
        if k - done >= D - 1:
            L.check(ctx.wait(D - 1))  # batch `done` finished (later ones still queued)
            on_done(done, arrs[done % D])
            done += 1
    L.check(ctx.wait(0))
    for k in range(done, k0 + count):
        on_done(k, arrs[k % D])


def dry_run(args, rank, world, local_rank, comm):
    """Control-plane rehearsal of a multi-rank run: no library, no GPU.
    ``FI_DRY_RUN_FAIL_RANK=r`` makes rank r exit 3 after joining (launcher test)."""
    if os.environ.get("FI_DRY_RUN_FAIL_RANK") == str(rank):
        sys.exit(3)
    joined = comm.allgather_obj({"rank": rank, "local_rank": local_rank, "pid": os.getpid()})
    comm.barrier()
    if rank == 0:
        print(json.dumps({"dry_run": True, "n_gpus": world, "ranks": [j["rank"] for j in joined],
                          "local_ranks": [j["local_rank"] for j in joined],
                          "distinct_pids": len({j["pid"] for j in joined}), "workload": args.workload}), flush=True)
    comm.close()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--workload", default="cfg2", choices=sorted(WORKLOADS))
    ap.add_argument("--images", type=int, default=0, help="override images per GPU")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--timed-stages", action="store_true",
                    help="diagnostic: every stage's event range inside the timed region (adds gaps)")
    ap.add_argument("--no-verify", action="store_true", help="skip the oracle check of the last timed batch "
                    "(profiling ablations only)")
    ap.add_argument("--dry-run", action="store_true",
                    help="control plane only (no GPU, no library): every rank joins the rendezvous, rank 0 prints "
                         "one JSON line naming the ranks that joined (tests the launcher)")
    args = ap.parse_args()

    # ---- ranks: an external launcher (torch.distributed.run) sets WORLD_SIZE;
    # without one, --gpus N > 1 starts its own N ranks before anything touches
    # the GPU in this process.  A mismatch is an error, never a 1-rank line.
    if "WORLD_SIZE" not in os.environ:
        if args.gpus > 1:
            sys.exit(launch_ranks(args.gpus))
    elif int(os.environ["WORLD_SIZE"]) != args.gpus:
        log(f"error: WORLD_SIZE={os.environ['WORLD_SIZE']} but --gpus {args.gpus}: launch one rank per GPU "
            f"(torch.distributed.run --nproc-per-node {args.gpus}) or run without a launcher")
        sys.exit(2)

    from flyimg_amd.parallel import env_rank_world, make_comm

    rank, world, local_rank = env_rank_world()
    comm = make_comm()
    if args.dry_run:
        return dry_run(args, rank, world, local_rank, comm)

    from flyimg_amd import _lib as L
    from flyimg_amd.parallel import RecordGather
    from flyimg_amd.processor import ImageProcessor, OptionsBag
    from flyimg_amd.runtime import Context

    if args.workload == "cfg4":
        return run_cfg4(args, rank, world, local_rank, comm)
    W, H, nimg, options, cfg_text = WORKLOADS[args.workload]
    if args.images:
        nimg = args.images
    ctx = Context(int(os.environ.get("FI_BENCH_DEVICE", local_rank)))  # override: rehearsal of N ranks on one GPU
    gather = RecordGather(comm, ctx)

    # ---- device-resident synthetic pool (distinct seed per global image) ----
    op = ImageProcessor(OptionsBag(options), W, H).to_op()
    src_stride = (W * 3 + 15) // 16 * 16
    src_bytes = src_stride * H
    from flyimg_amd.runtime import plan as fi_plan

    ow, oh, oc = fi_plan(W, H, op)
    dst_cap = ow * oh * oc
    pool = ctx.malloc(src_bytes * nimg)
    # one output set per in-flight batch (PIPE_DEPTH, the library's slots):
    # batch k+1 resamples while batch k's smart-crop stage still runs
    dsts = [ctx.malloc(dst_cap * nimg) for _ in range(PIPE_DEPTH)]
    t0 = time.perf_counter()
    for i in range(nimg):
        ctx.fill_synthetic(pool + i * src_bytes, W, H, src_stride, 0x5EED + rank * nimg + i)
    log(f"rank {rank}: pool {nimg} x {W}x{H} ({src_bytes * nimg / 1e9:.2f} GB) filled in {time.perf_counter() - t0:.1f} s")
    # one descriptor array per in-flight batch: batch k+2 is planned and
    # launched while batches k, k+1 run (fi_submit_batch_device); batch k's
    # records are finalized once k+2 is queued.
    arrs = [(L.FiImage * nimg)() for _ in range(PIPE_DEPTH)]
    for arr, dst in zip(arrs, dsts):
        for i in range(nimg):
            a = arr[i]
            a.src, a.src_w, a.src_h, a.src_stride, a.src_channels = pool + i * src_bytes, W, H, src_stride, 3
            a.target_w, a.target_h, a.flags, a.gravity, a.rotate = op.target_w, op.target_h, op.flags, op.gravity, op.rotate
            a.smartcrop_w, a.smartcrop_h = op.smartcrop_w, op.smartcrop_h
            a.dst, a.dst_capacity = dst + i * dst_cap, dst_cap
    bad = [0]
    recs = []

    def records(k, arr):
        bad[0] += sum(1 for i in range(nimg) if arr[i].status != 0)
        if world > 1:
            recs.extend((rank * nimg + i, arr[i].status, arr[i].out_w, arr[i].out_h, arr[i].crop_x,
                         arr[i].crop_y, arr[i].crop_w, arr[i].crop_h) for i in range(nimg))

    def run(k0, count):
        """Batches k0..k0+count-1, pipelined, then the final result gather."""
        run_batches(ctx, arrs, nimg, k0, count, records)
        if world > 1:
            gather.gather(recs)  # the one exchange step: every batch's records to rank 0
            recs.clear()

    run(0, args.warmup)
    bad[0] = 0
    # the timed region carries HIP event ranges around the resample stage only
    # (the roofline's live launch time); every other stage's range would add a
    # few microseconds between dependent kernels -- the stage split comes from
    # a separate instrumented pass after the verification below
    ctx.set_timing(1 if args.timed_stages else 2)
    ctx.reset_stats()
    comm.barrier()
    t0 = time.perf_counter()
    run(args.warmup, args.steps)  # ends with every batch drained (stream idle)
    t1 = time.perf_counter()
    comm.barrier()
    ctx.set_timing(False)
    el = t1 - t0
    stats = {k: ctx.stats(k) for k in ("batch", "resize", "sc_prep", "sc_score", "crop_apply",
                                      "host_plan", "host_plan_images", "host_plan_sc", "host_plan_tiles",
                                      "host_plan_blob", "host_launch", "host_wait", "host_total")}
    # images per resample kernel over the timed steps (counts kept by the library)
    paths = {p: ctx.stats(p)[1] // max(args.steps, 1) for p in KERNEL_OF_PATH}
    sc_paths = {p: ctx.stats(p)[1] // max(args.steps, 1) for p in SC_KERNEL_OF_PATH}
    ablation = ctx.stats("vr_ablation")[1]  # FI_VR_VARIANT profiling launches (wrong pixels)
    last = arrs[(args.warmup + args.steps - 1) % PIPE_DEPTH]
    allv = comm.allgather_obj({"elapsed": el, "stats": stats,
                               "ncand": sum(last[i].n_candidates for i in range(nimg)),
                               "bad": bad[0]})
    # correctness of the headline batch itself (untimed): the last timed batch's
    # records and outputs against the oracle, including images past 2^32 of pool
    vlast = (args.warmup + args.steps - 1) % PIPE_DEPTH
    vok, vtot, verr = (0, 0, None)
    if not args.no_verify:
        from oracle.verify import verify_batch, verify_sample  # the checker (test infrastructure)

        vok, vtot, verr = verify_batch(
            ctx, last, verify_sample(nimg, src_bytes), lambda i: pool + i * src_bytes,
            lambda i: 0x5EED + rank * nimg + i, W, H, src_stride, op, lambda i: dsts[vlast] + i * dst_cap, dst_cap)
        if verr:
            log(f"rank {rank}: VERIFY FAILED {vok}/{vtot}: {verr}")
    allv_v = comm.allgather_obj({"ok": vok, "tot": vtot, "err": verr})
    # stage split: an instrumented pass of a few more batches, every stage timed
    n_stage = min(args.steps, 5)
    run(args.warmup + args.steps, 3)  # clocks back up after the verification's idle GPU
    ctx.set_timing(True)
    ctx.reset_stats()
    run(args.warmup + args.steps + 3, n_stage)
    ctx.set_timing(False)
    stage_stats = {k: ctx.stats(k) for k in ("batch", "resize", "sc_prep", "sc_score", "crop_apply")}
    if rank == 0:
        T = max(v["elapsed"] for v in allv)
        mpix = world * nimg * W * H * args.steps / 1e6
        rs_ms, rs_n, rs_bytes = stats["resize"]
        achieved = (rs_bytes / max(rs_n, 1)) / (rs_ms / max(rs_n, 1) / 1e3) / 1e9 if rs_ms > 0 else 0.0
        result = {
            "metric": METRIC,
            "value": round(mpix / T, 3),
            "unit": "Mpix/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(T / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic (seeded smooth field + noise + skin discs, generated in HBM)",
            "config": {
                "workload": f"{args.workload}: {cfg_text}",
                "images_per_gpu": nimg, "src": f"{W}x{H} RGB8", "options": options,
                "out": f"{ow}x{oh}x{oc} before smart-crop apply",
                "parallelism": f"dp{world} (images sharded per GPU, {gather.backend} gather of 32-B result records)"
                               if world > 1 else "dp1",
                "record_gather": gather.backend,
                "arithmetic": "resample exact-integer i8 MFMA on u8 (k_rs_vr: weights rint(w*2^s) in two signed-byte "
                              "limbs, s = 15-22 by the largest weight, each row's sum kept; k_rs_vm / k_rs_hv: "
                              "three limbs at 2^22), int32 sums, Q16 intermediate as ImageMagick, +-1 LSB of IM's "
                              "f64; smartcrop prescale int32 (Pillow fixed point), maps f32/f64, scores f64 "
                              "(bit-exact)",
            },
            "roofline": {
                "bound": "hbm",
                "kernel": "resize stage: " + " + ".join(
                    f"{KERNEL_OF_PATH[p]} ({n} images)" for p, n in paths.items() if n) ,
                "achieved": round(achieved, 2),
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4),
                "traffic": None,
                "algorithmic_bytes_per_launch": round(rs_bytes / max(rs_n, 1)),
                "avg_launch_ms": round(rs_ms / max(rs_n, 1), 4),
            },
            "stages_ms_per_step": dict(
                {k: round(v[0] / max(v[1], 1), 4) for k, v in stage_stats.items()},
                **{k: round(v[0] / max(v[1], 1), 4) for k, v in stats.items() if k.startswith("host_")}),
            "stage_timing": f"stage ranges from an instrumented pass of {n_stage} further batches (every stage "
                            "timed); the timed region times the resample stage only (roofline.avg_launch_ms), "
                            "host_* over the timed region",
            "smartcrop_kernels": " + ".join(f"{SC_KERNEL_OF_PATH[p]} ({n} images)" for p, n in sc_paths.items() if n),
            "exact_rescored_crops_per_step": allv[0]["ncand"],
            "failed_images": sum(v["bad"] for v in allv),
            "verified": (f"{sum(v['ok'] for v in allv_v)}/{sum(v['tot'] for v in allv_v)} images of the last "
                         "timed batch vs the oracle (pixels +-1 LSB, crop box bit-exact on the GPU pixels)")
                        if not args.no_verify else "skipped (--no-verify)",
        }
        if ablation:
            result["ablation"] = (f"FI_VR_VARIANT={os.environ.get('FI_VR_VARIANT')}: {ablation} profiling launches "
                                  "with wrong pixels -- not a valid measurement")
        # HBM traffic of the dominant kernel from the committed rocprofv3 PMC
        # passes (tools/gpu_profile.sh -> profiles/traffic_<workload>_<kernel>.json)
        kern = [p for p, n in paths.items() if n]
        if len(kern) == 1:
            kname = KERNEL_OF_PATH[kern[0]].split()[0]
            tf = os.path.join(REPO, "profiles", f"traffic_{args.workload}_{kname}.json")
            if os.path.exists(tf):
                t = json.load(open(tf))
                ipl = rs_n and (nimg * args.steps) // rs_n or nimg
                src = f"profiles/traffic_{args.workload}_{kname}.json"
                if t.get("source_sha256") == source_hash():
                    result["roofline"]["traffic"] = round(t["hbm_bytes_per_image"] * ipl)
                    result["roofline"]["traffic_source"] = (f"{src}: {t['correction']}, measured per image x {ipl} "
                                                            "images on these kernel sources")
                else:
                    result["roofline"]["traffic_stale"] = (f"{src} was measured on other kernel sources "
                                                           "(source_sha256 differs): not reported")
        if not args.no_cpu_baseline:
            try:
                result["cpu_baseline"] = cpu_baseline(W, H, options)
            except Exception as e:  # noqa: BLE001
                result["cpu_baseline"] = {"value": None, "error": repr(e)}
        print(json.dumps(result), flush=True)
    verify_failed = any(v["err"] for v in allv_v)
    ctx.free(pool)
    for d in dsts:
        ctx.free(d)
    comm.close()
    ctx.close()
    if verify_failed:
        sys.exit(1)


def cfg4_batch(shard_len):
    """Images per cfg4 batch for a shard of shard_len images."""
    return min(4096, max(1024, 1 << (max(shard_len // 16, 1).bit_length() - 1)))


def cfg4_batches(shard, B):
    """The shard in batches of B images, the first one a quarter of that: a
    step starts with the first batch's host plan and upload and nothing to
    overlap them with (4096 images: 6.8 ms in the trace), later batches are
    planned while earlier ones run."""
    q = max(B // 4, 1) if len(shard) > B else B
    return [shard[:q]] + [shard[j:j + B] for j in range(q, len(shard), B)]


def run_cfg4(args, rank, world, local_rank, comm):
    """cfg4: the 65536-image mixed list, LPT-sharded by input bytes across the
    ranks (strong scaling: the total is fixed), each rank running its shard as
    pipelined batches of cfg4_batch(shard) images.  One step = every rank's whole shard.  Sources:
    synthetic images in a device pool, k copies per size class so that no two
    descriptors of one batch share source bytes."""
    import numpy as np

    from flyimg_amd import _lib as L
    from flyimg_amd.parallel import RecordGather, shard_lpt
    from flyimg_amd.processor import ImageProcessor, OptionsBag
    from flyimg_amd.runtime import Context
    from flyimg_amd.runtime import plan as fi_plan
    from flyimg_amd.runtime import plan_bytes

    n_total = args.images or 65536
    items = cfg4_list(n_total)
    # greedy LPT by SURVEY 8(e) B_img (the bytes the resample reads + writes),
    # planned per (size, op) class
    op_of = {}
    for W, H, k in items:
        if (W, H, k) not in op_of:
            op_of[(W, H, k)] = ImageProcessor(OptionsBag(CFG4_OPS[k]), W, H).to_op()
    keys = list(op_of)
    b_of = dict(zip(keys, plan_bytes([(W, H, op_of[(W, H, k)]) for W, H, k in keys])))
    shard = shard_lpt([float(max(b_of[it], 1)) for it in items], world)[rank]
    ctx = Context(int(os.environ.get("FI_BENCH_DEVICE", local_rank)))  # override: rehearsal of N ranks on one GPU
    gather = RecordGather(comm, ctx)
    # batch size: the largest power of two that still leaves the rank >= 16
    # batches to pipeline, within [1024, 4096] -- fewer, larger batches cut the
    # persistent launches' tails (one GPU: 1024 -> 4096 is 365 -> 342 ms per
    # step, profiles/r06/cfg4_batch_ab.txt); 8 ranks keep 1024
    B = int(os.environ.get("FI_BENCH_CFG4_BATCH", 0)) or cfg4_batch(len(shard))
    batches = cfg4_batches(shard, B)
    # distinct source bytes inside a batch, so repeat reads cannot
    # hit L2 / MALL -- each size class gets as many synthetic copies as the most
    # images of that class any one batch holds, and the j-th image of a class
    # in a batch reads copy j
    need = {}
    copy_of = {}
    for b in batches:
        seen = {}
        for i in b:
            wh = items[i][:2]
            copy_of[i] = seen.get(wh, 0)
            seen[wh] = copy_of[i] + 1
        for wh, n in seen.items():
            need[wh] = max(need.get(wh, 0), n)
    sizes = sorted(need)
    stride_of = {wh: (wh[0] * 3 + 15) // 16 * 16 for wh in sizes}
    off_of, total = {}, 0
    for wh in sizes:
        off_of[wh] = total
        total += stride_of[wh] * wh[1] * need[wh]
    pool = ctx.malloc(total)
    t0 = time.perf_counter()
    for k, wh in enumerate(sizes):
        for j in range(need[wh]):
            ctx.fill_synthetic(pool + off_of[wh] + j * stride_of[wh] * wh[1], wh[0], wh[1], stride_of[wh],
                               0x5EED + 7919 * k + 104729 * j)
    log(f"rank {rank}: cfg4 shard {len(shard)} of {n_total} images, pool of {len(sizes)} size classes x "
        f"{min(need.values()) if need else 0}-{max(need.values()) if need else 0} copies "
        f"({total / 1e9:.2f} GB) in {time.perf_counter() - t0:.1f} s")
    ops = {}
    for i in shard:
        W, H, k = items[i]
        if (W, H, k) not in ops:
            op = ImageProcessor(OptionsBag(CFG4_OPS[k]), W, H).to_op()
            ops[(W, H, k)] = (op, fi_plan(W, H, op))
    cap = max(sum(int(np.prod(ops[items[i]][1])) for i in b) for b in batches) if batches else 1
    dst = [ctx.malloc(cap) for _ in range(PIPE_DEPTH)]

    def fill(arr, b, slot):
        o = 0
        for j, i in enumerate(b):
            W, H, k = items[i]
            op, (ow, oh, oc) = ops[(W, H, k)]
            a = arr[j]
            a.src = pool + off_of[(W, H)] + copy_of[i] * stride_of[(W, H)] * H
            a.src_w, a.src_h, a.src_stride, a.src_channels = W, H, stride_of[(W, H)], 3
            a.target_w, a.target_h, a.flags, a.gravity, a.rotate = op.target_w, op.target_h, op.flags, op.gravity, op.rotate
            a.smartcrop_w, a.smartcrop_h = op.smartcrop_w, op.smartcrop_h
            a.dst, a.dst_capacity = dst[slot] + o, ow * oh * oc
            o += ow * oh * oc

    # the descriptor arrays, one per batch, built once before timing (as the
    # other workloads' are): the library writes each batch's results into
    # its array, the records are read from them column-wise
    arrs = []
    for k, b in enumerate(batches):
        arrs.append((L.FiImage * len(b))())
        fill(arrs[-1], b, k % PIPE_DEPTH)
    views = [L.struct_view(a) for a in arrs]
    idx_of = [np.asarray(b, dtype=np.int32) for b in batches]
    rec_fields = ("status", "out_w", "out_h", "crop_x", "crop_y", "crop_w", "crop_h")
    bad = [0]

    def step():
        recs = []

        def on_done(k):
            v = views[k]
            bad[0] += int(np.count_nonzero(v["status"]))
            recs.append(np.stack([idx_of[k]] + [v[f] for f in rec_fields], axis=1))

        D = PIPE_DEPTH
        done = 0
        for k, b in enumerate(batches):
            L.check(ctx.submit_device(arrs[k], len(b)))
            if k - done >= D - 1:
                L.check(ctx.wait(D - 1))
                on_done(done)
                done += 1
        L.check(ctx.wait(0))
        for k in range(done, len(batches)):
            on_done(k)
        if world > 1:
            # uneven shards: pad to the longest so every rank sends the same count
            r = np.concatenate(recs) if recs else np.zeros((0, 8), np.int32)
            n_max = max(comm.allgather_obj(len(r)))
            pad = np.zeros((n_max - len(r), 8), np.int32)
            pad[:, 0] = -1
            gather.gather(np.concatenate([r, pad]))

    for _ in range(args.warmup):
        step()
    bad[0] = 0
    ctx.set_timing(True)
    ctx.reset_stats()
    comm.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    t1 = time.perf_counter()
    comm.barrier()
    ctx.set_timing(False)
    names = ("batch", "resize", "sc_prep", "sc_score", "crop_apply", "mono", "host_plan", "host_plan_images",
             "host_plan_sc", "host_plan_tiles", "host_plan_vmtiles", "host_plan_vr", "host_plan_hv", "host_plan_blob",
             "host_launch", "host_wait",
             "host_total")
    stats = {k: ctx.stats(k) for k in names}
    paths = {p: ctx.stats(p)[1] // max(args.steps, 1) for p in KERNEL_OF_PATH}
    ablation = ctx.stats("vr_ablation")[1]
    # correctness of the timed work itself (untimed): 16 images of this rank's
    # last batch, spread over it, against the oracle (each image its own size
    # class and op; smart-crop boxes bit-exact on the GPU pixels)
    vok, vtot, verr = 0, 0, None
    if batches and not args.no_verify:
        from oracle.verify import verify_mixed_batch  # the checker (test infrastructure)

        lb, la = batches[-1], arrs[-1]
        slot = (len(batches) - 1) % PIPE_DEPTH
        views, vops, seeds, offs, o = [], [], [], [], 0
        for i in lb:
            W, H, k = items[i]
            op, (ow, oh, oc) = ops[(W, H, k)]
            wh = (W, H)
            views.append((pool + off_of[wh] + copy_of[i] * stride_of[wh] * H, W, H, stride_of[wh]))
            vops.append(op)
            seeds.append(0x5EED + 7919 * sizes.index(wh) + 104729 * copy_of[i])
            offs.append(o)
            o += ow * oh * oc
        idxs = sorted({int(v) for v in np.linspace(0, len(lb) - 1, 16)})
        vok, vtot, verr = verify_mixed_batch(ctx, la, views, vops, idxs, seeds, lambda j: dst[slot] + offs[j])
        if verr:
            log(f"rank {rank}: VERIFY FAILED {vok}/{vtot}: {verr}")
    allv = comm.allgather_obj({"elapsed": t1 - t0, "stats": stats, "bad": bad[0], "n": len(shard),
                               "vok": vok, "vtot": vtot, "verr": verr})
    if rank == 0:
        T = max(v["elapsed"] for v in allv)
        mpix = sum(W * H for W, H, _ in items) * args.steps / 1e6
        rs_ms, rs_n, rs_bytes = stats["resize"]
        achieved = (rs_bytes / max(rs_n, 1)) / (rs_ms / max(rs_n, 1) / 1e3) / 1e9 if rs_ms > 0 else 0.0
        gpu_ms = stats["batch"][0] / max(args.steps, 1)
        result = {
            "metric": METRIC,
            "value": round(mpix / T, 3),
            "unit": "Mpix/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(T / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic (seeded images in HBM; no two images of a batch share a source)",
            "config": {
                "workload": f"cfg4: {WORKLOADS['cfg4'][4]}",
                "images_total": n_total, "size_classes": len(sizes),
                "mean_mpix_per_image": round(mpix / args.steps / n_total, 3),
                "ops": CFG4_OPS, "batch": B, "first_batch": len(batches[0]) if batches else 0,
                "parallelism": f"dp{world} (LPT shards by B_img, RCCL gather of result records)",
                "record_gather": gather.backend,
            },
            "roofline": {
                "bound": "hbm",
                "kernel": "resize stage: " + " + ".join(
                    f"{KERNEL_OF_PATH[p]} ({n} images)" for p, n in paths.items() if n),
                "achieved": round(achieved, 2),
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4),
                "traffic": None,
                "avg_launch_ms": round(rs_ms / max(rs_n, 1), 4),
            },
            "rank0_gpu_busy_ms_per_step": round(gpu_ms, 3),
            "rank0_host_plan_ms_per_step": round(stats["host_plan"][0] / max(args.steps, 1), 3),
            "stages_ms_per_step": {k: round(v[0] / max(args.steps, 1), 4) for k, v in stats.items()},
            "shard_images": [v["n"] for v in allv],
            "failed_images": sum(v["bad"] for v in allv),
            "verified": (f"{sum(v['vok'] for v in allv)}/{sum(v['vtot'] for v in allv)} images of each rank's last "
                         "batch vs the oracle (pixels +-1 LSB, crop box bit-exact on the GPU pixels)")
                        if not args.no_verify else "skipped (--no-verify)",
        }
        if ablation:
            result["ablation"] = (f"FI_VR_VARIANT={os.environ.get('FI_VR_VARIANT')}: {ablation} profiling launches "
                                  "with wrong pixels -- not a valid measurement")
        tf = os.path.join(REPO, "profiles", "traffic_cfg4_resize.json")
        if os.path.exists(tf):
            t = json.load(open(tf))
            if t.get("source_sha256") == source_hash():
                ipl = len(shard) * args.steps / max(rs_n, 1)  # images per resize launch
                result["roofline"]["traffic"] = round(t["hbm_bytes_per_image"] * ipl)
                result["roofline"]["traffic_source"] = (f"profiles/traffic_cfg4_resize.json: {t['correction']}, "
                                                        "the resize launches of the sampled batches, per image")
            else:
                result["roofline"]["traffic_stale"] = "profiles/traffic_cfg4_resize.json measured on other sources"
        if not args.no_cpu_baseline:
            result["cpu_baseline"] = cfg4_cpu_baseline(items)
        print(json.dumps(result), flush=True)
    verify_failed = any(v["verr"] for v in allv)
    ctx.free(pool)
    for d in dst:
        ctx.free(d)
    comm.close()
    ctx.close()
    if verify_failed:
        sys.exit(1)


if __name__ == "__main__":
    main()
