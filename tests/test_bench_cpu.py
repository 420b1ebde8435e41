"""bench.py host legs on the CPU: the cfg4 list, the B_img sharding input
(fi_plan_bytes) and the bounded CPU baselines."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
from flyimg_amd import _lib as L  # noqa: E402
from flyimg_amd.parallel import shard_lpt  # noqa: E402
from flyimg_amd.processor import ImageProcessor, OptionsBag  # noqa: E402
from flyimg_amd.runtime import plan, plan_bytes  # noqa: E402


def test_plan_bytes_matches_survey_b_img():
    """B_img = R_touched * W_in * C_in + W_out * H_out * C_out (+16 with smc):
    the cfg2 and cfg3 figures of SURVEY.md 8(d)."""
    cfg2 = ImageProcessor(OptionsBag("w_500,smc_1"), 1920, 1080).to_op()
    cfg3 = ImageProcessor(OptionsBag("w_512,h_512,c_1"), 3840, 2160).to_op()
    b2, b3 = plan_bytes([(1920, 1080, cfg2), (3840, 2160, cfg3)])
    # cfg2: the 5x thumbnail sample step touches all 1080 rows; 500x281x3 out; crop record
    assert b2 == 1080 * 1920 * 3 + 500 * 281 * 3 + 16
    assert b3 == 25669632  # 25.67 MB
    # a copy (no resample) reads the extent window only
    same = ImageProcessor(OptionsBag("w_64,h_48"), 64, 48).to_op()
    ow, oh, oc = plan(64, 48, same)
    assert plan_bytes([(64, 48, same)]) == [48 * 64 * 3 + ow * oh * oc]


def test_plan_bytes_flags_unplannable_images():
    bad = ImageProcessor(OptionsBag("w_500"), 1920, 1080).to_op()
    bad.flags |= L.FI_OP_ROTATE
    bad.rotate = 45  # non-integral rotation: FI_EUNSUPPORTED
    assert plan_bytes([(1920, 1080, bad)]) == [-1]


def test_cfg4_shards_balance_b_img():
    items = bench.cfg4_list(512)
    ops = {}
    for W, H, k in items:
        ops.setdefault((W, H, k), ImageProcessor(OptionsBag(bench.CFG4_OPS[k]), W, H).to_op())
    keys = list(ops)
    b = dict(zip(keys, plan_bytes([(W, H, ops[(W, H, k)]) for W, H, k in keys])))
    cost = [float(b[it]) for it in items]
    assert min(cost) > 0
    for world in (2, 4, 8):
        shards = shard_lpt(cost, world)
        assert sorted(i for s in shards for i in s) == list(range(len(items)))
        loads = [sum(cost[i] for i in s) for s in shards]
        assert max(loads) <= 1.05 * (sum(loads) / world) + max(cost)


def test_cfg4_cpu_baseline_leg_on_a_tiny_list():
    """The cfg4 baseline leg runs (it used to raise TypeError and report null),
    reports the threads it used and the measured wall time."""
    items = [(96, 64, 0), (80, 120, 1), (128, 96, 3)]
    r = bench.cfg4_cpu_baseline(items, n_sample=3, threads=2)
    assert r["value"] and r["value"] > 0
    assert r["cores"] == 2 and r["kind"] == "port"
    assert r["images"] == 6 and r["wall_s"] > 0


def test_cpu_baseline_max_images_bounds_the_sample():
    r = bench.cpu_baseline(64, 48, "w_32,h_24,c_1", budget_s=30.0, threads=3, max_images=5)
    assert r["images"] == 5 and r["cores"] == 3 and r["wall_s"] < 30.0


class _FakeCtx:
    """fi_submit_batch_device / fi_wait stand-ins: a batch 'runs' for `gpu_s`
    after its submit; wait(keep) sleeps until at most `keep` remain."""

    def __init__(self, gpu_s, log):
        import time

        self.gpu_s, self.log, self.q, self.t = gpu_s, log, [], time

    def submit_device(self, arr, n):
        start = max([self.t.perf_counter()] + [e for _, e in self.q])
        self.q.append((arr, start + self.gpu_s))
        self.log.append(("submit", id(arr)))
        return 0

    def wait(self, keep):
        while len(self.q) > keep:
            arr, end = self.q.pop(0)
            self.t.sleep(max(0.0, end - self.t.perf_counter()))
            for i in range(len(arr)):
                arr[i].status, arr[i].crop_x = 0, i
            self.log.append(("done", id(arr)))
        return 0


def test_batch_loop_pipelines_and_gathers_once_without_blocking(tmp_path):
    """VERDICT r5 item 2 (CPU dry run of the non-blocking loop): each rank
    submits batch k before finalizing batch k-1, calls no collective inside
    the loop, and the records of every batch reach rank 0 in one gather at the
    end -- a rank whose batches are slow does not hold the other rank's
    batches back (the old per-batch gather made both ranks run at the slower
    one's pace, batch by batch)."""
    import threading
    import time

    from flyimg_amd.parallel import FileComm, RecordGather

    nimg, steps = 4, 6
    out, t_loop = {}, {}

    def rank_main(rank, gpu_s):
        comm = FileComm(rank, 2, run_id=f"loop_{os.getpid()}", root=str(tmp_path))
        log = []
        ctx = _FakeCtx(gpu_s, log)
        arrs = [(L.FiImage * nimg)() for _ in range(bench.PIPE_DEPTH)]
        recs = []

        def on_done(k, arr):
            log.append(("records", k))
            recs.extend((rank * 100 + k * nimg + i, arr[i].status, 0, 0, arr[i].crop_x, 0, 0, 0) for i in range(nimg))

        t0 = time.perf_counter()
        bench.run_batches(ctx, arrs, nimg, 0, steps, on_done)
        t_loop[rank] = time.perf_counter() - t0
        out[rank] = (log, RecordGather(comm).gather(recs))
        comm.close()

    ts = [threading.Thread(target=rank_main, args=(r, 0.002 if r == 0 else 0.05)) for r in (0, 1)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    log0, got0 = out[0]
    # pipelining: submit k precedes batch k-1's completion and its records
    kinds = [e[0] for e in log0]
    assert kinds[:bench.PIPE_DEPTH] == ["submit"] * bench.PIPE_DEPTH and kinds.count("submit") == steps
    for k in range(1, steps):
        assert log0.index(("records", k - 1)) > [i for i, e in enumerate(log0) if e[0] == "submit"][k]
    # rank 0's batches are not paced by rank 1's (6 x 50 ms): no per-batch rendezvous
    assert t_loop[0] < 0.5 * t_loop[1], t_loop
    # one final gather: rank 0 holds both ranks' records in rank order, rank 1 none
    assert out[1][1] is None
    assert len(got0) == 2 * steps * nimg
    assert [r[0] for r in got0] == [r * 100 + j for r in (0, 1) for j in range(steps * nimg)]


def _bench(args, **env):
    import subprocess

    e = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "FI_RDZV_ID")}
    e.update(env)
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, env=e, capture_output=True,
                          text=True, timeout=120)


def test_bench_launches_its_own_ranks_dry_run():
    """`bench.py --gpus N` without a launcher starts N rank
    processes; both join the rendezvous and rank 0's one JSON line comes back."""
    import json

    r = _bench(["--gpus", "2", "--dry-run"])
    assert r.returncode == 0, r.stderr
    lines = [ln for ln in r.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["ranks"] == [0, 1] and d["local_ranks"] == [0, 1] and d["distinct_pids"] == 2


def test_bench_refuses_world_size_mismatch():
    r = _bench(["--gpus", "8", "--dry-run"], WORLD_SIZE="1", RANK="0")
    assert r.returncode != 0 and r.stdout == ""
    assert "WORLD_SIZE=1 but --gpus 8" in r.stderr


def test_bench_launcher_fails_when_a_rank_fails():
    """a failing rank ends the run non-zero (the others are stopped, not left
    waiting in the rendezvous), and no JSON line is printed"""
    r = _bench(["--gpus", "2", "--dry-run"], FI_DRY_RUN_FAIL_RANK="1")
    assert r.returncode != 0 and r.stdout == ""


def test_cfg4_batch_size_leaves_every_rank_a_pipeline():
    """One GPU runs 4096-image batches (fewer persistent-launch tails), two
    ranks 2048, four and eight ranks 1024: every rank keeps >= 8 batches so
    batch k+1's host planning overlaps batch k."""
    assert [bench.cfg4_batch(65536 // n) for n in (1, 2, 4, 8)] == [4096, 2048, 1024, 1024]
    for n in (1, 2, 4, 8):
        shard = 65536 // n
        assert shard // bench.cfg4_batch(shard) >= 8
    assert bench.cfg4_batch(10) == 1024


def test_cfg4_batches_cover_the_shard_with_a_short_first_batch():
    for n, B in ((65536, 4096), (8192, 1024), (1000, 1024), (5000, 1024)):
        shard = list(range(n))
        bs = bench.cfg4_batches(shard, B)
        assert [i for b in bs for i in b] == shard
        assert all(len(b) <= B for b in bs)
        if n > B:
            assert len(bs[0]) == B // 4
