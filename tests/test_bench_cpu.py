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
