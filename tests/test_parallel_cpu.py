"""Multi-rank plumbing on CPU (world_size 2): the file rendezvous the bench
uses, the same shard/gather logic through a torch.distributed gloo wrapper,
and the LPT sharding."""
import multiprocessing as mp
import os
import random
import socket
import tempfile
import time

import pytest

from flyimg_amd.parallel import FileComm, RecordGather, shard_contiguous, shard_lpt

N_IMAGES = 10


def _records(rank, idx):
    # fi_record: image, status, out_w, out_h, crop_x, crop_y, crop_w, crop_h
    return [(i, 0, 500, 281, rank, i % 7, 100 + i, 99) for i in idx]


def _file_rank(rank, world, run_id, root, q):
    try:
        comm = FileComm(rank, world, run_id=run_id, root=root, timeout=60)
        g = comm.allgather_obj({"rank": rank, "t": 0.5 + rank})
        uid = comm.bcast_bytes(b"unique-id-bytes" if rank == 0 else None)
        comm.barrier()
        shard = list(shard_contiguous(N_IMAGES, world)[rank])
        got = RecordGather(comm).gather(_records(rank, shard))
        comm.close()
        q.put((rank, g, uid, got, None))
    except Exception as e:  # noqa: BLE001
        q.put((rank, None, None, None, repr(e)))


def _run(target, world, *args):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=target, args=(r, world) + args + (q,)) for r in range(world)]
    for p in ps:
        p.start()
    out = {}
    for _ in ps:
        r = q.get(timeout=120)
        out[r[0]] = r
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    return out


def _check(out, world):
    for r in range(world):
        assert out[r][4] is None, out[r][4]
        g = out[r][1]
        assert [x["rank"] for x in g] == list(range(world))
        assert max(x["t"] for x in g) == 0.5 + world - 1  # max-over-ranks timing input
        assert out[r][2] == b"unique-id-bytes"
    got = out[0][3]
    assert [rec[0] for rec in got] == list(range(N_IMAGES))  # every image once, in rank order
    assert all(rec[4] == r for r, part in enumerate(shard_contiguous(N_IMAGES, world)) for rec in got
               if rec[0] in part)
    for r in range(1, world):
        assert out[r][3] is None


def test_file_comm_world2():
    with tempfile.TemporaryDirectory() as root:
        out = _run(_file_rank, 2, f"t{os.getpid()}", root)
        _check(out, 2)
        assert not os.listdir(root)  # rank 0 removed the rendezvous directory


class GlooComm:
    """The five-method comm interface over torch.distributed (gloo, CPU)."""

    def __init__(self):
        import torch.distributed as dist

        self.dist = dist
        self.rank, self.world = dist.get_rank(), dist.get_world_size()

    def barrier(self):
        self.dist.barrier()

    def bcast_bytes(self, data):
        obj = [data]
        self.dist.broadcast_object_list(obj, src=0)
        return obj[0]

    def allgather_obj(self, obj):
        out = [None] * self.world
        self.dist.all_gather_object(out, obj)
        return out

    def close(self):
        self.dist.barrier()


def _gloo_rank(rank, world, port, as_array, q):
    try:
        import torch.distributed as dist

        dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
        comm = GlooComm()
        g = comm.allgather_obj({"rank": rank, "t": 0.5 + rank})
        uid = comm.bcast_bytes(b"unique-id-bytes" if rank == 0 else None)
        comm.barrier()
        shard = list(shard_contiguous(N_IMAGES, world)[rank])
        if as_array:  # bench.py's cfg4 form: an (n, 8) int32 block in, an array out on rank 0
            import numpy as np

            got = RecordGather(comm).gather(np.asarray(_records(rank, shard), dtype=np.int32))
            if got is not None:
                assert isinstance(got, np.ndarray) and got.dtype == np.int32 and got.shape[1] == 8
                got = [tuple(int(x) for x in r) for r in got]
        else:
            got = RecordGather(comm).gather(_records(rank, shard))
        comm.close()
        dist.destroy_process_group()
        q.put((rank, g, uid, got, None))
    except Exception as e:  # noqa: BLE001
        q.put((rank, None, None, None, repr(e)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("as_array", [False, True], ids=["tuples", "array"])
def test_gloo_world2_same_shard_and_gather_logic(as_array):
    pytest.importorskip("torch")
    out = _run(_gloo_rank, 2, _free_port(), as_array)
    _check(out, 2)


def test_shard_lpt_covers_and_balances():
    rnd = random.Random(20250112)
    for world in (1, 2, 3, 8):
        costs = [rnd.uniform(0.5, 24.0) for _ in range(257)]
        parts = shard_lpt(costs, world)
        flat = sorted(i for p in parts for i in p)
        assert flat == list(range(len(costs)))
        loads = [sum(costs[i] for i in p) for p in parts]
        # LPT bound: max load <= mean + max item
        assert max(loads) <= sum(costs) / world + max(costs) + 1e-9
        assert all(p == sorted(p) for p in parts)


def test_shard_contiguous_uniform():
    for n, world in ((1024, 8), (10, 3), (3, 8)):
        parts = shard_contiguous(n, world)
        assert [i for p in parts for i in p] == list(range(n))
        assert max(len(p) for p in parts) - min(len(p) for p in parts) <= 1


def test_file_comm_timeout_is_loud():
    with tempfile.TemporaryDirectory() as root:
        c = FileComm(0, 2, run_id="lonely", root=root, timeout=0.2)
        t0 = time.time()
        with pytest.raises(TimeoutError):
            c.allgather_obj(1)
        assert time.time() - t0 < 5


def _close_rank(rank, world, root, q):
    try:
        for it in range(25):
            comm = FileComm(rank, world, run_id=f"close{it}", root=root, timeout=10)
            comm.barrier()
            comm.close()  # rank 0 must not remove the directory under a reader
        q.put((rank, None, None, None, None))
    except Exception as e:  # noqa: BLE001
        q.put((rank, None, None, None, repr(e)))


def test_file_comm_close_waits_for_every_rank(tmp_path):
    """Regression: rank 0 used to delete the rendezvous directory right after
    its closing barrier, while another rank could still be polling for rank
    0's barrier file -- that rank then hung until its timeout."""
    out = _run(_close_rank, 4, str(tmp_path))
    for r in range(4):
        assert out[r][4] is None, out[r][4]


class _StubLib:
    """fi_rccl_* stand-ins: RCCL comes up on every rank except ``bad``."""

    def __init__(self, rank, bad):
        self.rank, self.bad = rank, bad

    def fi_rccl_get_unique_id(self, buf):
        buf.raw = bytes(range(128))
        return 0

    def fi_rccl_init(self, h, rank, world, data):
        return -5 if rank == self.bad else 0


def _rccl_rank(rank, world, run_id, root, bad, q):
    try:
        from flyimg_amd import _lib as L

        L.lib = lambda: _StubLib(rank, bad)  # this spawned process only

        class Ctx:
            h = None

        comm = FileComm(rank, world, run_id=run_id, root=root, timeout=60)
        try:
            g = RecordGather(comm, Ctx())
            res = g.backend
        except RuntimeError as e:
            res = "error: " + str(e)
        comm.close()
        q.put((rank, res, None, None, None))
    except Exception as e:  # noqa: BLE001
        q.put((rank, None, None, None, repr(e)))


@pytest.mark.parametrize("bad", [-1, 1])
def test_record_gather_fails_loudly_when_rccl_is_down(bad):
    """world > 1 with a context: RCCL on every rank, or every rank raises --
    never a silent fallback to the control-plane gather."""
    with tempfile.TemporaryDirectory() as root:
        out = _run(_rccl_rank, 2, f"r{os.getpid()}{bad}", root, bad)
    for r in range(2):
        assert out[r][4] is None, out[r][4]
        if bad < 0:
            assert out[r][1] == "rccl"
        else:
            assert out[r][1].startswith("error: RCCL record gather did not come up on ranks [1]")
