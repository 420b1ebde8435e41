"""Multi-GPU plumbing: one process per GPU, images sharded across ranks.

flyimg's path has no cross-image reduction: each rank runs
its own shard end to end on its own GPU; the only exchange is the final gather
of 32-byte per-image result records to rank 0, done with RCCL over xGMI by
libflyimg_hip (``fi_rccl_gather_records``).

Control plane (barriers, the RCCL unique id, max-over-ranks timing) needs no
GPU and must not load a second HIP runtime into the process, so it does not go
through torch: ``FileComm`` is a single-node rendezvous in a directory shared by
the ranks a ``torch.distributed.run`` agent starts (they share its PID as
parent).  Any object with the same five methods works (tests drive the shard
and gather logic through a torch.distributed gloo wrapper on CPU).
"""
from __future__ import annotations

import json
import os
import shutil
import time


def env_rank_world():
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")),
            int(os.environ.get("LOCAL_RANK", os.environ.get("RANK", "0"))))


class SoloComm:
    rank, world = 0, 1

    def barrier(self):
        pass

    def bcast_bytes(self, data: bytes | None) -> bytes:
        return data

    def allgather_obj(self, obj):
        return [obj]

    def close(self):
        pass


class FileComm:
    """Rendezvous through files under a run directory (single node)."""

    def __init__(self, rank: int, world: int, run_id: str | None = None, root: str = "/tmp", timeout: float = 600.0):
        self.rank, self.world, self.timeout = rank, world, timeout
        run_id = run_id or f"{os.getppid()}_{os.environ.get('MASTER_PORT', '0')}"
        self.dir = os.path.join(root, f"flyimg_rdzv_{run_id}")
        os.makedirs(self.dir, exist_ok=True)
        self.gen = 0

    def _path(self, tag, r):
        return os.path.join(self.dir, f"{tag}.{r}")

    def _put(self, tag, r, payload: bytes):
        tmp = self._path(tag, r) + ".tmp"
        with open(tmp, "wb") as f:
            f.write(payload)
        os.replace(tmp, self._path(tag, r))

    def _get(self, tag, r) -> bytes:
        p = self._path(tag, r)
        t0 = time.time()
        while not os.path.exists(p):
            if time.time() - t0 > self.timeout:
                raise TimeoutError(f"rank {self.rank}: waiting for {p}")
            time.sleep(0.002)
        with open(p, "rb") as f:
            return f.read()

    def allgather_obj(self, obj):
        self.gen += 1
        tag = f"ag{self.gen}"
        self._put(tag, self.rank, json.dumps(obj).encode())
        return [json.loads(self._get(tag, r)) for r in range(self.world)]

    def barrier(self):
        self.allgather_obj(0)

    def bcast_bytes(self, data: bytes | None) -> bytes:
        self.gen += 1
        tag = f"bc{self.gen}"
        if self.rank == 0:
            self._put(tag, 0, data)
        return self._get(tag, 0)

    def close(self):
        # the other ranks may still be reading rank 0's barrier file: each
        # acknowledges after its barrier, and rank 0 removes the directory
        # only once every acknowledgement is in
        self.barrier()
        if self.rank != 0:
            self._put("bye", self.rank, b"1")
            return
        for r in range(1, self.world):
            self._get("bye", r)
        shutil.rmtree(self.dir, ignore_errors=True)


def make_comm():
    """The control-plane comm of this rank.  ``FI_RDZV_ID`` (set by bench.py's
    own launcher) names the rendezvous; under ``torch.distributed.run`` the
    ranks share the agent's PID as parent and the master port."""
    rank, world, _ = env_rank_world()
    return SoloComm() if world == 1 else FileComm(rank, world, run_id=os.environ.get("FI_RDZV_ID") or None)


def shard_lpt(costs: list[float], world: int) -> list[list[int]]:
    """Greedy LPT: images (by cost, e.g. algorithmic bytes) to ranks."""
    order = sorted(range(len(costs)), key=lambda i: (-costs[i], i))
    load = [0.0] * world
    out = [[] for _ in range(world)]
    for i in order:
        r = min(range(world), key=lambda k: (load[k], k))
        out[r].append(i)
        load[r] += costs[i]
    for s in out:
        s.sort()
    return out


def shard_contiguous(n: int, world: int) -> list[range]:
    """Uniform batches: contiguous ranges."""
    base, extra = divmod(n, world)
    out, start = [], 0
    for r in range(world):
        k = base + (1 if r < extra else 0)
        out.append(range(start, start + k))
        start += k
    return out


class RecordGather:
    """Gather per-image result records to rank 0: RCCL through the C-ABI when a
    context is given, else through the control-plane comm (CPU tests)."""

    def __init__(self, comm, ctx=None):
        self.comm, self.ctx, self.backend = comm, ctx, "none"
        if comm.world == 1:
            self.backend = "local"
            return
        if ctx is not None and os.environ.get("FI_RECORD_GATHER", "rccl") == "rccl":
            import ctypes

            from . import _lib as L

            uid = ctypes.create_string_buffer(128)
            ok = 1
            if comm.rank == 0:
                ok = int(L.lib().fi_rccl_get_unique_id(uid) == 0)
            data = comm.bcast_bytes((uid.raw if ok else b"") if comm.rank == 0 else None)
            if len(data) == 128:
                ok = int(L.lib().fi_rccl_init(ctx.h, comm.rank, comm.world, data) == 0)
            else:
                ok = 0
            # every rank takes the same decision: a world > 1 run whose RCCL does not
            # come up everywhere fails (FI_RECORD_GATHER=comm selects the
            # control-plane gather explicitly) -- no silent fallback
            oks = comm.allgather_obj(ok)
            if not all(oks):
                raise RuntimeError(f"RCCL record gather did not come up on ranks "
                                   f"{[r for r, o in enumerate(oks) if not o]} (set FI_RECORD_GATHER=comm "
                                   f"to gather through the control plane)")
            self.backend = "rccl"
        else:
            self.backend = "comm"

    def gather(self, records):
        """records: list of 8-int tuples (fi_record), or an (n, 8) int32 array.
        Rank 0 gets all ranks' (as an (n * world, 8) array for an array input)."""
        self.start(records)
        return self.finish()

    # Non-blocking form (bench.py's batch loop): start() enqueues the gather
    # on the library's gather stream and returns; finish() waits for it and
    # returns rank 0's records.  One gather in flight: a start() with one
    # pending finishes it first (whose records are then dropped).
    _pending = None

    def start(self, records):
        if self._pending is not None:
            self.finish()
        import numpy as np

        as_array = isinstance(records, np.ndarray)
        if self.backend == "local":
            self._pending = ("local", records.copy() if as_array else list(records))
            return
        if self.backend == "rccl":
            import ctypes

            from . import _lib as L

            n = len(records)
            send = (L.FiRecord * max(n, 1))()
            if as_array:
                rec = np.ascontiguousarray(records, dtype=np.int32).reshape(n, 8)
                ctypes.memmove(send, rec.ctypes.data, rec.nbytes)
            else:
                for i, r in enumerate(records):
                    send[i] = L.FiRecord(*r)
            recv = (L.FiRecord * max(n * self.comm.world, 1))() if self.comm.rank == 0 else None
            L.check(L.lib().fi_rccl_gather_start(self.ctx.h, send, n, recv))
            self._pending = ("rccl", (n, recv, as_array))
            return
        self._pending = ("comm", (records.tolist() if as_array else [list(r) for r in records], as_array))

    def finish(self):
        if self._pending is None:
            return None
        kind, data = self._pending
        self._pending = None
        if kind == "local":
            return data
        if kind == "rccl":
            from . import _lib as L

            L.check(L.lib().fi_rccl_gather_finish(self.ctx.h))
            n, recv, as_array = data
            if self.comm.rank != 0:
                return None
            if as_array:
                import numpy as np

                return np.frombuffer(recv, dtype=np.int32, count=n * self.comm.world * 8).reshape(-1, 8).copy()
            return [tuple(getattr(recv[i], f) for f, _ in L.FiRecord._fields_) for i in range(n * self.comm.world)]
        # the control-plane gather is a rendezvous: it runs at finish()
        rows, as_array = data
        allr = self.comm.allgather_obj(rows)
        if self.comm.rank != 0:
            return None
        if as_array:
            import numpy as np

            return np.asarray([r for part in allr for r in part], dtype=np.int32).reshape(-1, 8)
        return [tuple(r) for part in allr for r in part]
