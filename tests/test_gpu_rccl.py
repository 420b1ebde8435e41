"""RCCL record gather on the GPU (MI355X) -- the multi-GPU result gather of
SURVEY.md 8(e) (fi_rccl_*) executed through the C-ABI on one
GPU: a 1-rank communicator (fi_rccl_get_unique_id + fi_rccl_init(rank 0,
world 1)) gathers 1024 records to rank 0 unchanged; and RecordGather raises
-- no control-plane fallback -- when the real fi_rccl_init fails."""
import ctypes

import pytest

from flyimg_amd import _lib as L
from flyimg_amd.parallel import RecordGather
from flyimg_amd.runtime import Context

pytestmark = pytest.mark.gpu


def _records(n):
    return [(i, i % 3 - 1, 500 + i, 281 - i % 7, i * 3, i * 5, 100 + i % 11, 90 + i % 13) for i in range(n)]


def test_rccl_one_rank_gather_identity():
    ctx = Context(0)
    try:
        lib = L.lib()
        uid = ctypes.create_string_buffer(128)
        L.check(lib.fi_rccl_get_unique_id(uid))
        L.check(lib.fi_rccl_init(ctx.h, 0, 1, uid.raw))
        recs = _records(1024)
        send = (L.FiRecord * 1024)(*[L.FiRecord(*r) for r in recs])
        recv = (L.FiRecord * 1024)()
        L.check(lib.fi_rccl_gather_records(ctx.h, send, 1024, recv))
        got = [tuple(getattr(recv[i], f) for f, _ in L.FiRecord._fields_) for i in range(1024)]
        assert got == recs
        # a second gather on the same communicator (the bench gathers every step)
        recs2 = [tuple(-v for v in r) for r in recs[:17]]
        send2 = (L.FiRecord * 17)(*[L.FiRecord(*r) for r in recs2])
        recv2 = (L.FiRecord * 17)()
        L.check(lib.fi_rccl_gather_records(ctx.h, send2, 17, recv2))
        assert [tuple(getattr(recv2[i], f) for f, _ in L.FiRecord._fields_) for i in range(17)] == recs2
    finally:
        ctx.close()


def test_rccl_gather_before_init_is_an_error():
    ctx = Context(0)
    try:
        send = (L.FiRecord * 1)()
        with pytest.raises(L.FiError):
            L.check(L.lib().fi_rccl_gather_records(ctx.h, send, 1, None))
    finally:
        ctx.close()


class _OneProcessComm:
    """A control-plane comm that claims rank 2 of world 2 (an out-of-range rank:
    the real fi_rccl_init refuses it at once, no peer is waited for)."""

    rank, world = 2, 2

    def bcast_bytes(self, data):
        return bytes(128)

    def allgather_obj(self, obj):
        return [obj]


def test_record_gather_raises_when_rccl_init_fails():
    ctx = Context(0)
    try:
        with pytest.raises(RuntimeError, match="RCCL record gather did not come up"):
            RecordGather(_OneProcessComm(), ctx)
    finally:
        ctx.close()
