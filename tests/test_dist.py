"""The N>1 path on CPU: contiguous record shards packed independently and
gathered to rank 0 (srpc_amd.shard) reproduce the single-batch wire bytes.
world_size 2, 3 and 8 over gloo; each rank's shard is packed by the CPU oracle
standing in for its GPU (the kernel itself is covered by the gpu tests).

Two gathers: torch.distributed's (``gather_packed`` without a comm) and the
library's argument / offset logic (``gather_packed(..., comm=...)`` ->
``NativeComm.gather_wire`` -> srpc_gather_wire's contract) driven through a
fake communicator that moves the bytes over gloo exactly as the C ABI's RCCL
group does: shard r lands at the prefix sum of the shard sizes on the root
(include/srpc_gpu.h srpc_gather_wire; multi.hip).  Uneven shards (n not a
multiple of 16 x world, empty shards at n < 16 x world) at 2/3/8 ranks."""
import ctypes
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import oracle
from srpc_amd import _lib
from srpc_amd.shard import NativeComm, gather_packed, gather_plan, run_gather_plan, shard_range


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


class FakeComm(NativeComm):
    """NativeComm whose transport is gloo instead of RCCL: the operations are
    the library's own (srpc_gather_plan -- the argument checks and the
    (kind, peer, offset, bytes) list that srpc_gather_wire enqueues on RCCL,
    multi.hip), replayed by srpc_amd.shard.run_gather_plan as blocking gloo
    send / recv.  Nothing about placement is restated in Python."""

    def __init__(self, rank, nranks):  # no RCCL communicator behind it
        self.rank, self.nranks, self.device = rank, nranks, -1
        self._h = None
        self.calls = []
        self.ops = []

    def _gather(self, local, shard_bytes, out, root_cap, sizes, root, stream):
        self.calls.append((shard_bytes, root_cap, tuple(sizes), root))
        ops = gather_plan(self.rank, self.nranks, root, shard_bytes, sizes, root_cap)
        self.ops.append(ops)
        run_gather_plan(ops, local, out, p2p=False)

    def close(self):
        pass


def _worker(rank, world, port, n, use_comm, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        lo, hi = shard_range(n, rank, world)
        cols = oracle.splitmix_columns_i32(4, hi - lo, first_record=lo)
        local = np.frombuffer(oracle.pack([oracle.INT32] * 4, cols, hi - lo), np.uint8).copy()
        comm = FakeComm(rank, world) if use_comm else None
        out = gather_packed(torch.from_numpy(local), 16, n, comm=comm)
        if rank == 0:
            q.put((out.numpy().tobytes(), comm.calls if comm else None, comm.ops if comm else None))
        else:
            assert out is None
            if comm and world > 1:  # every rank passed its own shard's bytes: one SEND to the root, or none
                assert [c[0] for c in comm.calls] == [(hi - lo) * 16]
                assert comm.ops == [[(_lib.SRPC_GATHER_SEND, 0, 0, (hi - lo) * 16)] if hi > lo else []]
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,n,use_comm", [(2, 4096, False), (2, 1000, False), (3, 4099, False), (2, 0, False),
                                              (3, 17, False), (2, 1000, True), (3, 4099, True), (8, 1001, True),
                                              (8, 17, True), (8, 0, True)])
def test_sharded_pack_gather_equals_single_batch(world, n, use_comm):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    # daemon ranks, killed if still alive: a rank stuck in the rendezvous
    # must not keep the test process from exiting
    procs = [ctx.Process(target=_worker, args=(r, world, port, n, use_comm, q), daemon=True) for r in range(world)]
    for p in procs:
        p.start()
    try:
        got, calls, ops = q.get(timeout=180)
        for p in procs:
            p.join(timeout=180)
            assert p.exitcode == 0
    finally:
        for p in procs:
            if p.is_alive():
                p.kill()
                p.join(timeout=10)
    want = oracle.pack([oracle.INT32] * 4, oracle.splitmix_columns_i32(4, n), n)
    assert got == want
    if use_comm:
        sizes = tuple((hi - lo) * 16 for lo, hi in (shard_range(n, r, world) for r in range(world)))
        # the root's one call: its own shard, capacity = the whole batch, every rank's size in rank order
        assert calls == [(sizes[0], n * 16, sizes, 0)]
        # the root's plan: its own shard copied, every other non-empty one received, at prefix sums
        offs = np.concatenate([[0], np.cumsum(sizes)[:-1]]).tolist()
        assert ops == [[(_lib.SRPC_GATHER_COPY if r == 0 else _lib.SRPC_GATHER_RECV, r, offs[r], sizes[r])
                        for r in range(world) if sizes[r]]]
        if n % (16 * world):
            assert len(set(sizes)) > 1  # uneven shards really were exercised


def test_gather_plan_checks_like_gather_wire():
    """srpc_gather_plan refuses what srpc_gather_wire refuses, with the same
    codes, before any operation is listed (host arithmetic: no GPU)."""
    E_INV, E_CAP = _lib.SRPC_E_INVALID, _lib.SRPC_E_CAPACITY

    def code(*a):
        try:
            gather_plan(*a)
            return 0
        except _lib.SrpcError as e:
            return e.code
    sizes = [32, 48, 0, 16]
    assert code(0, 4, 0, 32, sizes, 96) == 0
    assert code(0, 4, 0, 32, sizes, 95) == E_CAP          # concatenation larger than the root's buffer
    assert code(0, 4, 0, 31, sizes, 96) == E_INV          # the root's own entry is not its shard
    assert code(0, 4, 0, 32, None, 96) == E_INV           # the root needs every size
    assert code(1, 4, 0, 48, None, 0) == 0                # a sender needs none
    assert code(4, 4, 0, 0, sizes, 96) == E_INV           # rank out of range
    assert code(0, 4, 4, 0, sizes, 96) == E_INV           # root out of range
    assert code(0, 2, 0, 1, [1, 2**64 - 1], 2**64 - 1) == E_INV  # sizes overflow
    assert gather_plan(2, 4, 0, 0, None, 0) == []         # an empty shard sends nothing
    assert gather_plan(0, 4, 3, 32, sizes, 0) == [(_lib.SRPC_GATHER_SEND, 3, 0, 32)]
    assert gather_plan(3, 4, 3, 16, sizes, 96) == [(_lib.SRPC_GATHER_RECV, 0, 0, 32),
                                                   (_lib.SRPC_GATHER_RECV, 1, 32, 48),
                                                   (_lib.SRPC_GATHER_COPY, 3, 80, 16)]
    L = _lib.lib()
    k = ctypes.c_int(-1)
    few = (_lib.GatherOp * 1)()
    h = (ctypes.c_uint64 * 4)(*sizes)
    assert L.srpc_gather_plan(3, 4, 3, 16, h, 96, few, 1, ctypes.byref(k)) == E_CAP and k.value == 0
