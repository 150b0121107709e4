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
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import oracle
from srpc_amd.shard import NativeComm, gather_packed, shard_range


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


class FakeComm(NativeComm):
    """NativeComm with srpc_gather_wire's data movement done over gloo: the
    same argument checks as multi.hip (the root's own size, the capacity, the
    size list's length), the same placement (prefix sums, rank order)."""

    def __init__(self, rank, nranks):  # no RCCL communicator behind it
        self.rank, self.nranks, self.device = rank, nranks, -1
        self._h = None
        self.calls = []

    def _gather(self, local, shard_bytes, out, root_cap, sizes, root, stream):
        self.calls.append((shard_bytes, root_cap, tuple(sizes), root))
        assert len(sizes) == self.nranks and local.numel() >= shard_bytes
        if self.rank != root:
            if shard_bytes:
                dist.send(local[:shard_bytes].contiguous(), root)
            return
        assert sizes[root] == shard_bytes, "SRPC_E_INVALID: root's own size"
        assert sum(sizes) <= root_cap, "SRPC_E_CAPACITY"
        off = 0
        for r, b in enumerate(sizes):
            if b:
                view = out[off:off + b]
                if r == root:
                    view.copy_(local[:b])
                else:
                    buf = torch.empty(b, dtype=torch.uint8)
                    dist.recv(buf, r)
                    view.copy_(buf)
            off += b

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
            q.put((out.numpy().tobytes(), comm.calls if comm else None))
        else:
            assert out is None
            if comm and world > 1:  # every rank passed its own shard's bytes
                assert [c[0] for c in comm.calls] == [(hi - lo) * 16]
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,n,use_comm", [(2, 4096, False), (2, 1000, False), (3, 4099, False), (2, 0, False),
                                              (3, 17, False), (2, 1000, True), (3, 4099, True), (8, 1001, True),
                                              (8, 17, True), (8, 0, True)])
def test_sharded_pack_gather_equals_single_batch(world, n, use_comm):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n, use_comm, q)) for r in range(world)]
    for p in procs:
        p.start()
    got, calls = q.get(timeout=180)
    for p in procs:
        p.join(timeout=180)
        assert p.exitcode == 0
    want = oracle.pack([oracle.INT32] * 4, oracle.splitmix_columns_i32(4, n), n)
    assert got == want
    if use_comm:
        sizes = tuple((hi - lo) * 16 for lo, hi in (shard_range(n, r, world) for r in range(world)))
        # the root's one call: its own shard, capacity = the whole batch, every rank's size in rank order
        assert calls == [(sizes[0], n * 16, sizes, 0)]
        if n % (16 * world):
            assert len(set(sizes)) > 1  # uneven shards really were exercised
