"""The N>1 path on CPU: contiguous record shards packed independently and
gathered to rank 0 (srpc_amd.shard) reproduce the single-batch wire bytes.
world_size 2 and 3 over gloo; each rank's shard is packed by the CPU oracle
standing in for its GPU (the kernel itself is covered by the gpu tests)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import oracle
from srpc_amd.shard import gather_packed, shard_range


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, n, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        lo, hi = shard_range(n, rank, world)
        cols = oracle.splitmix_columns_i32(4, hi - lo, first_record=lo)
        local = np.frombuffer(oracle.pack([oracle.INT32] * 4, cols, hi - lo), np.uint8).copy()
        out = gather_packed(torch.from_numpy(local), 16, n)
        if rank == 0:
            q.put(out.numpy().tobytes())
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,n", [(2, 4096), (2, 1000), (3, 4099), (2, 0), (3, 17)])
def test_sharded_pack_gather_equals_single_batch(world, n):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = q.get(timeout=120)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    want = oracle.pack([oracle.INT32] * 4, oracle.splitmix_columns_i32(4, n), n)
    assert got == want
