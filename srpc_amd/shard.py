"""Multi-GPU sharding of record batches.

Records are independent and ``wire(batch) = wire(r0) | wire(r1) | ...`` (the
reference's packer appends, core.hpp:34), so a batch of N records is split into
contiguous per-rank ranges, each rank packs its range on its own GPU with no
collective on the data path, and -- where the packed bytes are needed in one
place -- the shards are gathered to a root rank over RCCL (xGMI) in rank
order, which reproduces the single-GPU wire bytes exactly.
"""
from __future__ import annotations

ALIGN_RECORDS = 16  # shard starts stay multiples of 16 records (16-byte aligned wire/columns)


def shard_range(n: int, rank: int, world: int, align: int = ALIGN_RECORDS) -> tuple[int, int]:
    """[lo, hi) records of ``rank``: contiguous, in rank order, starts aligned."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError(f"bad rank {rank} / world {world}")
    blocks = (n + align - 1) // align
    lo = min(n, (blocks * rank // world) * align)
    hi = min(n, (blocks * (rank + 1) // world) * align)
    return lo, hi


def shard_ranges(n: int, world: int, align: int = ALIGN_RECORDS) -> list[tuple[int, int]]:
    return [shard_range(n, r, world, align) for r in range(world)]


def gather_packed(local, record_bytes: int, n: int, root: int = 0, group=None):
    """Gather every rank's packed shard into one wire buffer on ``root``.

    ``local``: this rank's packed bytes (uint8 tensor on its device, exactly
    (hi-lo)*record_bytes long).  Returns the full wire tensor on root, None
    elsewhere.  Equal shards use one ``gather`` (RCCL ncclSend/ncclRecv to the
    root); unequal ones a batch of point-to-point sends into slices of the
    root's buffer.  Both are bound by the root's xGMI ingress.
    """
    import torch
    import torch.distributed as dist

    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    if local.is_cuda and dist.get_backend(group) == "gloo":
        # gloo moves host memory only: stage through the CPU (test rehearsals;
        # production runs use RCCL, which reads and writes HBM directly)
        out = gather_packed(local.cpu(), record_bytes, n, root, group)
        return out.to(local.device) if out is not None else None
    ranges = shard_ranges(n, world)
    sizes = [(hi - lo) * record_bytes for lo, hi in ranges]
    if local.numel() != sizes[rank]:
        raise ValueError(f"rank {rank}: local shard has {local.numel()} bytes, expected {sizes[rank]}")
    if world == 1:
        return local
    out = None
    if rank == root:
        out = torch.empty(n * record_bytes, dtype=torch.uint8, device=local.device)
    if all(s == sizes[0] for s in sizes):
        parts = list(out.view(world, sizes[0]).unbind(0)) if rank == root else None
        dist.gather(local, gather_list=parts, dst=root, group=group)
        return out
    ops = []
    if rank == root:
        for r, (lo, hi) in enumerate(ranges):
            view = out[lo * record_bytes: hi * record_bytes]
            if r == root:
                view.copy_(local)
            elif view.numel():
                ops.append(dist.P2POp(dist.irecv, view, r, group))
    elif local.numel():
        ops.append(dist.P2POp(dist.isend, local, root, group))
    if ops:
        for w in dist.batch_isend_irecv(ops):
            w.wait()
    return out
