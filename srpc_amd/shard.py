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


def gather_packed(local, record_bytes: int, n: int, root: int = 0, group=None, comm: "NativeComm | None" = None):
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
    if comm is not None:  # the library's RCCL gather (production path)
        return comm.gather_wire(local, sizes, root)
    # torch.distributed: the library's own plan (srpc_gather_plan, the list
    # srpc_gather_wire enqueues) replayed as point-to-point operations
    out = None
    if rank == root:
        out = torch.empty(n * record_bytes, dtype=torch.uint8, device=local.device)
    run_gather_plan(gather_plan(rank, world, root, sizes[rank], sizes, n * record_bytes), local, out, group)
    return out


def gather_plan(rank: int, nranks: int, root: int, shard_bytes: int, all_bytes, root_cap: int) -> list:
    """srpc_gather_plan of the C ABI: the (kind, peer, offset, bytes) operations
    rank ``rank`` of srpc_gather_wire enqueues, after the same argument checks
    (raises SrpcError with SRPC_E_INVALID / SRPC_E_CAPACITY as it would)."""
    import ctypes as C

    from . import _lib
    sizes = (C.c_uint64 * nranks)(*[int(b) for b in all_bytes]) if all_bytes is not None else None
    ops = (_lib.GatherOp * nranks)()
    k = C.c_int()
    _lib.check(_lib.lib().srpc_gather_plan(rank, nranks, root, shard_bytes, sizes, root_cap, ops, nranks,
                                           C.byref(k)), "srpc_gather_plan")
    return [(ops[i].kind, ops[i].peer, ops[i].offset, ops[i].bytes) for i in range(k.value)]


def run_gather_plan(ops, local, out, group=None, p2p: bool = True) -> None:
    """Replays srpc_gather_plan's list over torch.distributed: SEND -> isend of
    the shard, RECV -> irecv into out[offset:offset+bytes], COPY -> the root's
    own shard.  ``p2p=False`` uses blocking send/recv in list order (gloo)."""
    import torch.distributed as dist

    from . import _lib
    pending = []
    for kind, peer, off, b in ops:
        if kind == _lib.SRPC_GATHER_COPY:
            out[off:off + b].copy_(local[:b])
        elif kind == _lib.SRPC_GATHER_SEND:
            pending.append(dist.P2POp(dist.isend, local[:b].contiguous(), peer, group) if p2p else
                           ("send", local[:b].contiguous(), peer))
        elif kind == _lib.SRPC_GATHER_RECV:
            pending.append(dist.P2POp(dist.irecv, out[off:off + b], peer, group) if p2p else
                           ("recv", out[off:off + b], peer))
        else:
            raise ValueError(f"unknown gather op kind {kind}")
    if p2p:
        if pending:
            for w in dist.batch_isend_irecv(pending):
                w.wait()
        return
    for what, t, peer in pending:
        if what == "send":
            dist.send(t, peer, group)
        else:
            buf = t.new_empty(t.shape)  # out[...] slices are views: receive, then place
            dist.recv(buf, peer, group)
            t.copy_(buf)


class NativeComm:
    """One rank of an RCCL communicator owned by libsrpc_gpu (srpc_comm_init_rank):
    the gather of packed shards runs in the library (ncclSend / ncclRecv to
    the root inside one group, include/srpc_gpu.h srpc_gather_wire), not
    through torch.  The 128-byte RCCL id is made by rank 0 and handed to the
    other ranks over the caller's own process group."""

    def __init__(self, uid: bytes, nranks: int, rank: int, device: int):
        import ctypes as C

        from . import _lib
        self.rank, self.nranks, self.device = rank, nranks, device
        buf = (C.c_uint8 * len(uid)).from_buffer_copy(uid)
        h = C.c_void_p()
        _lib.check(_lib.lib().srpc_comm_init_rank(buf, nranks, rank, device, C.byref(h)), "srpc_comm_init_rank")
        self._h = h

    @staticmethod
    def unique_id() -> bytes:
        import ctypes as C

        from . import _lib
        buf = (C.c_uint8 * _lib.SRPC_COMM_ID_BYTES)()
        _lib.check(_lib.lib().srpc_comm_unique_id(buf), "srpc_comm_unique_id")
        return bytes(buf)

    @classmethod
    def from_process_group(cls, device: int, group=None) -> "NativeComm":
        import torch.distributed as dist
        rank, world = dist.get_rank(group), dist.get_world_size(group)
        obj = [cls.unique_id() if rank == 0 else None]
        dist.broadcast_object_list(obj, src=0, group=group)
        return cls(obj[0], world, rank, device)

    def gather_wire(self, local, all_bytes, root: int = 0, out=None, stream=None):
        """Every rank: its packed shard (uint8 device tensor).  Root: returns the
        concatenation in rank order (``out`` or a new tensor); others None."""
        import torch

        sizes = [int(b) for b in all_bytes]
        if len(sizes) != self.nranks:
            raise ValueError(f"{len(sizes)} shard sizes for {self.nranks} ranks")
        total = sum(sizes)
        if self.rank == root and out is None:
            out = torch.empty(max(total, 1), dtype=torch.uint8, device=local.device)
        self._gather(local, sizes[self.rank], out if self.rank == root else None,
                     total if self.rank == root else 0, sizes, root, stream)
        return out[:total] if self.rank == root else None

    def _gather(self, local, shard_bytes, out, root_cap, sizes, root, stream) -> None:
        """srpc_gather_wire of the C ABI: shard r lands at sum(sizes[:r]) of
        the root's ``out``."""
        import ctypes as C

        from . import _lib
        from .packer import _dptr, _stream
        h = (C.c_uint64 * len(sizes))(*sizes)
        _lib.check(_lib.lib().srpc_gather_wire(self._h, _dptr(local) if shard_bytes else None, shard_bytes,
                                               _dptr(out) if out is not None else None, root_cap, h, root,
                                               _stream(stream)), "srpc_gather_wire")

    def info(self) -> dict:
        """What the RCCL communicator itself reports (srpc_comm_rank)."""
        import ctypes as C

        from . import _lib
        r, nr = C.c_int(), C.c_int()
        _lib.check(_lib.lib().srpc_comm_rank(self._h, C.byref(r), C.byref(nr)), "srpc_comm_rank")
        return {"rank": r.value, "nranks": nr.value, "device": self.device}

    def close(self) -> None:
        from . import _lib
        if getattr(self, "_h", None) is not None and self._h.value:
            _lib.lib().srpc_comm_destroy(self._h)
            self._h.value = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def native_shard_range(n: int, rank: int, world: int) -> tuple[int, int]:
    """srpc_shard_range of the C ABI (host arithmetic, the same rule as shard_range)."""
    import ctypes as C

    from . import _lib
    lo, hi = C.c_uint64(), C.c_uint64()
    _lib.check(_lib.lib().srpc_shard_range(n, rank, world, C.byref(lo), C.byref(hi)), "srpc_shard_range")
    return lo.value, hi.value
