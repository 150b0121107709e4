// multi.hip -- record batches sharded over the node's GPUs, packed bytes
// gathered to a root over RCCL (xGMI) (north_star: "record batches
// sharded across the node's 8 GPUs with an RCCL gather of packed bytes").
//
// Why sharding is exact: the reference packer appends (buffer::append,
// core.hpp:34; packer::operator<<, packer.hpp:73), so the wire of a batch is
// the concatenation of its records' wires.  A batch of n records split into
// contiguous shards [lo_g, hi_g) in rank order, each packed on its own GPU and
// concatenated in rank order, is byte-identical to the single-GPU pack.
//
// The exchange is the only collective: a gather of every shard's wire bytes
// into the root's buffer at the shard's byte offset (the prefix sum of the
// shard sizes), as ncclSend / ncclRecv pairs inside one ncclGroupStart /
// ncclGroupEnd.  It is bound by the root's xGMI ingress, (G - 1) links.
// Two communicator forms: one process per GPU (srpc_comm_init_rank, the id
// exchanged by the caller, e.g. over its own process group) and one process
// driving G devices (srpc_comm_init_all, srpc_group_gather_wire).
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstring>
#include <new>
#include <vector>

#include "plan.h"
#include "srpc_gpu.h"

struct srpc_comm {
    ncclComm_t comm = nullptr;
    int rank = 0, nranks = 1, device = 0;
    bool owned = true;
};

namespace {
using namespace srpc_impl;

int nccl_rc(ncclResult_t r) { return r == ncclSuccess ? SRPC_OK : SRPC_E_HIP; }

// Ends a group of sends / receives.  When an operation could not be enqueued
// (rc != OK), the group is half built: RCCL's ncclGroupEnd returns the stored
// error without launching it, and every communicator it touched is aborted
// (ncclCommAbort), so no peer waits on a live communicator for an operation
// that will never come; those comms then refuse further work (comm = NULL)
// and srpc_comm_destroy only frees them.
int close_group(int rc, srpc_comm* const* comms, int n) {
    const int end = nccl_rc(ncclGroupEnd());
    if (rc == SRPC_OK) return end;
    for (int g = 0; g < n; ++g)
        if (comms[g] && comms[g]->comm) {
            DeviceGuard dg(comms[g]->device);
            (void)ncclCommAbort(comms[g]->comm);
            comms[g]->comm = nullptr;
        }
    return rc;
}

}  // namespace

extern "C" {

int srpc_shard_range(uint64_t n, int rank, int nranks, uint64_t* lo, uint64_t* hi) {
    if (nranks <= 0 || rank < 0 || rank >= nranks || !lo || !hi) return SRPC_E_INVALID;
    const uint64_t a = SRPC_SHARD_ALIGN_RECORDS;
    const uint64_t blocks = (n + a - 1) / a;
    // blocks * rank / nranks without overflow for any n < 2^64
    auto cut = [&](int r) {
        const unsigned __int128 b = static_cast<unsigned __int128>(blocks) * static_cast<unsigned>(r) / nranks;
        const unsigned __int128 x = b * a;
        return x > n ? n : static_cast<uint64_t>(x);
    };
    *lo = cut(rank);
    *hi = cut(rank + 1);
    return SRPC_OK;
}

int srpc_comm_unique_id(uint8_t* out) {
    if (!out) return SRPC_E_INVALID;
    ncclUniqueId id;
    if (ncclGetUniqueId(&id) != ncclSuccess) return SRPC_E_HIP;
    static_assert(sizeof(id) == SRPC_COMM_ID_BYTES, "RCCL unique id size");
    std::memcpy(out, &id, sizeof(id));
    return SRPC_OK;
}

int srpc_comm_init_rank(const uint8_t* id, int nranks, int rank, int device, srpc_comm** out) {
    if (!id || !out || nranks <= 0 || rank < 0 || rank >= nranks) return SRPC_E_INVALID;
    *out = nullptr;
    auto* c = new (std::nothrow) srpc_comm();
    if (!c) return SRPC_E_INVALID;
    c->rank = rank;
    c->nranks = nranks;
    c->device = device;
    ncclUniqueId uid;
    std::memcpy(&uid, id, sizeof(uid));
    DeviceGuard g(device);
    if (ncclCommInitRank(&c->comm, nranks, uid, rank) != ncclSuccess) {
        delete c;
        return SRPC_E_HIP;
    }
    *out = c;
    return SRPC_OK;
}

int srpc_comm_init_all(const int* devices, int ndev, srpc_comm** out) {
    if (!devices || !out || ndev <= 0) return SRPC_E_INVALID;
    std::vector<ncclComm_t> comms(static_cast<size_t>(ndev));
    if (ncclCommInitAll(comms.data(), ndev, devices) != ncclSuccess) return SRPC_E_HIP;
    for (int g = 0; g < ndev; ++g) {
        auto* c = new (std::nothrow) srpc_comm();
        if (!c) {
            for (int k = 0; k < ndev; ++k) (void)ncclCommDestroy(comms[static_cast<size_t>(k)]);
            for (int k = 0; k < g; ++k) delete out[k];
            return SRPC_E_INVALID;
        }
        c->comm = comms[static_cast<size_t>(g)];
        c->rank = g;
        c->nranks = ndev;
        c->device = devices[g];
        out[g] = c;
    }
    return SRPC_OK;
}

int srpc_comm_destroy(srpc_comm* c) {
    if (!c) return SRPC_E_INVALID;
    int rc = SRPC_OK;
    if (c->comm) {
        DeviceGuard g(c->device);
        rc = nccl_rc(ncclCommDestroy(c->comm));
    }
    delete c;
    return rc;
}

int srpc_comm_rank(const srpc_comm* c, int* rank, int* nranks) {
    if (!c) return SRPC_E_INVALID;
    if (rank) *rank = c->rank;
    if (nranks) *nranks = c->nranks;
    return SRPC_OK;
}

int srpc_allgather_u64(srpc_comm* c, const uint64_t* d_in, uint64_t* d_out, void* stream) {
    if (!c || !c->comm || !d_in || !d_out) return SRPC_E_INVALID;
    DeviceGuard g(c->device);
    return nccl_rc(ncclAllGather(d_in, d_out, 1, ncclUint64, c->comm, static_cast<hipStream_t>(stream)));
}

int srpc_gather_plan(int rank, int nranks, int root, uint64_t shard_bytes, const uint64_t* h_all_bytes,
                     uint64_t root_cap, srpc_gather_op* ops, int cap_ops, int* nops) {
    if (nranks <= 0 || rank < 0 || rank >= nranks || root < 0 || root >= nranks || !nops) return SRPC_E_INVALID;
    *nops = 0;
    if (cap_ops > 0 && !ops) return SRPC_E_INVALID;
    if (rank != root) {
        if (!shard_bytes) return SRPC_OK;
        if (cap_ops < 1) return SRPC_E_CAPACITY;
        ops[0] = srpc_gather_op{SRPC_GATHER_SEND, root, 0, shard_bytes};
        *nops = 1;
        return SRPC_OK;
    }
    // the root: sizes summed without overflow, its own entry its shard, the
    // concatenation within its buffer -- all before any operation is listed
    if (!h_all_bytes) return SRPC_E_INVALID;
    uint64_t total = 0;
    int want = 0;
    for (int r = 0; r < nranks; ++r) {
        if (h_all_bytes[r] > ~0ull - total) return SRPC_E_INVALID;
        total += h_all_bytes[r];
        want += h_all_bytes[r] != 0;
    }
    if (h_all_bytes[root] != shard_bytes) return SRPC_E_INVALID;
    if (total > root_cap) return SRPC_E_CAPACITY;
    if (want > cap_ops) return SRPC_E_CAPACITY;
    uint64_t off = 0;
    int k = 0;
    for (int r = 0; r < nranks; ++r) {
        const uint64_t b = h_all_bytes[r];
        if (b) ops[k++] = srpc_gather_op{r == root ? SRPC_GATHER_COPY : SRPC_GATHER_RECV, r, off, b};
        off += b;
    }
    *nops = k;
    return SRPC_OK;
}

int srpc_gather_wire(srpc_comm* c, const uint8_t* d_shard, uint64_t shard_bytes, uint8_t* d_root_wire,
                     uint64_t root_cap, const uint64_t* h_all_bytes, int root, void* stream) {
    if (!c || !c->comm || root < 0 || root >= c->nranks) return SRPC_E_INVALID;
    if (shard_bytes && !d_shard) return SRPC_E_INVALID;
    // every argument checked (srpc_gather_plan) before the group is opened
    std::vector<srpc_gather_op> ops(static_cast<size_t>(c->nranks));
    int nops = 0;
    if (int rc = srpc_gather_plan(c->rank, c->nranks, root, shard_bytes, h_all_bytes, root_cap, ops.data(),
                                  c->nranks, &nops))
        return rc;
    if (nops == 0) return SRPC_OK;
    if (c->rank == root && !d_root_wire) return SRPC_E_INVALID;
    auto s = static_cast<hipStream_t>(stream);
    DeviceGuard g(c->device);
    if (c->rank != root)  // one send, no group needed
        return nccl_rc(ncclSend(d_shard, ops[0].bytes, ncclUint8, root, c->comm, s));
    if (ncclGroupStart() != ncclSuccess) return SRPC_E_HIP;
    int rc = SRPC_OK;
    for (int k = 0; k < nops && rc == SRPC_OK; ++k) {
        const srpc_gather_op& op = ops[static_cast<size_t>(k)];
        if (op.kind == SRPC_GATHER_COPY) {
            if (hipMemcpyAsync(d_root_wire + op.offset, d_shard, op.bytes, hipMemcpyDeviceToDevice, s) != hipSuccess)
                rc = SRPC_E_HIP;
        } else {
            rc = nccl_rc(ncclRecv(d_root_wire + op.offset, op.bytes, ncclUint8, op.peer, c->comm, s));
        }
    }
    return close_group(rc, &c, 1);
}

int srpc_group_gather_wire(srpc_comm* const* comms, int ndev, const uint8_t* const* d_shards,
                           const uint64_t* h_bytes, uint8_t* d_root_wire, uint64_t root_cap, int root,
                           void* const* streams) {
    if (!comms || ndev <= 0 || !d_shards || !h_bytes || root < 0 || root >= ndev || !streams) return SRPC_E_INVALID;
    uint64_t total = 0;
    for (int g = 0; g < ndev; ++g) {
        if (!comms[g] || !comms[g]->comm || comms[g]->nranks != ndev || comms[g]->rank != g) return SRPC_E_INVALID;
        if (h_bytes[g] && !d_shards[g]) return SRPC_E_INVALID;
        if (h_bytes[g] > ~0ull - total) return SRPC_E_INVALID;
        total += h_bytes[g];
    }
    if (total > root_cap) return SRPC_E_CAPACITY;
    if (total && !d_root_wire) return SRPC_E_INVALID;
    // one group over every device's operations (a single process drives all ranks)
    if (ncclGroupStart() != ncclSuccess) return SRPC_E_HIP;
    int rc = SRPC_OK;
    uint64_t off = 0;
    for (int g = 0; g < ndev && rc == SRPC_OK; ++g) {
        const uint64_t b = h_bytes[g];
        auto sg = static_cast<hipStream_t>(streams[g]);
        auto sr = static_cast<hipStream_t>(streams[root]);
        if (b) {
            if (g == root) {
                DeviceGuard dg(comms[root]->device);
                if (hipMemcpyAsync(d_root_wire + off, d_shards[g], b, hipMemcpyDeviceToDevice, sr) != hipSuccess)
                    rc = SRPC_E_HIP;
            } else {
                rc = nccl_rc(ncclSend(d_shards[g], b, ncclUint8, root, comms[g]->comm, sg));
                if (rc == SRPC_OK) rc = nccl_rc(ncclRecv(d_root_wire + off, b, ncclUint8, g, comms[root]->comm, sr));
            }
        }
        off += b;
    }
    return close_group(rc, comms, ndev);
}

int srpc_group_pack_gather(const srpc_plan* const* plans, srpc_comm* const* comms, int ndev,
                           const void* const* const* d_cols, uint64_t n, uint8_t* const* d_shard_wire,
                           uint8_t* d_root_wire, uint64_t root_cap, int root, void* const* streams) {
    if (!plans || !comms || ndev <= 0 || !d_cols || !d_shard_wire || !streams) return SRPC_E_INVALID;
    if (root < 0 || root >= ndev) return SRPC_E_INVALID;
    uint64_t rb = 0;
    if (srpc_plan_record_bytes(plans[0], &rb) != SRPC_OK || rb == 0) return SRPC_E_INVALID;  // fixed schemas
    if (n > ~0ull / rb) return SRPC_E_INVALID;
    if (n * rb > root_cap) return SRPC_E_CAPACITY;
    if (n && !d_root_wire) return SRPC_E_INVALID;
    for (int g = 0; g < ndev; ++g)  // everything checked before the first shard is packed
        if (!plans[g] || !comms[g] || !comms[g]->comm || !d_cols[g] || !d_shard_wire[g]) return SRPC_E_INVALID;
    std::vector<uint64_t> bytes(static_cast<size_t>(ndev));
    std::vector<const uint8_t*> shards(static_cast<size_t>(ndev));
    for (int g = 0; g < ndev; ++g) {
        uint64_t lo = 0, hi = 0;
        srpc_shard_range(n, g, ndev, &lo, &hi);
        uint64_t rbg = 0;
        if (srpc_plan_record_bytes(plans[g], &rbg) != SRPC_OK || rbg != rb) return SRPC_E_INVALID;
        bytes[static_cast<size_t>(g)] = (hi - lo) * rb;
        shards[static_cast<size_t>(g)] = d_shard_wire[g];
        DeviceGuard dg(comms[g]->device);
        // shard g: its columns already hold records [lo, hi) on device g
        if (int rc = srpc_gpu_pack(plans[g], d_cols[g], hi - lo, d_shard_wire[g], (hi - lo) * rb, streams[g]))
            return rc;
    }
    return srpc_group_gather_wire(comms, ndev, shards.data(), bytes.data(), d_root_wire, root_cap, root, streams);
}

}  // extern "C"
