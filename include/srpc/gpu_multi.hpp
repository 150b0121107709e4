// srpc/gpu_multi.hpp -- record batches sharded over the node's GPUs,
// host C++ over the C ABI of include/srpc_gpu.h.
//
// The reference packer appends (core.hpp:34, packer.hpp:73): the wire of a
// batch is the concatenation of its records' wires.  So a batch of n records
// is cut into contiguous shards in rank order (shard_range), every shard is
// packed on its own GPU with no collective on the data path, and where the
// bytes are needed in one place the shards are gathered to a root over RCCL
// (xGMI), which reproduces the single-GPU wire exactly.
//
//   srpc::gpu::comm              one rank of a communicator (one process per GPU)
//   srpc::gpu::device_group      one process driving G devices (ncclCommInitAll)
//   srpc::gpu::sharded_packer<T> a device_group with one batch_packer<T> per device
#pragma once

#include <array>
#include <cstdint>
#include <string>
#include <utility>
#include <vector>

#include "gpu.hpp"

namespace srpc::gpu {

/// Records [lo, hi) of shard `rank` of n over nranks (starts 16-record aligned).
inline std::pair<uint64_t, uint64_t> shard_range(uint64_t n, int rank, int nranks) {
    uint64_t lo = 0, hi = 0;
    if (int rc = srpc_shard_range(n, rank, nranks, &lo, &hi); rc != SRPC_OK) throw plan_error("srpc_shard_range", rc);
    return {lo, hi};
}

using comm_id = std::array<uint8_t, SRPC_COMM_ID_BYTES>;

/// One rank of an RCCL communicator: rank 0 makes the id (unique_id()), the
/// caller hands it to the other processes, every rank constructs a comm.
class comm {
public:
    static comm_id unique_id() {
        comm_id id{};
        if (int rc = srpc_comm_unique_id(id.data()); rc != SRPC_OK) throw plan_error("srpc_comm_unique_id", rc);
        return id;
    }
    comm(comm_id const& id, int nranks, int rank, int device) {
        if (int rc = srpc_comm_init_rank(id.data(), nranks, rank, device, &_c); rc != SRPC_OK)
            throw plan_error("srpc_comm_init_rank", rc);
    }
    comm(comm&& o) noexcept : _c(o._c) { o._c = nullptr; }
    comm(comm const&) = delete;
    comm& operator=(comm const&) = delete;
    ~comm() {
        if (_c) srpc_comm_destroy(_c);
    }
    int rank() const {
        int r = 0;
        srpc_comm_rank(_c, &r, nullptr);
        return r;
    }
    int nranks() const {
        int n = 0;
        srpc_comm_rank(_c, nullptr, &n);
        return n;
    }
    srpc_comm* get() const { return _c; }

    /// Every rank: its shard's wire bytes; the root receives the batch's
    /// wire in d_root (all_bytes: every rank's shard bytes, root only).
    int gather_wire(const uint8_t* d_shard, uint64_t shard_bytes, uint8_t* d_root, uint64_t root_cap,
                    std::vector<uint64_t> const& all_bytes, int root = 0, void* stream = nullptr) const {
        return srpc_gather_wire(_c, d_shard, shard_bytes, d_root, root_cap, all_bytes.empty() ? nullptr : all_bytes.data(),
                                root, stream);
    }

private:
    srpc_comm* _c = nullptr;
};

/// One process driving several devices: rank g of the communicator is devices[g].
class device_group {
public:
    explicit device_group(std::vector<int> devices) : _dev(std::move(devices)), _c(_dev.size(), nullptr) {
        if (int rc = srpc_comm_init_all(_dev.data(), static_cast<int>(_dev.size()), _c.data()); rc != SRPC_OK)
            throw plan_error("srpc_comm_init_all", rc);
    }
    device_group(device_group const&) = delete;
    device_group& operator=(device_group const&) = delete;
    /// Moves hand the communicators over; the source keeps none to destroy.
    device_group(device_group&& o) noexcept : _dev(std::move(o._dev)), _c(std::move(o._c)) { o._c.clear(); }
    device_group& operator=(device_group&& o) noexcept {
        if (this != &o) {
            release();
            _dev = std::move(o._dev);
            _c = std::move(o._c);
            o._c.clear();
        }
        return *this;
    }
    ~device_group() { release(); }
    int size() const { return static_cast<int>(_dev.size()); }
    int device(int g) const { return _dev[static_cast<size_t>(g)]; }
    srpc_comm* const* comms() const { return _c.data(); }

private:
    void release() noexcept {
        for (srpc_comm* c : _c)
            if (c) srpc_comm_destroy(c);
        _c.clear();
    }
    std::vector<int> _dev;
    std::vector<srpc_comm*> _c;
};

/// A device_group with one plan of T (body, request or response envelope)
/// per device; pack_gather packs every shard on its device and gathers the
/// batch's wire on the root.
template <SrpcMessage T>
class sharded_packer {
public:
    explicit sharded_packer(std::vector<int> devices) : _group(devices) {
        for (int d : devices) _p.emplace_back(d);
    }
    static sharded_packer request(std::vector<int> devices, std::string const& method) {
        sharded_packer s(std::move(devices), 0);
        for (int g = 0; g < s._group.size(); ++g) s._p.push_back(batch_packer<T>::request(method, s._group.device(g)));
        return s;
    }

    int size() const { return _group.size(); }
    batch_packer<T> const& packer(int g) const { return _p[static_cast<size_t>(g)]; }
    uint64_t record_bytes() const { return _p.front().record_bytes(); }
    std::pair<uint64_t, uint64_t> shard(uint64_t n, int g) const { return shard_range(n, g, size()); }

    /// d_cols[g]: device g's columns holding records shard(n, g); d_shard_wire[g]
    /// its wire; d_root (on device root) receives n * record_bytes() bytes.
    int pack_gather(std::vector<const void* const*> const& d_cols, uint64_t n,
                    std::vector<uint8_t*> const& d_shard_wire, uint8_t* d_root, uint64_t root_cap, int root,
                    std::vector<void*> const& streams) const {
        std::vector<const srpc_plan*> plans;
        for (auto const& p : _p) plans.push_back(p.plan());
        return srpc_group_pack_gather(plans.data(), _group.comms(), size(), d_cols.data(), n, d_shard_wire.data(),
                                      d_root, root_cap, root, streams.data());
    }

private:
    sharded_packer(std::vector<int> devices, int) : _group(std::move(devices)) {}
    device_group _group;
    std::vector<batch_packer<T>> _p;
};

}  // namespace srpc::gpu
