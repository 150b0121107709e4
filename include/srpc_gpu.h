/*
 * srpc_gpu.h -- C ABI of the MI355X (gfx950) batched sRPC packer.
 *
 * This is the drop-in boundary for the reference's packer hot path.  The
 * reference has no FFI of its own: its "operator API" is the header-only C++
 * template surface of namespace srpc (include/srpc/packer.hpp:53-181).  Each
 * entry point below replaces a loop over one of those calls with one batched,
 * stream-ordered launch over N records:
 *
 *   srpc_gpu_pack    <- `packer p; for (r : batch) p << r;`
 *                       (packer.hpp:73 -> pack_arg 183-191 -> pack_struct 172-178),
 *                       and, with a request/response prefix, the loops over
 *                       pack_request (packer.hpp:77-82) / pack_response (86-91)
 *   srpc_gpu_unpack  <- `for (r : batch) r.unpack(bp);` (generated unpack,
 *                       examples/calculator_srpc.cpp:19-22, calling
 *                       packer::operator>> 70 -> pipe_output 210-222), and,
 *                       with a prefix, unpack_request / unpack_response / getv
 *                       (packer.hpp:95-162) for records of one known type
 *   srpc_plan_create <- the compile-time reflection over T::fields
 *                       (core.hpp:9-14, STRUCT_MEMBER) that fixes field order
 *                       and sizes; the C++ side (include/srpc/gpu.hpp) builds
 *                       the descriptor from T::fields automatically.
 *
 * Wire bytes are identical to the reference's: raw little-endian fields in
 * declaration order, no padding, nested messages inlined, strings as a u64
 * length followed by the bytes, records back to back.
 *
 * Conventions
 *   - All data pointers are DEVICE pointers (hipMalloc'd) unless named h_*.
 *     The library allocates nothing on the pack/unpack hot path.
 *   - `stream` is a hipStream_t (NULL = the default stream).  Calls are
 *     asynchronous and stream-ordered; they are safe to capture in a hipGraph.
 *   - Return values: 0 = launched; <0 = argument / HIP error (nothing launched);
 *     >0 = a data error detected on the host (see SRPC_ERR_*).  No exception
 *     ever crosses this ABI (the reference terminates instead: core.hpp:28-33
 *     throws inside noexcept functions).
 *   - Threading: a plan is immutable after creation and may be used from any
 *     host thread and on any stream of its device concurrently.
 */
#ifndef SRPC_GPU_H
#define SRPC_GPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SRPC_GPU_ABI_VERSION 8

/* Field kinds = the IDL type table of the reference (parser.hpp:253-290).
 * Nested message fields are flattened into their members by the caller. */
typedef enum srpc_kind {
    SRPC_KIND_BOOL = 1,   /* bool    : 1 byte               */
    SRPC_KIND_INT8 = 2,   /* int8_t  : 1 byte               */
    SRPC_KIND_CHAR = 3,   /* char    : 1 byte               */
    SRPC_KIND_INT16 = 4,  /* int16_t : 2 bytes LE           */
    SRPC_KIND_INT32 = 5,  /* int32_t : 4 bytes LE           */
    SRPC_KIND_INT64 = 6,  /* int64_t : 8 bytes LE           */
    SRPC_KIND_STRING = 7  /* u64 LE length + raw bytes      */
} srpc_kind;

/* Return codes. */
#define SRPC_OK 0
#define SRPC_E_INVALID (-1)     /* bad argument or schema                       */
#define SRPC_E_ALIGN (-2)       /* a device pointer violates the alignment rule */
#define SRPC_E_HIP (-3)         /* HIP runtime / launch failure                 */
#define SRPC_E_UNSUPPORTED (-4) /* no kernel for this schema / layout; chunked host call in a capture */
#define SRPC_E_CAPACITY (-5)    /* output buffer too small                      */
#define SRPC_ERR_BOUNDS 2       /* wire shorter than n records; the records that
                                   fit were decoded, the status says where the
                                   first missing one starts                      */

/* Device-side decode status bits (srpc_unpack_status.flags). */
#define SRPC_STATUS_PREFIX 1u   /* a record's envelope header != the plan's prefix */
#define SRPC_STATUS_BOUNDS 2u   /* a record (or string) ran past the wire end      */
#define SRPC_STATUS_STALLED 4u  /* srpc_gpu_unpack_var, several string fields: a
                                   tile's chars-offset look-back polled its
                                   predecessors past its budget (2^21 polls of
                                   one word, ~1 s: only a device shared with
                                   kernels that keep every earlier tile from
                                   being scheduled).  The outputs are not valid;
                                   retry the call.  The stream decode
                                   (srpc_gpu_unpack_var_stream) never waits and
                                   never reports it. */

/* Written by srpc_gpu_unpack when its d_status argument is non-NULL.
 * Reset by the call itself (stream-ordered) before decoding starts. */
typedef struct srpc_unpack_status {
    uint32_t flags;             /* OR of SRPC_STATUS_* over the batch          */
    uint32_t reserved;          /* diagnostics of srpc_gpu_unpack_var_stream: bit 0 =
                                   the cursor entered some block at a table slot
                                   other than the block's speculated start, bit 1 =
                                   it entered some block where no table slot was
                                   (that block was walked record by record),
                                   bit 2 = the first scan met such a position and
                                   the repair pass gave every block exit slots,
                                   bit 3 = some block had more possible entries
                                   than its exit slots hold (those may walk),
                                   bits 8-31 = scan waves that walked (saturating);
                                   0 from every other call                     */
    uint64_t first_bad_record;  /* smallest failing record index, or UINT64_MAX */
} srpc_unpack_status;

/* A flat record schema: fields in T::fields declaration order
 * (packer.hpp:172-178), plus an optional constant per-record header: the
 * `u64 len | method | u64 len | T::name` of pack_request, or the
 * `u8 code | u64 len | T::name` of pack_response. */
typedef struct srpc_schema_desc {
    uint32_t nfields;
    const int32_t* kinds;   /* host array of nfields srpc_kind values */
    const uint8_t* prefix;  /* host bytes, may be NULL when prefix_len == 0 */
    uint32_t prefix_len;
} srpc_schema_desc;

typedef struct srpc_plan srpc_plan;

/* Which kernel family a plan runs (srpc_plan_info). */
#define SRPC_PATH_DWORD 1   /* every field 4/8 B, no prefix, record <= 32 B:
                               one record per lane, register-assembled records          */
#define SRPC_PATH_TILE 2    /* any fixed-size schema: LDS-staged tiles, 16 B global I/O  */
#define SRPC_PATH_VAR 3     /* string fields: per-record sizes + wavefront/device scan   */

/* Validate a schema and prepare its kernels on `device` (allocates the
 * plan's small device-side prefix copy; never called on the hot path).
 * Limits of this build (the reference's pack_struct has none, packer.hpp:
 * 172-178): at most SRPC_MAX_FIELDS leaf fields after flattening and an
 * envelope prefix of at most SRPC_MAX_PREFIX bytes -- so a fixed record is at
 * most 1024 + 32 * 8 = 1280 bytes.  A schema past a limit is refused with
 * SRPC_E_UNSUPPORTED before any device work; nfields == 0, an unknown kind or
 * a NULL pointer is SRPC_E_INVALID.  (srpc::gpu::batch_packer<T> throws
 * srpc::gpu::plan_error carrying the code.) */
#define SRPC_MAX_FIELDS 32
#define SRPC_MAX_PREFIX 1024
int srpc_plan_create(const srpc_schema_desc* desc, int device, srpc_plan** out);
int srpc_plan_destroy(srpc_plan* plan);

/* Fixed wire bytes per record (prefix included); 0 for string schemas. */
int srpc_plan_record_bytes(const srpc_plan* plan, uint64_t* out);
/* Kernel family in use (SRPC_PATH_*). */
int srpc_plan_path(const srpc_plan* plan, int* out);
/* Testing hook: force a kernel family the schema is eligible for
 * (SRPC_PATH_TILE is valid for every fixed schema). */
int srpc_plan_force_path(srpc_plan* plan, int path);

/* Performance knobs (defaults are the measured best on
 * MI355X; results are identical for every setting). */
#define SRPC_TUNE_RECORDS_PER_LANE 1 /* 1 or 4 (4: 16-byte column loads, needs 4-byte
                                        fields and 16-byte aligned columns) */
#define SRPC_TUNE_ITER 2             /* records (or quads) per lane per launch: 1,2,4,8 */
#define SRPC_TUNE_NONTEMPORAL 3      /* bit0 non-temporal stores, bit1 loads      */
#define SRPC_TUNE_TILE_BYTES 4       /* TILE path: target LDS image bytes per tile
                                        (1024..49152), pack and unpack           */
#define SRPC_TUNE_WAVE_PACK_BYTES 11   /* TILE path: pack with one wave per tile of about this
                                         many image bytes (0 = workgroup tiles)        */
#define SRPC_TUNE_WAVE_UNPACK_BYTES 12 /* TILE path: the same for unpack                */
#define SRPC_TUNE_PACK_TILE_BYTES 9  /* TILE path: the same for the pack kernel only */
#define SRPC_TUNE_VAR_KERNEL 7       /* VAR: 1 = record tiles, one pass (default; unpack of
                                        records under 40 bytes on average keeps 0), 0 =
                                        offset scans + chunk walks, 2 = record tiles for
                                        every unpack */
#define SRPC_TUNE_VAR_IMAGE_BYTES 8  /* VAR record tiles: LDS image bytes (8192..65536,
                                        multiple of 16); larger tiles take the walk  */
#define SRPC_TUNE_VAR_CHARS_BYTES 10 /* VAR record tiles: LDS chars stage bytes
                                        (0..65536, multiple of 16)                   */
#define SRPC_TUNE_REC_KERNEL 13      /* TILE path: schema-specialised kernels for the
                                        layouts that have one: 1 = in the directions
                                        where they measured faster (default), 2 = both
                                        directions, 0 = generic kernels only        */
#define SRPC_TUNE_GRID 5             /* DWORD path: max workgroups (0 = one per
                                        256*iter records; else grid-stride)       */
int srpc_plan_tune(srpc_plan* plan, int knob, int value);

/* Pack n records.  d_cols[f] (host array of nfields device pointers) holds
 * n elements of field f's C type, 4-byte aligned (16-byte for the TILE
 * path).  d_wire receives n * record_bytes bytes; wire_cap is its size.
 * d_wire must be 16-byte aligned. */
int srpc_gpu_pack(const srpc_plan* plan, const void* const* d_cols, uint64_t n,
                  uint8_t* d_wire, uint64_t wire_cap, void* stream);

/* Unpack n records from wire_len bytes at d_wire into the columns d_cols.
 * Every record's prefix is checked against the plan's; mismatches are
 * reported in *d_status (if non-NULL), and the record's fields are still
 * decoded from their fixed positions.  If wire_len < n * record_bytes the
 * records that fit are decoded and SRPC_ERR_BOUNDS is returned (status
 * flags BOUNDS, first_bad_record = wire_len / record_bytes). */
int srpc_gpu_unpack(const srpc_plan* plan, const uint8_t* d_wire, uint64_t wire_len,
                    uint64_t n, void* const* d_cols, srpc_unpack_status* d_status,
                    void* stream);

/* ---- fixed-size records held as the caller's own structs (AoS) -------------
 * The reference's caller holds std::vector<T> and loops `p << r`
 * (packer.hpp:73).  These take the struct array itself, copied to the device
 * as raw bytes: record r's leaf field f is at d_records + r * record_stride +
 * field_offsets[f] (host array, nfields entries, T::fields order, nested
 * messages flattened), naturally aligned (offset, stride and base multiples of
 * the field size: SRPC_E_ALIGN otherwise).  Wire bytes are those of
 * srpc_gpu_pack / srpc_gpu_unpack.  unpack_aos writes only the leaf fields'
 * bytes of each struct; every other byte (padding, a vtable pointer) keeps
 * what d_records held.  srpc::gpu::batch_packer<T>::pack_records /
 * unpack_records compute the offsets from T::fields. */
int srpc_gpu_pack_aos(const srpc_plan* plan, const void* d_records, uint64_t record_stride,
                      const uint32_t* field_offsets, uint64_t n, uint8_t* d_wire, uint64_t wire_cap,
                      void* stream);
int srpc_gpu_unpack_aos(const srpc_plan* plan, const uint8_t* d_wire, uint64_t wire_len, uint64_t n,
                        void* d_records, uint64_t record_stride, const uint32_t* field_offsets,
                        srpc_unpack_status* d_status, void* stream);
/* Unpack into FRESH objects (the reference's `std::vector<T> out(n); for
 * (auto& r : out) r.unpack(...)`, generated T::unpack writing only the leaf
 * fields of default-constructed objects): as srpc_gpu_unpack_aos, but every
 * struct byte no leaf field covers is set from h_fill (host, record_stride
 * bytes: e.g. the bytes of a T{} -- its vtable pointer and the defaults of
 * members the message does not carry) instead of being kept, so the old
 * array is never read.  record_stride <= 256 (SRPC_E_UNSUPPORTED otherwise);
 * h_fill is copied during the call.  Records past a short wire (BOUNDS) are
 * left as they were, as in srpc_gpu_unpack_aos. */
int srpc_gpu_unpack_aos_fill(const srpc_plan* plan, const uint8_t* d_wire, uint64_t wire_len, uint64_t n,
                             void* d_records, uint64_t record_stride, const uint32_t* field_offsets,
                             const void* h_fill, srpc_unpack_status* d_status, void* stream);

/* ---- variable-length (string) schemas (SRPC_PATH_VAR) ----------------------
 * A string field f is given as its chars d_cols[f] plus n+1 u64 byte offsets
 * d_str_offs[f] (lengths are offs[i+1]-offs[i]; offs[0] need not be 0).
 * d_str_offs is a host array of nfields device pointers, NULL for fixed fields.
 * Record starts: d_rec_offs, n+1 u64, [0] = 0, [n] = total wire bytes.
 * Both calls need `scratch_bytes` of device scratch (8-byte aligned) from
 * srpc_plan_var_scratch_bytes(plan, n, wire_bytes), wire_bytes being the
 * pack call's wire_cap or the unpack call's wire_len; like the fixed calls
 * they are stream-ordered and allocate nothing. */
int srpc_plan_var_scratch_bytes(const srpc_plan* plan, uint64_t n, uint64_t wire_bytes,
                                uint64_t* out);

/* Pack n records (reference: the `p << r` / pack_request loop over records
 * with std::string members, packer.hpp:193-198).  Writes d_rec_offs[0..n]
 * (an exclusive scan of the record sizes) and the wire bytes.  If the batch
 * needs more than wire_cap bytes, only the first wire_cap are written and
 * *d_status (if non-NULL) gets SRPC_STATUS_BOUNDS with the first record that
 * did not fit; the caller reads d_rec_offs[n] for the size actually needed. */
int srpc_gpu_pack_var(const srpc_plan* plan, const void* const* d_cols,
                      const uint64_t* const* d_str_offs, uint64_t n, uint8_t* d_wire,
                      uint64_t wire_cap, uint64_t* d_rec_offs, srpc_unpack_status* d_status,
                      void* d_scratch, uint64_t scratch_bytes, void* stream);

/* Unpack n records whose starts are d_rec_offs[0..n] (the record index the
 * packer produced, or the frame boundaries of a socket stream) (reference:
 * pipe_output<std::string>, packer.hpp:216-222).  Fixed fields go to
 * d_cols[f] (aligned to their size); string field f's bytes go back to back
 * into d_cols[f] (16-byte aligned, room for wire_len bytes) with offsets
 * d_str_offs[f][0..n].  Prefix mismatches, string lengths past a record's
 * end and records whose size disagrees with the index are reported in
 * *d_status. */
int srpc_gpu_unpack_var(const srpc_plan* plan, const uint8_t* d_wire, uint64_t wire_len,
                        uint64_t n, const uint64_t* d_rec_offs, void* const* d_cols,
                        uint64_t* const* d_str_offs, srpc_unpack_status* d_status,
                        void* d_scratch, uint64_t scratch_bytes, void* stream);

/* Tile table (ABI 6): for every 256-record tile t of a string batch and
 * every string field s (in field order), the chars of field s in records
 * [0, min(256 t, n)): (ceil(n / 256) + 1) * nstrings u64, written by
 * srpc_gpu_var_tile_table from the batch's string offsets (e.g. the pack
 * call's input d_str_offs).  Given to srpc_gpu_unpack_var_tiled, every tile
 * of a schema with several string fields takes its output bases from it
 * instead of looking back at the tiles before it; each tile checks its own
 * totals against the table's differences (a wrong table is detected and the
 * batch decoded again with the look-back, bit-identically).  The table moves
 * 8 bytes per 256 records per string field beside the record index.
 * A NULL table: srpc_gpu_unpack_var. */
int srpc_var_tile_table_words(const srpc_plan* plan, uint64_t n, uint64_t* out);
int srpc_gpu_var_tile_table(const srpc_plan* plan, const uint64_t* const* d_str_offs, uint64_t n,
                            uint64_t* d_table, void* stream);
int srpc_gpu_unpack_var_tiled(const srpc_plan* plan, const uint8_t* d_wire, uint64_t wire_len,
                              uint64_t n, const uint64_t* d_rec_offs, const uint64_t* d_table,
                              void* const* d_cols, uint64_t* const* d_str_offs,
                              srpc_unpack_status* d_status, void* d_scratch, uint64_t scratch_bytes,
                              void* stream);

/* Unpack n records from a stream with NO record index -- the reference's own
 * decode of a concatenated batch with one shared cursor (buffer::_offset,
 * core.hpp:39; packer.hpp:210-222) -- e.g. the bytes a reference packer
 * appended.  The record starts are found on the device and written to
 * d_rec_offs[0..n] with the records decoded as by srpc_gpu_unpack_var: per
 * 8 KiB block, speculative walks from plausible record starts give a table
 * from "where the cursor enters the block" to "where it leaves" (records,
 * chars per string field); an in-order scan of the tables gives every block
 * its exact entry and output bases; then every block writes its records.
 * Nothing waits on the device; work is bounded by the stream's bytes on any
 * input (a cursor position no table holds is walked record by record).
 * The first record the cursor cannot read (prefix mismatch, or a field /
 * string past the end) is reported in *d_status as the first bad record
 * (PREFIX or BOUNDS), as orc_unpack / the reference would meet it; its start
 * is d_rec_offs[i] and every later entry is wire_len (those records are
 * BOUNDS too).  Scratch: srpc_plan_var_stream_scratch_bytes (256-byte
 * aligned). */
int srpc_plan_var_stream_scratch_bytes(const srpc_plan* plan, uint64_t n, uint64_t wire_len,
                                       uint64_t* out);
int srpc_gpu_unpack_var_stream(const srpc_plan* plan, const uint8_t* d_wire, uint64_t wire_len,
                               uint64_t n, uint64_t* d_rec_offs, void* const* d_cols,
                               uint64_t* const* d_str_offs, srpc_unpack_status* d_status,
                               void* d_scratch, uint64_t scratch_bytes, void* stream);

/* ---- multi-GPU: sharded batches, packed bytes gathered over RCCL -------------
 * The reference packer appends (core.hpp:34, packer.hpp:73), so a batch
 * split into contiguous record shards [lo_g, hi_g) in rank order, each packed
 * on its own GPU, concatenates back to the single-GPU wire exactly.  The only
 * collective is a gather of the shards' wire bytes to a root (ncclSend /
 * ncclRecv in one group), bound by the root's xGMI ingress. */
#define SRPC_SHARD_ALIGN_RECORDS 16  /* shard starts are multiples of 16 records */
#define SRPC_COMM_ID_BYTES 128       /* an RCCL unique id                         */
typedef struct srpc_comm srpc_comm;

/* Records [*lo, *hi) of shard `rank` of n records over nranks shards:
 * contiguous, in rank order, starts aligned to SRPC_SHARD_ALIGN_RECORDS.
 * Host arithmetic only. */
int srpc_shard_range(uint64_t n, int rank, int nranks, uint64_t* lo, uint64_t* hi);

/* One process per GPU: rank 0 makes an id, the caller distributes it
 * (e.g. over its own process group), every rank joins with its device. */
int srpc_comm_unique_id(uint8_t* id_out /* SRPC_COMM_ID_BYTES */);
int srpc_comm_init_rank(const uint8_t* id, int nranks, int rank, int device, srpc_comm** out);
/* One process driving ndev devices: out[g] is rank g on devices[g]. */
int srpc_comm_init_all(const int* devices, int ndev, srpc_comm** out /* ndev */);
int srpc_comm_destroy(srpc_comm* comm);
int srpc_comm_rank(const srpc_comm* comm, int* rank, int* nranks);

/* Each rank contributes one u64 (e.g. its shard's wire bytes, read from the
 * last entry of its d_rec_offs for string schemas); d_out gets nranks. */
int srpc_allgather_u64(srpc_comm* comm, const uint64_t* d_in, uint64_t* d_out, void* stream);

/* The gather's plan, host arithmetic only: the operations rank `rank` of
 * srpc_gather_wire enqueues, in order -- a non-root rank one SEND of its shard
 * (none when it is empty); the root a RECV from every other rank with bytes
 * and a COPY of its own shard, each at byte offset sum(h_all_bytes[0..peer))
 * of the root's wire.  The same argument checks as srpc_gather_wire
 * (SRPC_E_INVALID, SRPC_E_CAPACITY) in the same order; ops gets at most
 * cap_ops entries (SRPC_E_CAPACITY when nranks would not fit), *nops the
 * count.  srpc_gather_wire runs exactly this list, so a transport other
 * than RCCL (a test's gloo) can replay it byte for byte. */
#define SRPC_GATHER_SEND 1
#define SRPC_GATHER_RECV 2
#define SRPC_GATHER_COPY 3
typedef struct srpc_gather_op {
    int32_t kind;    /* SRPC_GATHER_SEND / _RECV / _COPY                       */
    int32_t peer;    /* SEND: the root; RECV: the sender; COPY: the root itself */
    uint64_t offset; /* byte offset into the root's wire (0 for SEND)           */
    uint64_t bytes;
} srpc_gather_op;
int srpc_gather_plan(int rank, int nranks, int root, uint64_t shard_bytes, const uint64_t* h_all_bytes,
                     uint64_t root_cap, srpc_gather_op* ops, int cap_ops, int* nops);

/* Gather: every rank calls it with its shard's wire bytes; the root receives
 * shard r at byte offset sum(h_all_bytes[0..r)) of d_root_wire (root_cap
 * bytes) -- the single-GPU wire of the whole batch.  h_all_bytes (host, one
 * entry per rank) is needed on the root only.  Stream-ordered.  Every
 * argument is checked before the RCCL group is opened; if an operation then
 * cannot be enqueued the group is ended unlaunched and the communicators it
 * touched are aborted (later calls on them return SRPC_E_INVALID). */
int srpc_gather_wire(srpc_comm* comm, const uint8_t* d_shard, uint64_t shard_bytes,
                     uint8_t* d_root_wire, uint64_t root_cap, const uint64_t* h_all_bytes,
                     int root, void* stream);
/* The same from one process for all ndev ranks of srpc_comm_init_all
 * (streams[g] on device g). */
int srpc_group_gather_wire(srpc_comm* const* comms, int ndev, const uint8_t* const* d_shards,
                           const uint64_t* h_bytes, uint8_t* d_root_wire, uint64_t root_cap,
                           int root, void* const* streams);
/* One process, ndev devices, a fixed-size schema: plans[g] (created on device
 * g) packs shard g -- d_cols[g] holds records srpc_shard_range(n, g, ndev) on
 * device g -- into d_shard_wire[g], then the shards are gathered into
 * d_root_wire on the root. */
int srpc_group_pack_gather(const srpc_plan* const* plans, srpc_comm* const* comms, int ndev,
                           const void* const* const* d_cols, uint64_t n, uint8_t* const* d_shard_wire,
                           uint8_t* d_root_wire, uint64_t root_cap, int root, void* const* streams);

/* ---- framed request batches of several methods (server side) ----------------
 * The reference server reads one frame (transport.hpp recv_data: BE32 length |
 * payload) and dispatches it by the method name it starts with (server.hpp:
 * 58-69).  A batch read from a socket holds frames of any method in any order.
 * srpc_frames_classify puts frame i (bytes [d_offs[i], d_offs[i+1]) of d_buf,
 * the last frame ending at buf_len) into bucket k when it is exactly one record
 * of req_plans[k]; the first matching plan wins:
 *   - a fixed-size plan whose prefix is the frame's constant
 *     `BE32 len | str(method) | str(Req::name)`: same length, same prefix;
 *   - a string plan (a method whose request has string fields; at most
 *     SRPC_FRAMES_MAX_STRINGS of them) whose prefix is `str(method) |
 *     str(Req::name)`: the frame's BE32 is its payload length, the payload
 *     starts with the prefix and its fields, each string length read from
 *     the frame, end exactly at the frame's end.
 * A frame whose offsets are out of order or run past buf_len is
 * SRPC_FRAME_UNKNOWN (no byte outside d_buf is read).
 * Outputs (device):
 *   d_class[i]             k, or SRPC_FRAME_UNKNOWN (the caller answers it);
 *   d_index[k*nframes + j] the frames of bucket k (j < d_counts[k]; order
 *                          within a bucket is unspecified);
 *   d_counts[0..nplans+1]  frames per bucket, then the response stream's total
 *                          bytes, then the number of unknown frames;
 *   d_out_off[0..nframes]  byte offset of frame i's response in the batch's
 *                          response stream (resp_bytes[k] per frame of bucket
 *                          k, 0 for unknown frames and for string plans' frames,
 *                          whose sizes srpc_frames_offsets adds), total at
 *                          [nframes].
 * nplans <= SRPC_FRAMES_MAX_PLANS.  Scratch: srpc_frames_scratch_bytes, 8-byte
 * aligned.  Stream-ordered; nothing is synchronised. */
#define SRPC_FRAME_UNKNOWN 0xFF
#define SRPC_FRAMES_MAX_PLANS 16
#define SRPC_FRAMES_MAX_STRINGS 16
int srpc_frames_scratch_bytes(uint64_t nframes, int nplans, uint64_t* out);
int srpc_frames_classify(const srpc_plan* const* req_plans, const uint32_t* resp_bytes, int nplans,
                         const uint8_t* d_buf, uint64_t buf_len, const uint32_t* d_offs,
                         uint64_t nframes, uint8_t* d_class, uint32_t* d_index, uint64_t* d_counts,
                         uint64_t* d_out_off, void* d_scratch, uint64_t scratch_bytes, void* stream);
/* d_out[j*record_bytes ..] = the record_bytes bytes at d_buf + d_offs[d_index[j]], j < n. */
int srpc_frames_gather(const uint8_t* d_buf, const uint32_t* d_offs, const uint32_t* d_index,
                       uint64_t n, uint32_t record_bytes, uint8_t* d_out, void* stream);
/* d_out + d_out_off[d_index[j]] = response j (record_bytes bytes of d_resp), j < n. */
int srpc_frames_scatter(const uint8_t* d_resp, const uint32_t* d_index, uint64_t n,
                        uint32_t record_bytes, const uint64_t* d_out_off, uint8_t* d_out,
                        void* stream);
/* String plans' buckets.  gather_var: the payloads (each frame after its BE32
 * length) of frames d_index[0..n) back to back into d_out -- the records of a
 * string request plan -- and their record index d_rec_offs[0..n] (n+1 u64) for
 * srpc_gpu_unpack_var.  Frames must be ones srpc_frames_classify put in a
 * string plan's bucket.  Scratch: srpc_frames_scratch_bytes(n, 1, ..). */
int srpc_frames_gather_var(const uint8_t* d_buf, const uint32_t* d_offs, const uint32_t* d_index,
                           uint64_t n, uint8_t* d_out, uint64_t* d_rec_offs, void* d_scratch,
                           uint64_t scratch_bytes, void* stream);
/* scatter_var: response j (bytes [d_rec_offs[j], d_rec_offs[j+1]) of d_resp, as
 * srpc_gpu_pack_var wrote them with their index) framed as `BE32 len |
 * response` at d_out + d_out_off[d_index[j]], j < n. */
int srpc_frames_scatter_var(const uint8_t* d_resp, const uint64_t* d_rec_offs,
                            const uint32_t* d_index, uint64_t n, const uint64_t* d_out_off,
                            uint8_t* d_out, void* stream);
/* The reply stream's offsets once string plans' responses are packed: frame i
 * takes resp_bytes[k] (fixed plan k), 4 + its response's bytes (string plan k:
 * d_var_rec_offs[k], a host array of nplans device pointers -- the index
 * srpc_gpu_pack_var wrote for bucket k's records in d_index order; NULL for
 * fixed plans), 0 (unknown).  Writes d_out_off[0..nframes] and *d_total.
 * Same plans, d_class, d_index and d_counts as the classify call; same
 * scratch size. */
int srpc_frames_offsets(const srpc_plan* const* req_plans, const uint32_t* resp_bytes, int nplans,
                        const uint8_t* d_class, uint64_t nframes, const uint32_t* d_index,
                        const uint64_t* d_counts, const uint64_t* const* d_var_rec_offs,
                        uint64_t* d_out_off, uint64_t* d_total, void* d_scratch,
                        uint64_t scratch_bytes, void* stream);

/* ---- utilities --------------------------------------------------------------*/

/* Synthetic input of SURVEY.md §8c: nfields int32 columns, record i field f =
 * low 32 bits of splitmix64 draw number (first_record + i) * nfields + f + 1
 * from state `seed`.  Used by bench.py to build inputs in HBM. */
int srpc_gpu_fill_splitmix_i32(int32_t* const* d_cols, uint32_t nfields, uint64_t n,
                               uint64_t seed, uint64_t first_record, void* stream);

/* Host-terminated pack / unpack (ABI 7): columns and wire bytes in HOST
 * memory (pinned for overlap), as the reference's batches start and end --
 * the packer's byte vector written to the socket (transport.hpp:94-123) and
 * the received bytes the generated unpack reads (calculator_srpc.cpp:19-22).
 * A fixed-width batch moves in chunks of `chunk_records` through a ring of
 * `depth` device buffers carved from d_scratch (256-byte aligned, at least
 * srpc_plan_host_scratch_bytes), pipelined over internal streams (H2D /
 * kernels / D2H), ordered after the work on `stream` and before what is
 * enqueued on it later.  The results equal srpc_gpu_pack / srpc_gpu_unpack
 * on the whole batch, statuses included (first_bad_record is batch-relative).
 * chunk_records == 0 is the direct mode: when every host buffer is page-
 * locked and device-mapped (hipHostMalloc, hipHostRegister, torch pin_memory)
 * the kernels read and write them in place over PCIe, both directions at
 * once, no scratch, no copies; each buffer's pinned allocation must cover its
 * n records (else SRPC_E_INVALID, nothing launched).  Every argument is
 * checked before anything is enqueued.  The chunked mode borrows three
 * streams and their events from a per-device pool (created on first use, kept
 * for the process, grown only by calls in flight at once); unlike the other
 * calls it is not meant for hipGraph capture.  An error part way through the
 * chunked ring still orders everything the call enqueued before `stream`'s
 * later work.  String schemas: SRPC_E_UNSUPPORTED. */
int srpc_plan_host_scratch_bytes(const srpc_plan* plan, uint64_t chunk_records, uint32_t depth,
                                 uint64_t* out);
int srpc_gpu_pack_host(const srpc_plan* plan, const void* const* h_cols, uint64_t n, uint8_t* h_wire,
                       uint64_t wire_cap, uint64_t chunk_records, uint32_t depth, void* d_scratch,
                       uint64_t scratch_bytes, void* stream);
int srpc_gpu_unpack_host(const srpc_plan* plan, const uint8_t* h_wire, uint64_t wire_len, uint64_t n,
                         void* const* h_cols, uint64_t chunk_records, uint32_t depth, void* d_scratch,
                         uint64_t scratch_bytes, srpc_unpack_status* d_status, void* stream);

/* Measurement hook (bench.py): the data-path kernels launched by the NEXT
 * srpc_gpu_pack / _unpack / _pack_var / _unpack_var call made on this host
 * thread record the begin timestamp of the first kernel into `start_event`
 * and the end timestamp of the last into `stop_event` (hipEvent_t handles
 * created with timing enabled; either may be NULL), taken from the dispatch
 * packets themselves (hipExtLaunchKernel) -- kernel-only time, the interval
 * rocprofv3 --kernel-trace reports.  Status-reset launches are not timed.
 * The hook is consumed by that one call, whatever it returns. */
int srpc_time_next_call(void* start_event, void* stop_event);

const char* srpc_status_string(int code);
int srpc_gpu_abi_version(void);

#ifdef __cplusplus
}
#endif

#endif /* SRPC_GPU_H */
