// srpc/packer.hpp -- scalar (one message at a time) sRPC packer, MI355X build.
//
// Same API and wire bytes as the reference's include/srpc/packer.hpp, so
// generated stubs, servicers and the server link unchanged:
//   rpc_status_code          (reference packer.hpp:16-20)
//   request_t / response_t   (packer.hpp:22-51)
//   packer: ctors, data/size/offset/clear/buf, >>, <<, pack_request,
//           pack_response, unpack_request, unpack_response, getv
//                            (packer.hpp:53-181)
// Wire format (normative): fields are raw little-endian host
// bytes in T::fields order with no padding; nested messages are inlined;
// std::string / const char* are a u64 length followed by the bytes;
// pack_request = str(method) str(T::name) body; pack_response = u8 code
// str(T::name) body.
//
// Batches of records go through the GPU instead: srpc/gpu.hpp
// (srpc::gpu::batch_packer<T>), which produces exactly the bytes of a loop of
// `p << r` / `p.pack_request(...)` over the batch.
//
// Deliberate differences, invisible on valid input: every read is bounds-
// checked BEFORE it happens (the reference reads first, then throws inside a
// noexcept function => std::terminate, packer.hpp:210-214 + core.hpp:28-33);
// a short read zero-fills the value and sets buf()->failed().  A dynamic_cast
// that fails in unpack_request/unpack_response/getv leaves the default value
// instead of dereferencing nullptr.  `p >> msg` on a message type decodes it
// with msg.unpack() instead of memcpy'ing the object representation.
#pragma once

#include <cstdint>
#include <cstdio>
#include <cstring>
#include <memory>
#include <string>
#include <type_traits>
#include <utility>
#include <vector>

#include "core.hpp"

namespace srpc {

enum rpc_status_code : uint8_t {
    RPC_SUCCESS = 0,
    RPC_ERR_FUNCTION_NOT_REGISTERED,
    RPC_ERR_RECV_TIMEOUT
};

template <SrpcMessage T>
class request_t {
public:
    T value() const { return _value; }
    const std::string& method_name() const { return _method_name; }

    void set_value(T&& v) { _value = std::move(v); }
    void set_value(T const& v) { _value = v; }
    void set_method_name(std::string const& s) { _method_name = s; }

private:
    std::string _method_name;
    T _value{};
};

template <SrpcMessage T>
class response_t {
public:
    response_t() : _code(RPC_SUCCESS) {}

    rpc_status_code code() const { return _code; }
    T value() const { return _value; }

    void set_code(rpc_status_code c) { _code = c; }
    void set_value(T const& v) { _value = v; }

private:
    rpc_status_code _code;
    T _value{};
};

class packer {
public:
    using ptr = std::shared_ptr<packer>;

    packer() : _buf(std::make_shared<buffer>()) {}
    packer(const uint8_t* bytes, size_t len) : _buf(std::make_shared<buffer>(bytes, len)) {}
    packer(std::vector<uint8_t> const& bytes) : _buf(std::make_shared<buffer>(bytes)) {}
    packer(std::vector<uint8_t>&& bytes) : _buf(std::make_shared<buffer>(std::move(bytes))) {}
    packer(buffer::ptr buf_ptr) : _buf(std::move(buf_ptr)) {}

    /// Unread bytes start here / this many of them remain.
    const uint8_t* data() const { return _buf->curdata(); }
    size_t size() const { return _buf->cursize(); }
    size_t offset() const noexcept { return _buf->offset(); }
    void clear() noexcept { _buf->reset(); }
    buffer::ptr buf() noexcept { return _buf; }
    /// False once a read ran past the end of the buffer.
    bool ok() const noexcept { return !_buf->failed(); }

    template <typename T>
    packer& operator>>(T& v) {
        pipe_output(v);
        return *this;
    }

    /// By value, as in the reference: string literals decay to const char*.
    template <typename T>
    packer& operator<<(T v) {
        pack_arg(v);
        return *this;
    }

    /// Request envelope: str(method) | str(T::name) | body  (client -> server).
    template <SrpcMessage T>
    void pack_request(request_t<T> const& req) {
        pack_arg(req.method_name());
        pack_cstr(T::name);
        pack_struct(req.value());
    }

    /// Response envelope: u8 code | str(T::name) | body  (server -> client).
    template <SrpcMessage T>
    void pack_response(response_t<T> const& resp) {
        pack_arg(resp.code());
        pack_cstr(T::name);
        pack_struct(resp.value());
    }

    /// Server side: decode a request whose message type is R.
    template <SrpcMessage R>
    [[nodiscard]] request_t<R> unpack_request() noexcept {
        request_t<R> req;
        std::string method_name;
        *this >> method_name;
        req.set_method_name(method_name);
        std::string message_name;
        *this >> message_name;
        if (auto msg = make_registered<R>(message_name)) {
            msg->unpack(_buf);
            req.set_value(std::move(*msg));
        }
        return req;
    }

    /// Client side: decode a response whose message type is R.
    template <SrpcMessage R>
    [[nodiscard]] response_t<R> unpack_response() noexcept {
        response_t<R> res;
        rpc_status_code status = RPC_SUCCESS;
        *this >> status;
        res.set_code(status);
        std::string message_name;
        *this >> message_name;
        if (auto msg = make_registered<R>(message_name)) {
            msg->unpack(_buf);
            res.set_value(*msg);
        }
        return res;
    }

    /// Decode `str(T::name) | body`; the caller owns the returned object
    /// (nullptr if the name is not registered).
    template <SrpcMessage T>
    [[nodiscard]] T* getv() noexcept {
        std::string message_name;
        *this >> message_name;
        auto msg = make_registered<T>(message_name);
        if (!msg) {
            fprintf(stderr, "message %s not found!", message_name.c_str());
            return nullptr;
        }
        msg->unpack(_buf);
        return msg.release();
    }

private:
    template <typename T>
    static std::unique_ptr<T> make_registered(std::string const& name) {
        auto it = message_registry.find(name);
        if (it == message_registry.end()) return nullptr;
        std::unique_ptr<message_base> base = it->second();
        T* t = dynamic_cast<T*>(base.get());
        if (!t) return nullptr;
        base.release();
        return std::unique_ptr<T>(t);
    }

    template <typename T>
    void pack_arg(T const& arg) {
        if constexpr (std::is_base_of_v<message_base, T>) {
            pack_struct(arg);
        } else if constexpr (std::is_same_v<T, std::string>) {
            const uint64_t len = arg.size();
            pack_raw(len);
            _buf->append(reinterpret_cast<const uint8_t*>(arg.data()), arg.size());
        } else if constexpr (std::is_same_v<std::decay_t<T>, const char*> ||
                             std::is_same_v<std::decay_t<T>, char*>) {
            pack_cstr(arg);
        } else {
            static_assert(std::is_trivially_copyable_v<T>, "packer: unsupported field type");
            pack_raw(arg);
        }
    }

    void pack_cstr(const char* s) {
        const uint64_t len = std::strlen(s);
        pack_raw(len);
        _buf->append(reinterpret_cast<const uint8_t*>(s), len);
    }

    template <typename T>
    void pack_raw(T const& v) {
        _buf->append(reinterpret_cast<const uint8_t*>(&v), sizeof(T));
    }

    /// Message bodies: every T::fields member in declaration order.
    template <typename T>
        requires has_fields_v<T>
    void pack_struct(T const& arg) {
        std::apply([this, &arg](const auto&... member) { (pack_arg(arg.*(std::get<MEMBER_ADDR>(member))), ...); },
                   T::fields);
    }

    template <typename T>
    void pipe_output(T& v) noexcept {
        if constexpr (std::is_base_of_v<message_base, T>) {
            v.unpack(_buf);
        } else if constexpr (std::is_same_v<T, std::string>) {
            int64_t len = 0;
            pipe_output(len);
            if (len < 0 || !_buf->has(static_cast<size_t>(len))) {
                v.clear();
                _buf->increment(-1);  // clamp to the end and flag
                return;
            }
            v.assign(reinterpret_cast<const char*>(_buf->curdata()), static_cast<size_t>(len));
            _buf->increment(len);
        } else {
            static_assert(std::is_trivially_copyable_v<T>, "packer: unsupported field type");
            if (!_buf->has(sizeof(T))) {
                std::memset(static_cast<void*>(&v), 0, sizeof(T));
                _buf->increment(-1);
                return;
            }
            std::memcpy(static_cast<void*>(&v), _buf->curdata(), sizeof(T));
            _buf->increment(sizeof(T));
        }
    }

    buffer::ptr _buf;
};

}  // namespace srpc
