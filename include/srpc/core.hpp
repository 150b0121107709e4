// srpc/core.hpp -- core types of the sRPC C++ API (MI355X build).
//
// Source-compatible with the reference's include/srpc/core.hpp: generated
// message structs and stubs (examples/calculator_srpc.cpp) compile unchanged
// against this header.  Same names and meanings:
//   STRUCT_MEMBER            (reference core.hpp:9-11)   -> (name, &T::member) tuple
//   buffer                   (core.hpp:16-40)            -> byte vector + read cursor
//   message_base             (core.hpp:43-49)            -> name / fields / virtual unpack
//   servicer_base            (core.hpp:52-57)
//   function_traits          (core.hpp:59-93)
//   SrpcMessage/SrpcService  (core.hpp:125-129)
//   message_registry         (core.hpp:131-134)
// Deliberate differences (no caller can observe them on valid input):
//   * buffer::increment never throws; an out-of-range advance clamps the
//     cursor to the end and raises the buffer's `failed()` flag (the reference
//     throws inside noexcept callers, i.e. std::terminate, core.hpp:28-33).
//   * message_registry is an `inline` variable: one registry per program, not
//     one per translation unit (the reference's is namespace-scope `static`).
//   * the members are not `constexpr`, so the header builds with libstdc++ 11
//     (g++ 11) and clang alike.
#pragma once

#include <cstddef>
#include <cstdint>
#include <functional>
#include <memory>
#include <string>
#include <tuple>
#include <type_traits>
#include <unordered_map>
#include <vector>

namespace srpc {

#ifndef STRUCT_MEMBER
#define STRUCT_MEMBER(struct_t, member_name, member_str) std::make_tuple(member_str, &struct_t::member_name)
#endif

constexpr int MEMBER_NAME = 0;
constexpr int MEMBER_ADDR = 1;

/// Growable byte buffer with a read cursor.  Writers append at the end,
/// readers consume from the cursor; nested unpack() calls share one cursor.
struct buffer : public std::vector<uint8_t> {
    using ptr = std::shared_ptr<buffer>;

    buffer() = default;
    buffer(const uint8_t* bytes, size_t len) : std::vector<uint8_t>(bytes, bytes + len) {}
    buffer(std::vector<uint8_t> const& bytes) : std::vector<uint8_t>(bytes) {}
    buffer(std::vector<uint8_t>&& bytes) : std::vector<uint8_t>(std::move(bytes)) {}

    size_t cursize() const noexcept { return size() - _offset; }
    size_t offset() const noexcept { return _offset; }
    const uint8_t* data() const noexcept { return std::vector<uint8_t>::data(); }
    const uint8_t* curdata() const noexcept { return std::vector<uint8_t>::data() + _offset; }

    /// Advance the cursor by k bytes.  Out of range: clamp and flag.
    void increment(int64_t k) noexcept {
        if (k < 0 || static_cast<uint64_t>(k) > cursize()) {
            _failed = true;
            _offset = size();
            return;
        }
        _offset += static_cast<size_t>(k);
    }
    /// True when the next `k` bytes exist.
    bool has(size_t k) const noexcept { return k <= cursize(); }

    void append(const uint8_t* s, size_t len) { insert(end(), s, s + len); }
    template <typename It>
    void append(It b, It e) { insert(end(), b, e); }
    void reset() noexcept {
        _offset = 0;
        _failed = false;
        clear();
    }

    /// Set once a read ran past the end (the reference would have terminated).
    bool failed() const noexcept { return _failed; }
    void set_failed() noexcept { _failed = true; }

private:
    size_t _offset = 0;
    bool _failed = false;
};

/// To be inherited by generated messages.
struct message_base {
    virtual ~message_base() = default;
    virtual void unpack(buffer::ptr) {}

    static constexpr const char* name = nullptr;
    static constexpr auto fields = std::make_tuple();
};

/// To be inherited by generated servicers.
struct servicer_base {
    virtual ~servicer_base() = default;

    static constexpr const char* name = nullptr;
    static constexpr auto methods = std::make_tuple();
};

template <typename F>
struct function_traits;

template <typename R, typename I>
struct function_traits<R (*)(const I&)> {
    using input_type = I;
    using return_type = R;
};

template <typename I, typename R>
struct function_traits<std::function<R(const I&)>> {
    using input_type = I;
    using return_type = R;
};

template <typename C, typename R, typename I>
struct function_traits<R (C::*)(I)> {
    using class_type = C;
    using input_type = I;
    using return_type = R;
};

template <typename C, typename R, typename I>
struct function_traits<R (C::*)(I) const> {
    using class_type = C;
    using input_type = I;
    using return_type = R;
};

template <typename T, typename = void>
struct has_methods : std::false_type {};
template <typename T>
struct has_methods<T, std::void_t<decltype(T::methods)>> : std::true_type {};
template <typename T>
constexpr bool has_methods_v = has_methods<T>::value;

template <typename T, typename = void>
struct has_fields : std::false_type {};
template <typename T>
struct has_fields<T, std::void_t<decltype(T::fields)>> : std::true_type {};
template <typename T>
constexpr bool has_fields_v = has_fields<T>::value;

template <typename T, typename = void>
struct has_name : std::false_type {};
template <typename T>
struct has_name<T, std::void_t<decltype(T::name)>> : std::true_type {};
template <typename T>
constexpr bool has_name_v = has_name<T>::value;

template <typename D, typename B>
concept Derived = std::is_base_of_v<B, D>;

template <typename T>
concept SrpcMessage = has_name_v<T> && has_fields_v<T> && Derived<T, message_base>;

template <typename T>
concept SrpcService = has_name_v<T> && has_methods_v<T> && Derived<T, servicer_base>;

using message_factory = std::function<std::unique_ptr<message_base>()>;

/// Message name -> factory.  Populated by generated stubs.
inline std::unordered_map<std::string, message_factory> message_registry{};

}  // namespace srpc
