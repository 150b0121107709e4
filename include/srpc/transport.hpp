// srpc/transport.hpp -- TCP framing for sRPC (MI355X build).
//
// Same API and frames as the reference's include/srpc/transport.hpp:
//   message_t                      (reference transport.hpp:18-29)
//   transport::create_server_socket(port)              (:33-65)
//   transport::create_client_socket(server_ip, port)   (:67-92)
//   transport::send_data(fd, data, len)                (:94-105)
//   transport::recv_data(fd) -> message_t              (:107-123)
// Frame = u32 BIG-endian payload length | payload.
//
// Fixed here (no effect on the bytes on the wire):
//   * create_client_socket connects to `server_ip` (the reference ignores it
//     and resolves the null host, so a 0.0.0.0 server and a ::1 client never
//     meet -- SURVEY.md §4); the server listens dual-stack where it can.
//   * send/recv loop over partial transfers.
//   * recv_data's buffer is owned by the returned message_t (the reference
//     leaks it, transport.hpp:115).
#pragma once

#include <arpa/inet.h>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <sys/socket.h>
#include <sys/types.h>
#include <unistd.h>

#include <cerrno>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <string>

namespace srpc {

#ifndef SOCKET_SEND_FLAGS
#define SOCKET_SEND_FLAGS MSG_NOSIGNAL
#endif
#ifndef BACKLOG_SZ
#define BACKLOG_SZ 64
#endif

struct message_t {
    message_t() = default;
    /// Wrap caller-owned bytes.
    message_t(uint8_t* data, size_t size) : _size(size), _data(data) {}
    /// Allocate `size` owned bytes.
    explicit message_t(size_t size)
        : _size(size), _own(new uint8_t[size ? size : 1], std::default_delete<uint8_t[]>()), _data(_own.get()) {}

    const uint8_t* data() const noexcept { return _data; }
    uint8_t* mutable_data() noexcept { return _data; }
    size_t size() const noexcept { return _size; }

private:
    size_t _size = 0;
    std::shared_ptr<uint8_t> _own;
    uint8_t* _data = nullptr;
};

namespace transport {

/// Listen on `port` (all interfaces; IPv6 dual-stack when available).
[[nodiscard]] inline int32_t create_server_socket(const std::string& port) {
    addrinfo hints{};
    hints.ai_family = AF_UNSPEC;
    hints.ai_socktype = SOCK_STREAM;
    hints.ai_flags = AI_PASSIVE;
    addrinfo* res = nullptr;
    if (int st = getaddrinfo(nullptr, port.c_str(), &hints, &res); st != 0) {
        fprintf(stderr, "srpc::transport::create_server_socket(): getaddrinfo error: %s\n", gai_strerror(st));
        return -1;
    }
    int32_t fd = -1;
    // Prefer an IPv6 wildcard with V6ONLY off (accepts IPv4 too), else IPv4.
    for (int pass = 0; pass < 2 && fd < 0; ++pass) {
        for (addrinfo* ai = res; ai; ai = ai->ai_next) {
            if ((pass == 0) != (ai->ai_family == AF_INET6)) continue;
            int s = socket(ai->ai_family, ai->ai_socktype, ai->ai_protocol);
            if (s < 0) continue;
            int one = 1, zero = 0;
            setsockopt(s, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
            if (ai->ai_family == AF_INET6) setsockopt(s, IPPROTO_IPV6, IPV6_V6ONLY, &zero, sizeof(zero));
            if (bind(s, ai->ai_addr, ai->ai_addrlen) == 0 && listen(s, BACKLOG_SZ) == 0) {
                fd = s;
                break;
            }
            close(s);
        }
    }
    freeaddrinfo(res);
    if (fd < 0) fprintf(stderr, "srpc::transport::create_server_socket(): bind/listen failed.\n");
    return fd;
}

/// Connect to server_ip:port (every resolved address is tried in turn).
[[nodiscard]] inline int32_t create_client_socket(const std::string& server_ip, const std::string& port) {
    addrinfo hints{};
    hints.ai_family = AF_UNSPEC;
    hints.ai_socktype = SOCK_STREAM;
    addrinfo* res = nullptr;
    const char* host = server_ip.empty() ? nullptr : server_ip.c_str();
    if (int st = getaddrinfo(host, port.c_str(), &hints, &res); st != 0) {
        fprintf(stderr, "srpc::transport::create_client_socket(): getaddrinfo error: %s\n", gai_strerror(st));
        return -1;
    }
    int32_t fd = -1;
    for (addrinfo* ai = res; ai && fd < 0; ai = ai->ai_next) {
        int s = socket(ai->ai_family, ai->ai_socktype, ai->ai_protocol);
        if (s < 0) continue;
        if (connect(s, ai->ai_addr, ai->ai_addrlen) == 0) {
            int one = 1;
            setsockopt(s, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
            fd = s;
        } else {
            close(s);
        }
    }
    freeaddrinfo(res);
    if (fd < 0) fprintf(stderr, "srpc::transport::create_client_socket(): error connecting socket.\n");
    return fd;
}

/// Write all `len` bytes (loops over partial sends).  False on error.
inline bool send_all(int32_t fd, const void* p, size_t len) {
    const uint8_t* b = static_cast<const uint8_t*>(p);
    while (len) {
        ssize_t k = send(fd, b, len, SOCKET_SEND_FLAGS);
        if (k < 0 && errno == EINTR) continue;
        if (k <= 0) return false;
        b += k;
        len -= static_cast<size_t>(k);
    }
    return true;
}

/// Read exactly `len` bytes.  False on error or orderly shutdown.
inline bool recv_all(int32_t fd, void* p, size_t len) {
    uint8_t* b = static_cast<uint8_t*>(p);
    while (len) {
        ssize_t k = recv(fd, b, len, MSG_WAITALL);
        if (k < 0 && errno == EINTR) continue;
        if (k <= 0) return false;
        b += k;
        len -= static_cast<size_t>(k);
    }
    return true;
}

/// One frame: u32 big-endian length, then the payload.
inline void send_data(int32_t socket_fd, const uint8_t* data, size_t len) {
    const uint32_t size_network = htonl(static_cast<uint32_t>(len));
    if (!send_all(socket_fd, &size_network, sizeof(size_network))) {
        fprintf(stderr, "srpc::transport::send_data(): failed to send data size.\n");
        return;
    }
    if (len && !send_all(socket_fd, data, len)) {
        fprintf(stderr, "srpc::transport::send_data(): failed to send data payload.\n");
    }
}

/// Receive one frame; an empty message_t on error or end of stream.
[[nodiscard]] inline message_t recv_data(int socket_fd) {
    uint32_t size_network = 0;
    if (!recv_all(socket_fd, &size_network, sizeof(size_network))) return message_t{};
    const uint32_t size = ntohl(size_network);
    message_t m(static_cast<size_t>(size));
    if (size && !recv_all(socket_fd, m.mutable_data(), size)) {
        fprintf(stderr, "srpc::transport::recv_data(): failed to receive data payload.\n");
        return message_t{};
    }
    return m;
}

}  // namespace transport

}  // namespace srpc
