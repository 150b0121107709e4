// srpc/server.hpp -- blocking sRPC server (MI355X build).
//
// Same API as the reference's include/srpc/server.hpp:
//   server::call(funcname, packer)      (reference server.hpp:17-30)
//   server::register_service(servicer)  (:34-43)
//   server::start(port)                 (:45-74)
//   server::__testable_start(port)      (:76, defined by callers)
// Dispatch: the request frame is `str(method) | str(T::name) | body`; the
// method name selects the handler, which decodes the body with getv<I>(),
// calls the servicer and answers pack_response(RPC_SUCCESS, result).
//
// Fixed here: an unknown method answers the single status byte
// RPC_ERR_FUNCTION_NOT_REGISTERED and returns (the reference then
// dereferences end(), server.hpp:20-26); the decoded argument is freed (the
// reference leaks getv's object, :108); a connection serves requests until
// the peer closes it (the reference closes after one request, :71, which
// breaks a stub's second call on the same channel).
//
// For batches of requests of one method, srpc/gpu_server.hpp decodes and
// encodes whole batches on the GPU with the same frames.
#pragma once

#include <cassert>
#include <cstdio>
#include <functional>
#include <memory>
#include <string>
#include <type_traits>
#include <unordered_map>

#include "core.hpp"
#include "packer.hpp"
#include "transport.hpp"

namespace srpc {

class server {
public:
    server() = default;
    ~server() = default;

    /// Run the handler registered for `funcname` on the request left in `p`
    /// (positioned after the method name); returns the response packer.
    packer::ptr call(std::string const& funcname, packer::ptr p) {
        packer::ptr rp = std::make_shared<packer>();
        auto it = _function_registry.find(funcname);
        if (it == _function_registry.end()) {
            fprintf(stderr, "srpc::server::call(): function %s not registered.\n", funcname.c_str());
            (*rp) << static_cast<uint8_t>(RPC_ERR_FUNCTION_NOT_REGISTERED);
            return rp;
        }
        it->second(rp.get(), p.get());
        return rp;
    }

    template <SrpcService S>
    void register_service(S& service_instance) {
        static_assert(std::tuple_size_v<decltype(S::methods)> > 0, "S::methods is empty!");
        std::apply(
            [this, &service_instance](const auto&... method) {
                (register_method(std::get<MEMBER_NAME>(method), std::get<MEMBER_ADDR>(method), service_instance),
                 ...);
            },
            S::methods);
    }

    /// Serve forever on `port`.
    void start(std::string const&& port) {
        const int32_t listening_fd = transport::create_server_socket(port);
        if (listening_fd < 0) return;
        while (true) {
            sockaddr_storage client_addr{};
            socklen_t addr_size = sizeof(client_addr);
            const int32_t fd = accept(listening_fd, reinterpret_cast<sockaddr*>(&client_addr), &addr_size);
            if (fd < 0) {
                fprintf(stderr, "srpc::server::start(): accept failed.\n");
                continue;
            }
            serve_connection(fd);
            close(fd);
        }
    }

    /// Answer requests on one connected socket until the peer closes it.
    /// Returns the number of requests served.
    size_t serve_connection(int32_t fd) {
        size_t served = 0;
        while (true) {
            message_t msg = transport::recv_data(fd);
            if (msg.data() == nullptr) break;
            packer::ptr p = std::make_shared<packer>(msg.data(), msg.size());
            std::string funcname;
            (*p) >> funcname;
            packer::ptr r = call(funcname, p);
            transport::send_data(fd, r->data(), r->size());
            ++served;
        }
        return served;
    }

    void __testable_start(std::string const&&);

private:
    template <typename F, SrpcService S>
    void register_method(std::string const& name, F func, S& instance) {
        using input_type = typename function_traits<F>::input_type;
        using return_type = typename function_traits<F>::return_type;
        static_assert(std::is_base_of_v<message_base, std::decay_t<input_type>>);
        static_assert(std::is_base_of_v<message_base, std::decay_t<return_type>>);
        S* inst = &instance;
        _function_registry[name] = [this, func, inst](packer* rp, packer* cp) {
            call_proxy_impl(func, *inst, rp, cp);
        };
    }

    template <SrpcMessage R, typename C, SrpcMessage I, SrpcService S>
    void call_proxy_impl(R (C::*func)(I&), S& instance, packer* rp, packer* cp) {
        std::unique_ptr<I> arg(cp->getv<I>());
        if (!arg) {
            (*rp) << static_cast<uint8_t>(RPC_ERR_FUNCTION_NOT_REGISTERED);
            return;
        }
        R result = (instance.*func)(*arg);
        response_t<R> response;
        response.set_code(RPC_SUCCESS);
        response.set_value(result);
        rp->pack_response(response);
    }

    std::unordered_map<std::string, std::function<void(packer*, packer*)>> _function_registry;
};

}  // namespace srpc
