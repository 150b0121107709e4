// echo_records.hpp -- TEST INFRASTRUCTURE ONLY.
//
// Deterministic multiple_primitives requests (the reference packer test's
// message with a string, tests/packer_test.cpp:26-45) for the string-bodied
// e2e pin: an Echo service whose `echo` answers each
// request with every integer + 1 and the string with "!" appended.  Shared by
//   - oracle/ref_shim.cpp ref_server_echo: the REFERENCE server dispatching
//     the requests one by one -> tests/golden/manifest.json "echo_responses"
//     (tests/golden/make_golden.py);
//   - tools/e2e_square.hip --echo: the same requests over 127.0.0.1 to
//     srpc::gpu::batch_server, echo served in GPU batches.
// Works on any struct with the multiple_primitives member names.
#pragma once

#include <cstdint>
#include <string>

namespace echo_fixture {

inline uint64_t next(uint64_t& s) {  // splitmix64
    uint64_t z = (s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

constexpr uint64_t kSeed = 0xEC40;
constexpr const char* kMethod = "Echo_servicer::echo";

/// Request i (any byte value in the string, NUL included; lengths 0..40).
template <class MP>
void fill_request(MP& r, uint64_t i) {
    uint64_t s = kSeed + i * 0xD1B54A32D192ED03ull;
    r.arg1 = static_cast<int8_t>(next(s));
    r.arg2 = static_cast<char>(next(s));
    r.arg3 = static_cast<int64_t>(next(s));
    r.arg4.resize(next(s) % 41);
    uint64_t w = 0;
    for (size_t j = 0; j < r.arg4.size(); ++j) {
        if (j % 8 == 0) w = next(s);
        r.arg4[j] = static_cast<char>(w >> (8 * (j % 8)));
    }
}

/// The service's answer.
template <class MP>
MP answer(MP const& q) {
    MP r;
    r.arg1 = static_cast<int8_t>(static_cast<uint8_t>(q.arg1) + 1u);
    r.arg2 = static_cast<char>(static_cast<uint8_t>(q.arg2) + 1u);
    r.arg3 = static_cast<int64_t>(static_cast<uint64_t>(q.arg3) + 1u);
    r.arg4 = q.arg4 + "!";
    return r;
}

}  // namespace echo_fixture
