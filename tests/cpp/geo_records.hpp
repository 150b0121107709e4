// geo_records.hpp -- TEST INFRASTRUCTURE ONLY.
//
// Deterministic records of tests/cpp/batchgen_example.contract (Geo service),
// shared by the two sides of the f3 pin:
//   - oracle/ref_shim.cpp fills the reference-style structs (written the way
//     /root/reference/include/srpc/generator.hpp:100-134 emits them) and packs
//     them with the REFERENCE packer -> tests/golden/manifest.json "batchgen"
//     digests (tests/golden/make_golden.py);
//   - tests/cpp/batchgen_gpu_test.cpp fills the structs srpc_amd.batchgen
//     generated, packs them through the generated batch views on the GPU and
//     writes the bytes out for tests/test_batchgen.py to hash.
// Works on any struct with the Record / Point member names.
#pragma once

#include <cstdint>

namespace geo_fixture {

inline uint64_t next(uint64_t& s) {  // splitmix64
    uint64_t z = (s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

constexpr uint64_t kSeed = 0x6E0;
constexpr uint64_t kRecords = 20000;

template <class Rec>
void fill_record(Rec& r, uint64_t& s) {
    r.id = static_cast<int64_t>(next(s));
    r.in.tag = static_cast<int8_t>(next(s));
    r.in.small = static_cast<int16_t>(next(s));
    r.flag = (next(s) & 1) != 0;
    r.label.resize(next(s) % 41);
    for (auto& ch : r.label) ch = static_cast<char>('a' + next(s) % 26);
    r.c = static_cast<char>(next(s));
    r.p.x = static_cast<int32_t>(next(s));
    r.p.y = static_cast<int32_t>(next(s));
    const uint64_t d = next(s);
    r.note.resize(d % 5 == 0 ? (d >> 8) % 300 : 0);
    for (auto& ch : r.note) ch = static_cast<char>(next(s) & 0xff);  // any byte, NUL included
}

template <class Pt>
void fill_point(Pt& p, uint64_t& s) {
    p.x = static_cast<int32_t>(next(s));
    p.y = static_cast<int32_t>(next(s));
}

}  // namespace geo_fixture
