// oracle/ref_shim.cc -- TEST INFRASTRUCTURE ONLY.
//
// C entry points around the reference's own crc32c::Extend, compiled from the
// sources where they lie (/root/reference/karma-util/crc32c.cc + coding.cc) by
// oracle/Makefile into oracle/_ref/libkarma_ref_crc32c.so.  Used to generate
// tests/golden/ and as bench.py's cpu_baseline (kind "reference").  No
// reference source is copied into this repository.
#include <cstddef>
#include <cstdint>
#include <thread>
#include <vector>

#include "karma-util/crc32c.h"  // /root/reference/karma-util/crc32c.h:16

extern "C" {

uint32_t ref_crc32c_extend(uint32_t init_crc, const void* data, size_t n) {
    return crc32c::Extend(init_crc, static_cast<const char*>(data), n);
}

// CRC of n_rec fixed-size records laid out back to back in host memory, split
// round-robin over nthreads std::threads (the survey's CPU-baseline shape).
int ref_crc32c_fixed_mt(const void* base, uint64_t rec_bytes, uint64_t n_rec, uint32_t* out, int nthreads) {
    if (nthreads < 1) nthreads = 1;
    const char* b = static_cast<const char*>(base);
    std::vector<std::thread> th;
    for (int t = 0; t < nthreads; ++t)
        th.emplace_back([=] {
            for (uint64_t r = t; r < n_rec; r += nthreads) out[r] = crc32c::Value(b + r * rec_bytes, rec_bytes);
        });
    for (auto& x : th) x.join();
    return 0;
}

// Ragged records: out[r] = Extend(init ? init[r] : 0, base + off[r], len[r]).
int ref_crc32c_ragged_mt(const void* base, const uint64_t* off, const uint32_t* len, const uint32_t* init,
                         uint64_t n_rec, uint32_t* out, int nthreads) {
    if (nthreads < 1) nthreads = 1;
    const char* b = static_cast<const char*>(base);
    std::vector<std::thread> th;
    for (int t = 0; t < nthreads; ++t)
        th.emplace_back([=] {
            for (uint64_t r = t; r < n_rec; r += nthreads)
                out[r] = crc32c::Extend(init ? init[r] : 0u, b + off[r], len[r]);
        });
    for (auto& x : th) x.join();
    return 0;
}

}  // extern "C"
