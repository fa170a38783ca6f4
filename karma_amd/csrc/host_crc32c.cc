// karma_amd/csrc/host_crc32c.cc -- the synchronous single-buffer path:
// crc32c::Extend (reference: karma-util/crc32c.h:16, crc32c.cc:275-376).
//
// Karma calls Extend once per record from its io threads (segment_file.cc:22,
// wal.cc:60, frame.cc:56-57).  One record is ~0.2-4 KiB: far below the cost of
// a kernel launch, so this entry point stays on the host and the GPU is
// reached through the batch C ABI (capi.cc).  Two host implementations with
// identical results:
//   * the x86 CRC32 instruction (SSE4.2, same Castagnoli polynomial) -- the
//     path the reference left commented out (crc32c.cc:264-279);
//   * slicing-by-8 tables generated from the polynomial (gf2.h) elsewhere.
#include <cstddef>
#include <cstdint>
#include <cstring>

#include "gf2.h"
#include "karma-util/crc32c.h"
#include "karma_crc32c.h"

#if defined(__x86_64__)
#include <nmmintrin.h>
#endif

namespace {

struct Slice8 {
    uint32_t t[8][256];  // t[k][e] = byte value e advanced by k + 1 bytes
    Slice8() {
        karma::gf2::byte_table(t[0]);
        for (int k = 1; k < 8; ++k)
            for (int e = 0; e < 256; ++e) t[k][e] = (t[k - 1][e] >> 8) ^ t[0][t[k - 1][e] & 0xffu];
    }
};

const Slice8& slice8() {
    static const Slice8 s;
    return s;
}

inline uint32_t load_le32(const uint8_t* p) {
    uint32_t v;
    std::memcpy(&v, p, 4);
#if __BYTE_ORDER__ == __ORDER_BIG_ENDIAN__
    v = __builtin_bswap32(v);
#endif
    return v;
}

uint32_t reg_slice8(uint32_t l, const uint8_t* p, size_t n) {
    const Slice8& s = slice8();
    while (n && (reinterpret_cast<uintptr_t>(p) & 7u)) {
        l = s.t[0][(l ^ *p++) & 0xffu] ^ (l >> 8);
        --n;
    }
    while (n >= 8) {
        const uint32_t lo = load_le32(p) ^ l;
        const uint32_t hi = load_le32(p + 4);
        l = s.t[7][lo & 0xffu] ^ s.t[6][(lo >> 8) & 0xffu] ^ s.t[5][(lo >> 16) & 0xffu] ^ s.t[4][lo >> 24] ^
            s.t[3][hi & 0xffu] ^ s.t[2][(hi >> 8) & 0xffu] ^ s.t[1][(hi >> 16) & 0xffu] ^ s.t[0][hi >> 24];
        p += 8;
        n -= 8;
    }
    while (n--) l = s.t[0][(l ^ *p++) & 0xffu] ^ (l >> 8);
    return l;
}

#if defined(__x86_64__)
__attribute__((target("sse4.2"))) uint32_t reg_sse42(uint32_t l, const uint8_t* p, size_t n) {
    while (n && (reinterpret_cast<uintptr_t>(p) & 7u)) {
        l = _mm_crc32_u8(l, *p++);
        --n;
    }
    uint64_t r = l;
    while (n >= 8) {
        uint64_t w;
        std::memcpy(&w, p, 8);
        r = _mm_crc32_u64(r, w);
        p += 8;
        n -= 8;
    }
    l = static_cast<uint32_t>(r);
    while (n--) l = _mm_crc32_u8(l, *p++);
    return l;
}

bool have_sse42() {
    static const bool yes = __builtin_cpu_supports("sse4.2");
    return yes;
}
#endif

}  // namespace

namespace crc32c {

uint32_t Extend(uint32_t init_crc, const char* data, size_t n) {
    const uint8_t* p = reinterpret_cast<const uint8_t*>(data);
    uint32_t l = ~init_crc;  // pre-conditioning (crc32c.cc:283)
    if (n) {
#if defined(__x86_64__)
        l = have_sse42() ? reg_sse42(l, p, n) : reg_slice8(l, p, n);
#else
        l = reg_slice8(l, p, n);
#endif
    }
    return ~l;  // post-conditioning (crc32c.cc:375)
}

}  // namespace crc32c

namespace karma {
// Exposed for tests: the portable path alone (must equal the SSE4.2 path).
uint32_t host_extend_portable(uint32_t init_crc, const void* data, size_t n) {
    return ~reg_slice8(~init_crc, static_cast<const uint8_t*>(data), n);
}
}  // namespace karma

extern "C" uint32_t karma_crc32c_extend_host(uint32_t init_crc, const void* data, size_t n) {
    return crc32c::Extend(init_crc, static_cast<const char*>(data), n);
}

// crc32c_combine: CRC of A || B from CRC(A), CRC(B) and |B|.  With Z_n = "advance the
// register over n zero bytes" (gf2.h), Value(A || B) = Z_|B|(Value(A)) ^ Value(B); the
// same identity gives Extend(c, D) = Z_|D|(c) ^ Value(D).  This is the algebra the GPU
// combine kernels run with table lookups.
extern "C" uint32_t karma_crc32c_combine(uint32_t crc_a, uint32_t crc_b, uint64_t len_b) {
    return karma::gf2::Map::zero_bytes(len_b).apply(crc_a) ^ crc_b;
}

extern "C" uint32_t karma_crc32c_extend_host_portable(uint32_t init_crc, const void* data, size_t n) {
    return karma::host_extend_portable(init_crc, data, n);
}
