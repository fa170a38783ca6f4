// karma_amd/csrc/gf2.h -- host-side GF(2) algebra of the CRC-32C register.
//
// The CRC register l of karma-util/crc32c.cc (reflected Castagnoli polynomial
// 0x82F63B78; byte step `l = T[(l ^ b) & 0xff] ^ (l >> 8)`, crc32c.cc:286-290)
// evolves linearly over GF(2).  Everything the MI355X engine needs is one
// linear map:
//
//   Z_d(x)  = the register x pushed through d zero bytes.
//
// Z_4(l ^ w) is one 4-byte word step (STEP4 with a 4-byte stride, crc32c.cc:293-299);
// Z_16 is the reference's kStrideExtensionTable (crc32c.cc:64-242); the GPU
// uses Z_S for its stride S = 128 bytes and Z_{D*2^k} to combine partial
// results.  Z_d is represented by its 32 columns and turned
// into four 256-entry "slicing" tables T_k[e] = Z_d(e << 8k) so that
// Z_d(x) = T_0[x&0xff] ^ T_1[(x>>8)&0xff] ^ T_2[(x>>16)&0xff] ^ T_3[x>>24].
#pragma once
#include <cstdint>
#include <cstring>

namespace karma {
namespace gf2 {

constexpr uint32_t kPoly = 0x82F63B78u;  // reflected CRC-32C polynomial

// Z_1 on a full register: one zero byte.
inline uint32_t zero_byte(uint32_t x) {
    uint32_t lo = x & 0xffu;
    for (int k = 0; k < 8; ++k) lo = (lo >> 1) ^ ((lo & 1u) ? kPoly : 0u);
    return lo ^ (x >> 8);
}

struct Map {
    uint32_t col[32];  // col[i] = Z(1 << i)

    uint32_t apply(uint32_t x) const {
        uint32_t r = 0;
        for (int i = 0; i < 32; ++i)
            if (x & (1u << i)) r ^= col[i];
        return r;
    }
    static Map identity() {
        Map m;
        for (int i = 0; i < 32; ++i) m.col[i] = 1u << i;
        return m;
    }
    static Map one_byte() {
        Map m;
        for (int i = 0; i < 32; ++i) m.col[i] = zero_byte(1u << i);
        return m;
    }
    // (a ∘ b)(x) = a(b(x))
    static Map compose(const Map& a, const Map& b) {
        Map m;
        for (int i = 0; i < 32; ++i) m.col[i] = a.apply(b.col[i]);
        return m;
    }
    // The inverse map (Z_d is invertible: the CRC polynomial has a constant term), by
    // Gauss-Jordan elimination on [M | I]: row r holds bit r of every column.
    static Map inverse(const Map& m) {
        uint64_t rows[32];
        for (int r = 0; r < 32; ++r) {
            uint64_t row = 1ull << (32 + r);
            for (int i = 0; i < 32; ++i)
                if ((m.col[i] >> r) & 1u) row |= 1ull << i;
            rows[r] = row;
        }
        for (int c = 0; c < 32; ++c) {
            int piv = c;
            while (piv < 32 && !((rows[piv] >> c) & 1u)) ++piv;
            if (piv == 32) return identity();  // singular: not a CRC shift (never happens)
            const uint64_t t = rows[piv];
            rows[piv] = rows[c];
            rows[c] = t;
            for (int r = 0; r < 32; ++r)
                if (r != c && ((rows[r] >> c) & 1u)) rows[r] ^= rows[c];
        }
        Map inv;
        for (int i = 0; i < 32; ++i) {
            uint32_t col = 0;
            for (int r = 0; r < 32; ++r) col |= (uint32_t)((rows[r] >> (32 + i)) & 1u) << r;
            inv.col[i] = col;
        }
        return inv;
    }
    // Z_d by square-and-multiply over Z_1 (d may be up to 2^63).
    static Map zero_bytes(uint64_t d) {
        Map result = identity();
        Map p = one_byte();
        while (d) {
            if (d & 1u) result = compose(p, result);
            d >>= 1;
            if (d) p = compose(p, p);
        }
        return result;
    }
};

// Four slicing tables (1024 words) of a map: out[k*256 + e] = m(e << 8k).
inline void slicing_tables(const Map& m, uint32_t* out) {
    for (int k = 0; k < 4; ++k)
        for (uint32_t e = 0; e < 256; ++e) out[k * 256 + e] = m.apply(e << (8 * k));
}

// The byte table of the reference (kByteExtensionTable, crc32c.cc:19-62).
inline void byte_table(uint32_t* out) {
    for (uint32_t e = 0; e < 256; ++e) out[e] = zero_byte(e);
}

}  // namespace gf2
}  // namespace karma
