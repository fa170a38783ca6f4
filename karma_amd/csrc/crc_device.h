// karma_amd/csrc/crc_device.h -- device-side building blocks shared by the
// gfx950 kernels (crc_fixed.hip, crc_ragged.hip).
//
// Notation: R(X) is the CRC register of karma-util/crc32c.cc
// after byte X (`l`, crc32c.cc:283), Z_d the linear map "advance the register
// over d zero bytes" (gf2.h).  A 4-byte word step is R <- Z_4(R ^ w)
// (crc32c.cc:293-299 with a 4-byte stride); a byte step is STEP1
// (crc32c.cc:286-290).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#include "bounds.h"
#include "engine.h"

namespace karma {
namespace engine {
namespace dev {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) const u32x4 gu32x4;

// ---- LDS image of the streaming kernels ------------------------------------
// [0, 128 KiB): the Z_S slicing tables, bank-replicated.  Byte address of
//   table k, entry e, for lane L:  (k>>1)<<16 | e<<8 | (k&1)<<7 | (L&31)<<2
// so one v_perm_b32 builds it from the register (entry = byte k) and a
// per-lane constant, and the 32 lanes of each ds_read_b32 half-wave hit 32
// distinct banks (no conflicts on random data).
// [128 KiB, +17 KiB): Z4, Z16, Z32, Z64 slicing tables and the byte table.
// [145 KiB, +12 KiB): Z_U, Z_2U, Z_4U of the batch's unit size U (the cross-group
//   combine of k_units_fixed; loaded only when a wave's 8 units belong to one record).
constexpr int kRepWords = 32768;
constexpr int kSmallBase = kRepWords;
constexpr int kSmallWords = kBlobWords - 1024;
constexpr int kCombLdsBase = kRepWords + kSmallWords;
constexpr int kLdsWords = kRepWords + kSmallWords;       // 148,480 bytes
constexpr int kLdsWordsComb = kLdsWords + 3 * 1024;      // 160,768 bytes
constexpr int kLZ4 = kSmallBase + (kBlobZ4 - 1024);
constexpr int kLZ16 = kSmallBase + (kBlobZ16 - 1024);
constexpr int kLZ32 = kSmallBase + (kBlobZ32 - 1024);
constexpr int kLZ64 = kSmallBase + (kBlobZ64 - 1024);
constexpr int kLT8 = kSmallBase + (kBlobT8 - 1024);


constexpr uint32_t kSel0 = 0x0c0c0004u;  // {X.b0, acc.b0, 0, 0}
constexpr uint32_t kSel1 = 0x0c0c0105u;  // {X.b1, acc.b1, 0, 0}
constexpr uint32_t kSel2 = 0x0c070204u;  // {X.b0, acc.b2, X.b3, 0}
constexpr uint32_t kSel3 = 0x0c070305u;  // {X.b1, acc.b3, X.b3, 0}

// The engine is written for CDNA4 alone: v_bitop3_b32 below (and the LDS sizes) are gfx950's.
#if defined(__HIP_DEVICE_COMPILE__) && !defined(__gfx950__)
#error "karma_amd kernels target gfx950 (MI355X) only: build with --offload-arch=gfx950"
#endif

// a ^ b ^ c in one VALU instruction (gfx950's v_bitop3_b32, truth table 0x96: the parity of the
// three input bits); the compiler does not form it from xor chains by itself.
__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}

__device__ __forceinline__ uint32_t lds_at_byte(const uint32_t* lds, uint32_t byte_addr) {
    return *reinterpret_cast<const uint32_t*>(reinterpret_cast<const uint8_t*>(lds) + byte_addr);
}

// acc <- Z_S(acc) ^ w through the replicated tables (S = kChunk = 128 bytes).
__device__ __forceinline__ uint32_t stride_step(const uint32_t* lds, uint32_t X, uint32_t acc, uint32_t w) {
    const uint32_t i0 = __builtin_amdgcn_perm(X, acc, kSel0);
    const uint32_t i1 = __builtin_amdgcn_perm(X, acc, kSel1);
    const uint32_t i2 = __builtin_amdgcn_perm(X, acc, kSel2);
    const uint32_t i3 = __builtin_amdgcn_perm(X, acc, kSel3);
    return xor3(xor3(lds_at_byte(lds, i0), lds_at_byte(lds, i1), w), lds_at_byte(lds, i2), lds_at_byte(lds, i3));
}

// The half-replicated image (16 copies, 64 KiB; the fused WAL walker, which also needs LDS
// for its walkers' tiles): row e (256 bytes) holds entry e of the four tables, 16 copies
// each: byte address of table k, entry e, for lane L = e<<8 | k<<6 | (L&15)<<2, so one
// v_perm_b32 per table builds it from acc byte k and byte k of the lane constant
// (lane_const16).  Lanes L and L+16 share a bank: random data costs 2-way conflicts.
constexpr int kRep16Words = 16384;
__device__ __forceinline__ uint32_t lane_const16() {
    const uint32_t c = (threadIdx.x & 15u) << 2;
    return c | ((64u + c) << 8) | ((128u + c) << 16) | ((192u + c) << 24);
}
__device__ __forceinline__ uint32_t stride_step16(const uint32_t* lds, uint32_t X, uint32_t acc, uint32_t w) {
    const uint32_t i0 = __builtin_amdgcn_perm(X, acc, 0x0c0c0004u);  // {X.b0, acc.b0, 0, 0}
    const uint32_t i1 = __builtin_amdgcn_perm(X, acc, 0x0c0c0105u);  // {X.b1, acc.b1, 0, 0}
    const uint32_t i2 = __builtin_amdgcn_perm(X, acc, 0x0c0c0206u);  // {X.b2, acc.b2, 0, 0}
    const uint32_t i3 = __builtin_amdgcn_perm(X, acc, 0x0c0c0307u);  // {X.b3, acc.b3, 0, 0}
    return xor3(xor3(lds_at_byte(lds, i0), lds_at_byte(lds, i1), w), lds_at_byte(lds, i2), lds_at_byte(lds, i3));
}

// The same lookups with lanes 16-31 of each 32-lane half taking the tables in the order 1, 0, 3, 2:
// one ds_read_b32 then reads table k in lanes 0-15 and table k ^ 1 in lanes 16-31, whose bank
// columns differ by 16 (k << 6 bytes), so the 16-copy image is read without bank conflicts
// (the four lookups are xored, in any order).
__device__ __forceinline__ uint32_t stride_step16s(const uint32_t* lds, uint32_t X, uint32_t acc, uint32_t w) {
    const bool sw = (threadIdx.x & 16u) != 0;
    const uint32_t s0 = sw ? 0x0c0c0105u : 0x0c0c0004u, s1 = sw ? 0x0c0c0004u : 0x0c0c0105u;
    const uint32_t s2 = sw ? 0x0c0c0307u : 0x0c0c0206u, s3 = sw ? 0x0c0c0206u : 0x0c0c0307u;
    const uint32_t i0 = __builtin_amdgcn_perm(X, acc, s0);
    const uint32_t i1 = __builtin_amdgcn_perm(X, acc, s1);
    const uint32_t i2 = __builtin_amdgcn_perm(X, acc, s2);
    const uint32_t i3 = __builtin_amdgcn_perm(X, acc, s3);
    return xor3(xor3(lds_at_byte(lds, i0), lds_at_byte(lds, i1), w), lds_at_byte(lds, i2), lds_at_byte(lds, i3));
}

// The 8-copy image (32 KiB: entry e, table t, copy c at byte e<<7 | t<<5 | c<<2): lane L reads
// copy L & 7, and the four lane octets of each 32-lane half take the tables in rotated order
// (octet q: t = (i + q) & 3 in lookup i), so each ds_read_b32 touches 32 distinct bank columns
// (t<<3 | c).  The index needs a bit-field extract and a shift-or (the 16- and 32-copy images'
// 256-byte rows take one v_perm_b32), for half the LDS of the 16-copy image.
constexpr int kRep8Words = 8192;
__device__ __forceinline__ uint32_t stride_step8(const uint32_t* lds, uint32_t acc, uint32_t w) {
    const uint32_t q = (threadIdx.x >> 3) & 3u, c4 = (threadIdx.x & 7u) << 2;
    uint32_t l[4];
#pragma unroll
    for (uint32_t i = 0; i < 4; ++i) {
        const uint32_t t = (i + q) & 3u;
        l[i] = lds_at_byte(lds, (__builtin_amdgcn_ubfe(acc, 8u * t, 8u) << 7) | (t << 5) | c4);
    }
    return xor3(xor3(l[0], l[1], w), l[2], l[3]);
}
template <int THREADS>
__device__ __forceinline__ void load_rep8_stride(uint32_t* lds, const uint32_t* __restrict__ blob) {
    constexpr int NV = kRep8Words / 4;  // vector v: words 4v..4v+3 = copies 4(v&1)..+3 of (e, t)
    constexpr int IT = (NV + THREADS - 1) / THREADS;
    u32x4* l4 = reinterpret_cast<u32x4*>(lds);
#pragma unroll
    for (int q = 0; q < IT; ++q) {
        const int v = (int)threadIdx.x + q * THREADS;
        if (v < NV) {
            const int e = v >> 3, t = (v >> 1) & 3;
            const uint32_t x = *(const __attribute__((address_space(1))) uint32_t*)(blob + kBlobStride + t * 256 + e);
            l4[v] = u32x4{x, x, x, x};
        }
    }
}

// Z(x) for a map stored as four plain 256-entry tables at word `base`.
__device__ __forceinline__ uint32_t zmap(const uint32_t* lds, int base, uint32_t x) {
    return xor3(lds[base + (x & 255u)], lds[base + 256 + ((x >> 8) & 255u)], lds[base + 512 + ((x >> 16) & 255u)]) ^
           lds[base + 768 + (x >> 24)];
}

// Lane fold of the four word slots in the reference's STEP4W order
// (crc32c.cc:312-319): Z4(a3 ^ Z4(a2 ^ Z4(a1 ^ Z4(a0)))).  (The expanded form
// Z16(a0)^Z12(a1)^Z8(a2)^Z4(a3), one LDS round trip instead of four, measured
// no faster and costs 8 KiB of LDS: DESIGN.md §4.)
__device__ __forceinline__ uint32_t lane_fold_at(const uint32_t* lds, int z4, uint32_t a0, uint32_t a1, uint32_t a2,
                                                 uint32_t a3) {
    uint32_t c = zmap(lds, z4, a0);
    c = zmap(lds, z4, c ^ a1);
    c = zmap(lds, z4, c ^ a2);
    return zmap(lds, z4, c ^ a3);
}
__device__ __forceinline__ uint32_t lane_fold(const uint32_t* lds, uint32_t a0, uint32_t a1, uint32_t a2,
                                              uint32_t a3) {
    return lane_fold_at(lds, kLZ4, a0, a1, a2, a3);
}

// One data byte (STEP1).
__device__ __forceinline__ uint32_t byte_step(const uint32_t* lds, int t8, uint32_t r, uint32_t b) {
    return lds[t8 + ((r ^ b) & 255u)] ^ (r >> 8);
}

// Record bytes live in device global memory: loads go through address space 1
// so hipcc emits global_load_dwordx4 (vmcnt only) instead of flat loads, whose
// lgkmcnt share would serialise them against the LDS lookups.  NT = the
// non-temporal policy (bytes are read exactly once).
// (The bounds build checks every record-byte load against the kernel's arena: bounds.h.)
template <bool NT>
__device__ __forceinline__ u32x4 ldg(const uint8_t* p) {
    p = KB_BYTES(p, 16);
    if constexpr (NT) return __builtin_nontemporal_load((gu32x4*)(p));
    return *(gu32x4*)(p);
}
__device__ __forceinline__ u32x4 ld16(const uint8_t* p) { return *(gu32x4*)(KB_BYTES(p, 16)); }
// 16 bytes of library metadata (unit descriptors): not record bytes, never checked.
__device__ __forceinline__ u32x4 ldmeta16(const void* p) { return *(gu32x4*)(p); }

__device__ __forceinline__ const uint8_t* pmin(const uint8_t* a, const uint8_t* b) { return a < b ? a : b; }
__device__ __forceinline__ const uint8_t* pmax(const uint8_t* a, const uint8_t* b) { return a > b ? a : b; }
__device__ __forceinline__ const uint8_t* floor16(const uint8_t* p) {
    return reinterpret_cast<const uint8_t*>(reinterpret_cast<uintptr_t>(p) & ~uintptr_t(15));
}
__device__ __forceinline__ const uint8_t* ceil16(const uint8_t* p) {
    return reinterpret_cast<const uint8_t*>((reinterpret_cast<uintptr_t>(p) + 15) & ~uintptr_t(15));
}

// Register after bytes [from, to) of an aligned 16-byte block already loaded
// into v (0 <= from <= to <= 16): whole aligned words through Z4 (one LDS
// round trip per word), the rest byte by byte.
__device__ __forceinline__ uint32_t steps_in_vec(const uint32_t* lds, int z4, int t8, uint32_t r, const u32x4& v,
                                                 uint32_t from, uint32_t to) {
    if (from >= to) return r;
    // 128-bit shift register of the block, consumed from byte 0 upwards
    uint64_t lo = v.x | ((uint64_t)v.y << 32), hi = v.z | ((uint64_t)v.w << 32);
    uint32_t i = 0;
    for (; i < to; ++i) {  // leading bytes until `from` is reached and 4-aligned
        if (i >= from && (i & 3u) == 0 && i + 4 <= to) break;
        if (i >= from) r = byte_step(lds, t8, r, (uint32_t)lo & 255u);
        lo = (lo >> 8) | (hi << 56);
        hi >>= 8;
    }
    for (; i + 4 <= to; i += 4) {  // whole words
        r = zmap(lds, z4, r ^ (uint32_t)lo);
        lo = (lo >> 32) | (hi << 32);
        hi >>= 32;
    }
    for (; i < to; ++i) {  // trailing bytes
        r = byte_step(lds, t8, r, (uint32_t)lo & 255u);
        lo = (lo >> 8) | (hi << 56);
        hi >>= 8;
    }
    return r;
}

// The same for the block at `blk`, loaded here.
__device__ __forceinline__ uint32_t steps_in_block(const uint32_t* lds, int z4, int t8, uint32_t r, const uint8_t* blk,
                                                   uint32_t from, uint32_t to) {
    if (from >= to) return r;
    return steps_in_vec(lds, z4, t8, r, ld16(blk), from, to);
}

// A whole record step by step (records with no aligned 16-byte block inside).
__device__ __forceinline__ uint32_t short_record(const uint32_t* lds, int z4, int t8, const uint8_t* p, uint64_t n,
                                                 uint32_t init) {
    uint32_t r = ~init;
    const uint8_t* e = p + n;
    const uint8_t* q = p;
    while (q < e) {
        const uint8_t* blk = floor16(q);
        const uint32_t to = (uint32_t)((e - blk) < 16 ? (e - blk) : 16);
        r = steps_in_block(lds, z4, t8, r, blk, (uint32_t)(q - blk), to);
        q = blk + 16;
    }
    return ~r;
}

struct Geom {
    const uint8_t* a;  // first aligned body byte
    const uint8_t* b;  // end of the aligned body
    const uint8_t* e;  // record end
    bool is_short;     // no aligned 16-byte block inside (includes n == 0)
};

__device__ __forceinline__ Geom geom(const uint8_t* p, uint64_t n) {
    Geom g;
    g.e = p + n;
    g.a = ceil16(p);
    g.b = floor16(g.e);
    g.is_short = (g.b - g.a) < 16;
    return g;
}

// Register entering the body: ~init advanced over the unaligned head [p, a).
__device__ __forceinline__ uint32_t head_register(const uint32_t* lds, int z4, int t8, const uint8_t* p, const Geom& g,
                                                  uint32_t init) {
    uint32_t h = ~init;
    if (p < g.a) h = steps_in_block(lds, z4, t8, h, g.a - 16, (uint32_t)(p - (g.a - 16)), 16u);
    return h;
}

// Register after the unaligned tail [b, e) given the register at b.
__device__ __forceinline__ uint32_t tail_register(const uint32_t* lds, int z4, int t8, uint32_t r, const Geom& g) {
    if (g.e > g.b) r = steps_in_block(lds, z4, t8, r, g.b, 0u, (uint32_t)(g.e - g.b));
    return r;
}

// MODE (timing experiments of the tools build only, wrong results): bit 0 = main-loop
// steps without the LDS lookups (KARMA_CRC_VARIANT=6, ab.h), bit 1 = stream_unit without
// the lane fold and group tree.  The shipped library instantiates MODE 0 only.
// MODE bit 3: the 16-copy stride image (stride_step16, lane_const16).
// MODE bit 4 (with bit 3): the conflict-free lane order of the 16-copy image (stride_step16s).
template <int MODE = 0>
__device__ __forceinline__ void step4(const uint32_t* lds, uint32_t X, uint32_t& a0, uint32_t& a1, uint32_t& a2,
                                      uint32_t& a3, const u32x4& v) {
    if constexpr ((MODE & 32) != 0) {  // the 8-copy image (stride_step8)
        a0 = stride_step8(lds, a0, v.x);
        a1 = stride_step8(lds, a1, v.y);
        a2 = stride_step8(lds, a2, v.z);
        a3 = stride_step8(lds, a3, v.w);
        return;
    }
    if constexpr ((MODE & 88) == 88) {
        // MODE bit 6 (with bits 3-4): phased, every lookup of the window in flight together -- the 16
        // indices, the 16 reads, the xors, kept apart by scheduling barriers (lane_record_end's note)
        const bool swp = (threadIdx.x & 16u) != 0;
        const uint32_t s0 = swp ? 0x0c0c0105u : 0x0c0c0004u, s1 = swp ? 0x0c0c0004u : 0x0c0c0105u;
        const uint32_t s2 = swp ? 0x0c0c0307u : 0x0c0c0206u, s3 = swp ? 0x0c0c0206u : 0x0c0c0307u;
        const uint32_t acc[4] = {a0, a1, a2, a3};
        uint32_t ix[16], l[16];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            ix[4 * k] = __builtin_amdgcn_perm(X, acc[k], s0);
            ix[4 * k + 1] = __builtin_amdgcn_perm(X, acc[k], s1);
            ix[4 * k + 2] = __builtin_amdgcn_perm(X, acc[k], s2);
            ix[4 * k + 3] = __builtin_amdgcn_perm(X, acc[k], s3);
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int k = 0; k < 16; ++k) l[k] = lds_at_byte(lds, ix[k]);
        __builtin_amdgcn_sched_barrier(0);
        a0 = xor3(xor3(l[0], l[1], v.x), l[2], l[3]);
        a1 = xor3(xor3(l[4], l[5], v.y), l[6], l[7]);
        a2 = xor3(xor3(l[8], l[9], v.z), l[10], l[11]);
        a3 = xor3(xor3(l[12], l[13], v.w), l[14], l[15]);
        return;
    }
    if constexpr ((MODE & 88) == 64) {  // the same phasing on the 32-copy image (stride_step)
        const uint32_t acc[4] = {a0, a1, a2, a3};
        uint32_t ix[16], l[16];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            ix[4 * k] = __builtin_amdgcn_perm(X, acc[k], kSel0);
            ix[4 * k + 1] = __builtin_amdgcn_perm(X, acc[k], kSel1);
            ix[4 * k + 2] = __builtin_amdgcn_perm(X, acc[k], kSel2);
            ix[4 * k + 3] = __builtin_amdgcn_perm(X, acc[k], kSel3);
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int k = 0; k < 16; ++k) l[k] = lds_at_byte(lds, ix[k]);
        __builtin_amdgcn_sched_barrier(0);
        a0 = xor3(xor3(l[0], l[1], v.x), l[2], l[3]);
        a1 = xor3(xor3(l[4], l[5], v.y), l[6], l[7]);
        a2 = xor3(xor3(l[8], l[9], v.z), l[10], l[11]);
        a3 = xor3(xor3(l[12], l[13], v.w), l[14], l[15]);
        return;
    }
    if constexpr ((MODE & 24) == 24) {
        a0 = stride_step16s(lds, X, a0, v.x);
        a1 = stride_step16s(lds, X, a1, v.y);
        a2 = stride_step16s(lds, X, a2, v.z);
        a3 = stride_step16s(lds, X, a3, v.w);
        return;
    }
    if constexpr (MODE & 8) {
        a0 = stride_step16(lds, X, a0, v.x);
        a1 = stride_step16(lds, X, a1, v.y);
        a2 = stride_step16(lds, X, a2, v.z);
        a3 = stride_step16(lds, X, a3, v.w);
        return;
    }
    if constexpr (MODE & 1) {
        a0 = ((a0 << 1) | (a0 >> 31)) ^ v.x;
        a1 = ((a1 << 1) | (a1 >> 31)) ^ v.y;
        a2 = ((a2 << 1) | (a2 >> 31)) ^ v.z;
        a3 = ((a3 << 1) | (a3 >> 31)) ^ v.w;
        return;
    }
    a0 = stride_step(lds, X, a0, v.x);
    a1 = stride_step(lds, X, a1, v.y);
    a2 = stride_step(lds, X, a2, v.z);
    a3 = stride_step(lds, X, a3, v.w);
}

__device__ __forceinline__ const uint8_t* floor128(const uint8_t* p) {
    return reinterpret_cast<const uint8_t*>(reinterpret_cast<uintptr_t>(p) & ~uintptr_t(kChunk - 1));
}
// The chunk of a group of G lanes: 16 G bytes on the absolute 16 G-byte grid.
template <int G>
__device__ __forceinline__ const uint8_t* floor_chunk(const uint8_t* p) {
    return reinterpret_cast<const uint8_t*>(reinterpret_cast<uintptr_t>(p) & ~uintptr_t(16 * G - 1));
}

// A 16-byte window with bytes [0, h) zeroed (h < 16), with its last t bytes zeroed (t < 16), and
// with x xored into word k: the edges of a ragged record stepped over its whole 16-byte blocks.
__device__ __forceinline__ u32x4 mask_head(const u32x4& v, uint32_t h) {
    auto m = [&](uint32_t k) {
        const int r = (int)h - 4 * (int)k;
        return r <= 0 ? ~0u : r >= 4 ? 0u : (~0u << (8 * r));
    };
    return u32x4{v.x & m(0), v.y & m(1), v.z & m(2), v.w & m(3)};
}
__device__ __forceinline__ u32x4 mask_tail(const u32x4& v, uint32_t t) {
    auto m = [&](uint32_t k) {
        const int r = 16 - (int)t - 4 * (int)k;  // bytes of word k that stay
        return r >= 4 ? ~0u : r <= 0 ? 0u : (~0u >> (8 * (4 - r)));
    };
    return u32x4{v.x & m(0), v.y & m(1), v.z & m(2), v.w & m(3)};
}
__device__ __forceinline__ u32x4 xor_word(const u32x4& v, uint32_t k, uint32_t x) {
    return u32x4{v.x ^ (k == 0 ? x : 0u), v.y ^ (k == 1 ? x : 0u), v.z ^ (k == 2 ? x : 0u), v.w ^ (k == 3 ? x : 0u)};
}

// Register contribution of the 16-aligned span [us, ue).  The span is read in
// 128-byte chunks on the ABSOLUTE 128-byte grid (every group load is one whole
// cache line, whatever the span's alignment), 8 lanes per group, lane l owning
// bytes [16l, 16l+16) of each chunk as four word slots.  Windows before us are
// zero (a zero prefix does not change the register); in the last chunk the
// lanes past ue skip their step, so lane l's pending words end at a different
// distance from ue: with m the lane holding the last window, lane l's end lies
// 16*((m - l) mod 8) bytes before ue, and the group tree runs over the lanes
// rotated by m + 1.  `inj` is xored into the word at `inj_at` (the body's first
// word carries the record's entering register).  EDGES (the ragged units): the window at us
// has its first `head` bytes zeroed and inj xored into its word head / 4, the window ending at
// ue its last `tail` bytes zeroed (inj_at unused).  PF chunk loads stay in flight
// per lane.  MODE: step4's and stream_unit's timing forms (tools build only, wrong results).
// Every lane of the wave must call this (cross-lane shuffles); the result is valid in group lane 0.
template <int PF, bool NT, bool EDGES = false, int MODE = 0>
__device__ __forceinline__ uint32_t group_unit(const uint32_t* lds, uint32_t X, uint32_t l, const uint8_t* us,
                                               const uint8_t* ue, const uint8_t* inj_at, uint32_t inj,
                                               uint32_t head = 0, uint32_t tail = 0) {
    uint32_t a0 = 0, a1 = 0, a2 = 0, a3 = 0;
    uint32_t m = kGroupLanes - 1;
    if (ue > us) {
        const uint8_t* base = floor128(us);
        const int64_t nch = (ue - base + kChunk - 1) / kChunk;
        m = (uint32_t)((reinterpret_cast<uintptr_t>(ue) - 16) >> 4) & (kGroupLanes - 1);
        const uint8_t* w = base + 16 * l;
        const uint8_t* wl = base + (nch - 1) * kChunk + 16 * l;  // this lane's window in the last chunk
        const bool lok = wl < ue;
        const uint8_t* lclamp = lok ? wl : ue - 16;               // always a valid address
        // (Chunk 0 under a branch, its injected word xored before the PF loads are issued: the
        // compiler then waits for chunk 0 before issuing them.  Issuing all PF + 1 loads together
        // (clamped, masked after) measured 0.7-1.2 % SLOWER on every ragged layout, and so did the
        // kernel pipelined across units: profiles/r05_ragged_group_unit_pipe_ab.txt, DESIGN.md §4.
        // Rechecked with a scheduling barrier after the PF loads, so that the ISA really has all
        // seven chunk loads in flight before the first wait: still 0.5-0.8 % slower,
        // profiles/r05_gue.txt.)
        {
            const bool ok = w >= us && w < ue;
            u32x4 v = ok ? ldg<NT>(w) : u32x4{0u, 0u, 0u, 0u};
            if constexpr (EDGES) {
                if (w == ue - 16) v = mask_tail(v, tail);  // (a one-chunk unit's last window)
                if (w == us) v = xor_word(mask_head(v, head), head >> 2, inj);
            } else {
                if (w == inj_at) v.x ^= inj;
            }
            a0 = v.x;
            a1 = v.y;
            a2 = v.z;
            a3 = v.w;
        }
        int64_t rem = nch - 1;  // chunks after chunk 0; the final one is masked per lane
        w += kChunk;
        u32x4 nb[PF];
#pragma unroll
        for (int q = 0; q < PF; ++q) nb[q] = ldg<NT>(pmin(w + q * kChunk, lclamp));
        while (rem > PF) {  // PF full chunks (at least one more follows)
            u32x4 cur[PF];
#pragma unroll
            for (int q = 0; q < PF; ++q) cur[q] = nb[q];
            w += PF * kChunk;
#pragma unroll
            for (int q = 0; q < PF; ++q) nb[q] = ldg<NT>(pmin(w + q * kChunk, lclamp));
#pragma unroll
            for (int q = 0; q < PF; ++q) step4<MODE>(lds, X, a0, a1, a2, a3, cur[q]);
            rem -= PF;
        }
#pragma unroll
        for (int q = 0; q < PF; ++q) {
            if constexpr (EDGES) {
                if (q == rem - 1 && l == m) nb[q] = mask_tail(nb[q], tail);  // the unit's last window
            }
            if (q < rem - 1 || (q == rem - 1 && lok)) step4<MODE>(lds, X, a0, a1, a2, a3, nb[q]);
        }
    }
    if constexpr ((MODE & 2) != 0) return a0 ^ a1 ^ a2 ^ a3;  // timing build only: no fold, no tree
    uint32_t c = lane_fold(lds, a0, a1, a2, a3);
    // rotate so the lane holding the last window comes last (identity when m == 7)
    const uint32_t lane = threadIdx.x & 63u;
    c = __shfl(c, (int)((lane & ~(kGroupLanes - 1u)) | ((l + m + 1) & (kGroupLanes - 1))), 64);
    // group tree over 8 lanes: v_t = Z_{16*2^d}(v_t) ^ v_{t+2^d}
    uint32_t t = __shfl_down(c, 1, kGroupLanes);
    c = zmap(lds, kLZ16, c) ^ t;
    t = __shfl_down(c, 2, kGroupLanes);
    c = zmap(lds, kLZ32, c) ^ t;
    t = __shfl_down(c, 4, kGroupLanes);
    c = zmap(lds, kLZ64, c) ^ t;
    return c;
}

// ---- one unit as seen by one lane of its group
struct LaneUnit {
    const uint8_t* us;      // unit span [us, ue)
    const uint8_t* ue;
    const uint8_t* w;       // this lane's window in chunk 0
    const uint8_t* lclamp;  // last address this lane may prefetch
    int64_t nch;            // 128-byte chunks on the absolute grid (0: empty unit)
    uint32_t m;             // lane holding the unit's last window
    bool lok;               // this lane's window in the last chunk lies inside the unit
};

// G lanes per group (8 for the streaming kernels; 4 for the small-record kernel), a chunk
// of 16 G bytes.
template <int G = kGroupLanes>
__device__ __forceinline__ LaneUnit lane_unit(const uint8_t* us, const uint8_t* ue, uint32_t l) {
    constexpr int64_t C = 16 * G;
    LaneUnit L;
    L.us = us;
    L.ue = ue;
    L.nch = 0;
    L.m = G - 1;
    L.lok = false;
    L.w = us;
    L.lclamp = us;
    if (ue > us) {
        const uint8_t* base = floor_chunk<G>(us);
        L.nch = (ue - base + C - 1) / C;
        L.m = (uint32_t)((reinterpret_cast<uintptr_t>(ue) - 16) >> 4) & (G - 1);
        L.w = base + 16 * l;
        const uint8_t* wl = base + (L.nch - 1) * C + 16 * l;
        L.lok = wl < ue;
        L.lclamp = L.lok ? wl : ue - 16;
    }
    return L;
}

// ---- software-pipelined unit stream ----------------------------------------
// The loads a lane has in flight for one unit: its chunk-0 window and chunks
// 1..PF (clamped to its last valid window).  Every address is valid whatever
// the unit (empty and out-of-range units point at a safe 16-byte block), so
// the loads are issued without branches and their results are first used one
// unit later: the compiler never has to wait for a just-issued load
// (s_waitcnt vmcnt(0)), and a group's load stream has no gap at unit
// boundaries.
template <int PF>
struct UnitLoads {
    u32x4 v0;
    u32x4 nb[PF];
};

template <int PF, bool NT, int G = kGroupLanes>
__device__ __forceinline__ void issue_unit_loads(const LaneUnit& L, UnitLoads<PF>& Ld) {
    const bool ok0 = L.nch > 0 && L.w >= L.us && L.w < L.ue;
    Ld.v0 = ldg<NT>(ok0 ? L.w : L.lclamp);
#pragma unroll
    for (int q = 0; q < PF; ++q) Ld.nb[q] = ldg<NT>(pmin(L.w + (q + 1) * 16 * G, L.lclamp));
}

// Streams unit L whose first loads are in Ld; `issue_next(Ld)` is called once,
// before the unit's last PF chunks are consumed, to put the next unit's first
// loads in flight.  `inj` is xored into the word at `inj_at` (nullptr: none).
// One batch of PF chunks is in flight while the previous one is stepped (a
// two-bank ring that never runs dry measured no faster: DESIGN.md §4).
// Every lane of the wave must call this (cross-lane shuffles); the result is
// valid in group lane 0.
// (G < 8: the LDS image's stride tables must be Z_{16 G}, and the tree takes log2 G levels.)
// EDGES (the ragged units): as group_unit's, the window at L.us has its first `head` bytes zeroed
// and inj xored into its word head / 4, the window ending at L.ue its last `tail` bytes zeroed
// (inj_at unused).
template <int PF, bool NT, int MODE = 0, int G = kGroupLanes, bool EDGES = false, typename IssueNext>
__device__ __forceinline__ uint32_t stream_unit(const uint32_t* lds, uint32_t X, uint32_t l, const LaneUnit& L,
                                                UnitLoads<PF>& Ld, const uint8_t* inj_at, uint32_t inj,
                                                IssueNext&& issue_next, uint32_t head = 0, uint32_t tail = 0) {
    static_assert(G == 8 || G == 4 || G == 2, "groups of 8, 4 or 2 lanes");
    constexpr int C = 16 * G;
    const bool ok0 = L.nch > 0 && L.w >= L.us && L.w < L.ue;
    u32x4 v = ok0 ? Ld.v0 : u32x4{0u, 0u, 0u, 0u};
    if constexpr (EDGES) {
        if (ok0 && L.w == L.ue - 16) v = mask_tail(v, tail);  // (a one-chunk unit's last window)
        if (ok0 && L.w == L.us) v = xor_word(mask_head(v, head), head >> 2, inj);
    } else {
        if (ok0 && L.w == inj_at) v.x ^= inj;
    }
    uint32_t a0 = v.x, a1 = v.y, a2 = v.z, a3 = v.w;
    int64_t rem = L.nch - 1;  // chunks after chunk 0; the final one is masked per lane
    const uint8_t* w = L.w + C;
    while (rem > PF) {
        u32x4 cur[PF];
#pragma unroll
        for (int q = 0; q < PF; ++q) cur[q] = Ld.nb[q];
        w += PF * C;
#pragma unroll
        for (int q = 0; q < PF; ++q) Ld.nb[q] = ldg<NT>(pmin(w + q * C, L.lclamp));
#pragma unroll
        for (int q = 0; q < PF; ++q) step4<MODE>(lds, X, a0, a1, a2, a3, cur[q]);
        rem -= PF;
    }
    constexpr int D = PF;
    u32x4 cur[D];
#pragma unroll
    for (int q = 0; q < D; ++q) cur[q] = Ld.nb[q];
    issue_next(Ld);
#pragma unroll
    for (int q = 0; q < D; ++q) {
        if constexpr (EDGES) {
            if (q == rem - 1 && l == L.m) cur[q] = mask_tail(cur[q], tail);  // the unit's last window
        }
        if (q < rem - 1 || (q == rem - 1 && L.lok)) step4<MODE>(lds, X, a0, a1, a2, a3, cur[q]);
    }
    // lane fold (crc32c.cc STEP4W order), then the 8-lane tree with the lane
    // holding the unit's last window rotated to the end
    if constexpr ((MODE & 2) != 0) return a0 ^ a1 ^ a2 ^ a3;  // timing build only: no fold, no tree
    uint32_t c = lane_fold(lds, a0, a1, a2, a3);
    const uint32_t lane = threadIdx.x & 63u;
    c = __shfl(c, (int)((lane & ~(G - 1u)) | ((l + L.m + 1) & (G - 1))), 64);
    uint32_t t = __shfl_down(c, 1, G);
    c = zmap(lds, kLZ16, c) ^ t;
    if constexpr (G >= 4) {
        t = __shfl_down(c, 2, G);
        c = zmap(lds, kLZ32, c) ^ t;
    }
    if constexpr (G == 8) {
        t = __shfl_down(c, 4, G);
        c = zmap(lds, kLZ64, c) ^ t;
    }
    return c;
}

// One batch of up to 64 small records, one per lane (this lane's record: pi, ni bytes, init
// initi, vi = a real record), checksummed by groups of G lanes: the small-record kernel's body
// (k_ragged_direct4; also the fused WAL walker's list pass, wal_device.hip).  The head and tail
// byte steps run for the 64 records at once (lane i: record i, serial steps with per-record
// trip counts); the bodies stream in 64 / (64 / G) rounds of 64 / G groups, registers passed in
// and out by shuffles, each round's loads issued before the previous round's last chunks are
// stepped (stream_unit).  A group with no body in a round streams an empty unit at `safe`
// (16-byte aligned, always mapped): every load is issued unconditionally.  Returns this
// lane's CRC (valid when vi); every lane of the wave must call it.
// ALL: every round's first 1 + PF chunk loads are issued at once, before the head steps
// (records of up to 16 G (1 + PF) bytes then wait on memory once per batch instead of once per
// round; longer ones stream the rest within their round).
template <int G, int PF, bool NT, int MODE, bool ALL = false>
__device__ __forceinline__ uint32_t direct_batch(const uint32_t* lds, uint32_t X, const uint8_t* safe,
                                                 const uint8_t* pi, uint32_t ni, uint32_t initi, bool vi) {
    constexpr int NG = 64 / G, NR = 64 / NG;  // groups per wave, rounds
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t l = lane & (G - 1);
    const uint32_t grp = lane / G;
    const Geom gi = geom(pi, ni);
    const bool body = vi && !gi.is_short;
    const uint64_t ai = reinterpret_cast<uintptr_t>(body ? gi.a : safe);
    const uint64_t bi = reinterpret_cast<uintptr_t>(body ? gi.b : safe);
    auto unit_of = [&](uint32_t r) {  // round r's record of this group: NG r + grp
        const int src = (int)(r * NG + grp);
        const uint8_t* us = reinterpret_cast<const uint8_t*>((uintptr_t)__shfl((long long)ai, src));
        const uint8_t* ue = reinterpret_cast<const uint8_t*>((uintptr_t)__shfl((long long)bi, src));
        return lane_unit<G>(us, ue, l);
    };
    uint32_t Ri = 0;
    if constexpr (ALL) {
        UnitLoads<PF> Ld[NR];
#pragma unroll
        for (int r = 0; r < NR; ++r) issue_unit_loads<PF, NT, G>(unit_of(r), Ld[r]);
        const bool tail = body && gi.e > gi.b;
        const u32x4 tv = ld16(tail ? gi.b : safe);
        const uint32_t hi = body ? ((MODE & 4) ? initi : head_register(lds, kLZ4, kLT8, pi, gi, initi)) : 0u;
#pragma unroll
        for (int r = 0; r < NR; ++r) {
            const uint32_t sh = __shfl(hi, (int)(r * NG + grp));
            const LaneUnit L = unit_of(r);
            const uint32_t R = stream_unit<PF, NT, MODE, G>(lds, X, l, L, Ld[r], L.us, sh, [](UnitLoads<PF>&) {});
            const uint32_t Rr = __shfl(R, (int)((lane % NG) * G));  // group (lane % NG)'s register
            if (lane / NG == (uint32_t)r) Ri = Rr;
        }
        if (!vi) return 0u;
        return gi.is_short ? short_record(lds, kLZ4, kLT8, pi, ni, initi)
               : (MODE & 4) ? Ri ^ tv.x
                            : ~steps_in_vec(lds, kLZ4, kLT8, Ri, tv, 0u, tail ? (uint32_t)(gi.e - gi.b) : 0u);
    }
    LaneUnit L = unit_of(0);
    UnitLoads<PF> Ld;
    issue_unit_loads<PF, NT, G>(L, Ld);
    const bool tail = body && gi.e > gi.b;
    const u32x4 tv = ld16(tail ? gi.b : safe);
    const uint32_t hi = body ? ((MODE & 4) ? initi : head_register(lds, kLZ4, kLT8, pi, gi, initi)) : 0u;
#pragma unroll 1
    for (uint32_t round = 0; round < NR; ++round) {
        const uint32_t sh = __shfl(hi, (int)(round * NG + grp));
        LaneUnit N = L;
        const uint32_t R = stream_unit<PF, NT, MODE, G>(lds, X, l, L, Ld, L.us, sh, [&](UnitLoads<PF>& nx) {
            if (round + 1 < NR) {
                N = unit_of(round + 1);
                issue_unit_loads<PF, NT, G>(N, nx);
            }
        });
        const uint32_t Rr = __shfl(R, (int)((lane % NG) * G));  // group (lane % NG)'s register
        if (lane / NG == round) Ri = Rr;
        L = N;
    }
    if (!vi) return 0u;
    return gi.is_short ? short_record(lds, kLZ4, kLT8, pi, ni, initi)
           : (MODE & 4) ? Ri ^ tv.x
                        : ~steps_in_vec(lds, kLZ4, kLT8, Ri, tv, 0u, tail ? (uint32_t)(gi.e - gi.b) : 0u);
}

// Copy WORDS words (WORDS % 4 == 0, both pointers 16-byte aligned) from global
// memory into LDS with THREADS threads: every thread issues all of its 16-byte
// loads before its first LDS store, so the copy costs about one memory latency
// instead of one per loop trip.
template <int WORDS, int THREADS>
__device__ __forceinline__ void copy_to_lds(uint32_t* lds, const uint32_t* __restrict__ g) {
    static_assert(WORDS % 4 == 0, "whole 16-byte vectors");
    constexpr int N4 = WORDS / 4;
    constexpr int IT = (N4 + THREADS - 1) / THREADS;
    const u32x4* g4 = reinterpret_cast<const u32x4*>(g);
    u32x4* l4 = reinterpret_cast<u32x4*>(lds);
    u32x4 v[IT];
#pragma unroll
    for (int q = 0; q < IT; ++q) {
        const int i = (int)threadIdx.x + q * THREADS;
        if (i < N4) v[q] = *(const gu32x4*)(g4 + i);
    }
#pragma unroll
    for (int q = 0; q < IT; ++q) {
        const int i = (int)threadIdx.x + q * THREADS;
        if (i < N4) l4[i] = v[q];
    }
}

template <int WORDS, int THREADS>
struct LdsCopy {  // a global -> LDS copy split in two: the loads, then (after other loads) the stores
    static constexpr int N4 = WORDS / 4, IT = (N4 + THREADS - 1) / THREADS;
    u32x4 v[IT];
    __device__ __forceinline__ void load(const uint32_t* __restrict__ g) {
#pragma unroll
        for (int q = 0; q < IT; ++q) {  // (clamped, not branched: a load under a branch is waited for at the join)
            const int i = (int)threadIdx.x + q * THREADS;
            v[q] = *(const gu32x4*)(reinterpret_cast<const u32x4*>(g) + (i < N4 ? i : N4 - 1));
        }
    }
    __device__ __forceinline__ void store(uint32_t* lds) const {
#pragma unroll
        for (int q = 0; q < IT; ++q) {
            const int i = (int)threadIdx.x + q * THREADS;
            if (i < N4) reinterpret_cast<u32x4*>(lds)[i] = v[q];
        }
    }
};

// The streaming kernels' LDS image (kBlockThreads threads).
__device__ __forceinline__ void load_stream_tables(uint32_t* lds, const uint32_t* __restrict__ blob) {
    static_assert(kSmallWords % 4 == 0 && (kRepWords / 4) % kBlockThreads == 0, "table copy shape");
    // word index = region*16384 + row*64 + half*32 + lane32; table k = region*2 + half.
    // Each 16-byte LDS vector holds 4 copies of one entry; a thread's entries
    // are blob words 0..1023 (the 4 Z_S tables), read once each.
    constexpr int IT = kRepWords / 4 / kBlockThreads;
    uint32_t e[IT];
#pragma unroll
    for (int q = 0; q < IT; ++q) {
        const int idx = ((int)threadIdx.x + q * kBlockThreads) * 4;
        const int region = idx >> 14, row = (idx >> 6) & 255, half = (idx >> 5) & 1;
        e[q] = *(const __attribute__((address_space(1))) uint32_t*)(blob + kBlobStride + (region * 2 + half) * 256 + row);
    }
    copy_to_lds<kSmallWords, kBlockThreads>(lds + kSmallBase, blob + 1024);
    u32x4* l4 = reinterpret_cast<u32x4*>(lds);
#pragma unroll
    for (int q = 0; q < IT; ++q) l4[(int)threadIdx.x + q * kBlockThreads] = u32x4{e[q], e[q], e[q], e[q]};
}

// The 16-copy image of a blob's stride tables for THREADS threads, [0, kRep16Words)
// (stride_step16, lane_const16); `between` runs after the table loads are issued and
// before they are stored (the caller's other copies overlap them).
template <int THREADS, typename Between>
__device__ __forceinline__ void load_rep16_stride(uint32_t* lds, const uint32_t* __restrict__ blob, Between&& between) {
    // vector v of row e: table k = (v >> 2) & 3, copies 4 (v & 3) .. +3
    constexpr int NV = kRep16Words / 4;
    constexpr int IT = (NV + THREADS - 1) / THREADS;
    uint32_t e[IT];
#pragma unroll
    for (int q = 0; q < IT; ++q) {
        const int v = (int)threadIdx.x + q * THREADS;
        const int row = v >> 4, k = (v >> 2) & 3;
        e[q] = v < NV ? *(const __attribute__((address_space(1))) uint32_t*)(blob + kBlobStride + k * 256 + row) : 0u;
    }
    between();
    u32x4* l4 = reinterpret_cast<u32x4*>(lds);
#pragma unroll
    for (int q = 0; q < IT; ++q) {
        const int v = (int)threadIdx.x + q * THREADS;
        if (v < NV) l4[v] = u32x4{e[q], e[q], e[q], e[q]};
    }
}

// The 16-copy image of a stream / quad blob for THREADS threads: [0, kRep16Words) the
// stride tables (stride_step16, lane_const16), the small tables at kSmallBase as in load_stream_tables.
template <int THREADS>
__device__ __forceinline__ void load_stream_tables16(uint32_t* lds, const uint32_t* __restrict__ blob) {
    load_rep16_stride<THREADS>(lds, blob, [&] { copy_to_lds<kSmallWords, THREADS>(lds + kSmallBase, blob + 1024); });
}

// Per-lane constant of the replicated-table address (see the LDS image above).
__device__ __forceinline__ uint32_t lane_const() {
    const uint32_t l32 = threadIdx.x & 31u;
    return (l32 * 4u) | ((128u + l32 * 4u) << 8) | (1u << 24);
}

// ---- combine-blob LDS image: Z_{D*2^k} (k = 0..6), Z4, byte table ----------
template <int WORDS = kCombWords, int THREADS = 1024>
__device__ __forceinline__ void load_comb_tables(uint32_t* lds, const uint32_t* __restrict__ blob) {
    copy_to_lds<WORDS, THREADS>(lds, blob);
}

// Z_L for L = 16n, 0 < n < 2^kCombSmallMaps (binary decomposition over Z_{16*2^i}).
__device__ __forceinline__ uint32_t zshift16(const uint32_t* lds, uint32_t x, uint32_t n) {
#pragma unroll
    for (int i = 0; i < kCombSmallMaps; ++i)
        if (n & (1u << i)) x = zmap(lds, kCombSmall + i * 1024, x);
    return x;
}

// Lane i + D's x for the lanes a reduction tree keeps (lane 0 at the last level; at level D the
// lanes that are multiples of 2D): D = 1, 2, 4, 8 through DPP row shifts (VALU, within the lane's
// row of 16), D = 16 and 32 through v_readlane -- instead of ds_bpermute round trips, which a
// chain of tree levels waits on one after another.  Other lanes get values the tree never uses.
template <int D>
__device__ __forceinline__ uint32_t tree_down(uint32_t x) {
    static_assert(D == 1 || D == 2 || D == 4 || D == 8 || D == 16 || D == 32, "tree levels");
    if constexpr (D <= 8) {
        return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x100 + D, 0xf, 0xf, false);  // row_shl:D
    } else if constexpr (D == 16) {  // lanes 0 and 32 take lanes 16 and 48
        const uint32_t a = (uint32_t)__builtin_amdgcn_readlane((int)x, 16);
        const uint32_t b = (uint32_t)__builtin_amdgcn_readlane((int)x, 48);
        return (threadIdx.x & 32u) ? b : a;
    } else {
        return (uint32_t)__builtin_amdgcn_readlane((int)x, 32);
    }
}

// Tree over the 64 lanes of a wave with maps Z_{D*2^d}: lane 0 gets
// XOR_l Z_{D*(63-l)}(v_l).
__device__ __forceinline__ uint32_t wave_tree(const uint32_t* lds, uint32_t v) {
    v = zmap(lds, 0, v) ^ tree_down<1>(v);
    v = zmap(lds, 1024, v) ^ tree_down<2>(v);
    v = zmap(lds, 2 * 1024, v) ^ tree_down<4>(v);
    v = zmap(lds, 3 * 1024, v) ^ tree_down<8>(v);
    v = zmap(lds, 4 * 1024, v) ^ tree_down<16>(v);
    return zmap(lds, 5 * 1024, v) ^ tree_down<32>(v);
}

// ---- small records staged through LDS (k_ragged_staged, k_wal_list_crc) ----------------
constexpr uint32_t kStgBytes = 12288;        // staging per wave: kStgVecs whole-wave 1 KiB loads (64 x 188 B)
constexpr int kStgVecs = (int)(kStgBytes / 1024);  // 16-byte loads per lane and batch
static_assert(kStgBytes % 1024 == 0, "every lane's loads land inside the stage: no guard per load");
constexpr int kStgZ4 = kRep16Words;          // [0, 64 KiB) the 16-copy Z_16 stride tables
constexpr int kStgT8 = kStgZ4 + 1024;
constexpr int kStgBuf = kStgT8 + 256;
constexpr int kStgLdsWords = kStgBuf + kStgWaves * (int)(kStgBytes / 4);  // 160,256 bytes
static_assert(kStgLdsWords * 4 <= 160 * 1024, "LDS of one workgroup");

// A wave-uniform 64-bit value into scalar registers (readfirstlane is int -> int: each half is
// taken as uint32_t before widening, or a low word >= 2^31 would sign-extend into the high one).
__device__ __forceinline__ uint64_t uniform64(uint64_t x) {
    const uint32_t h = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(x >> 32));
    const uint32_t l = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)x);
    return ((uint64_t)h << 32) | l;
}


// One DPP move of a 64-bit value (both halves; lanes the row pattern leaves without a source, or
// rows outside RM, take `old`).
template <int CTRL, int RM>
__device__ __forceinline__ uint64_t dpp64(uint64_t old, uint64_t x) {
    const uint32_t lo = (uint32_t)__builtin_amdgcn_update_dpp((int)(uint32_t)old, (int)(uint32_t)x, CTRL, RM, 0xf, false);
    const uint32_t hi =
        (uint32_t)__builtin_amdgcn_update_dpp((int)(uint32_t)(old >> 32), (int)(uint32_t)(x >> 32), CTRL, RM, 0xf, false);
    return ((uint64_t)hi << 32) | lo;
}
// Inclusive prefix min of lo and max of hi over the wave's lanes, through DPP (row shifts 1, 2, 4,
// 8, then the gfx9 row broadcasts): VALU steps instead of six dependent rounds of ds_bpermute,
// which share the LDS pipe and its counter with the stride lookups.
__device__ __forceinline__ void wave_prefix_minmax(uint64_t& lo, uint64_t& hi) {
    auto step = [&](uint64_t a, uint64_t b) {
        lo = a < lo ? a : lo;
        hi = b > hi ? b : hi;
    };
    step(dpp64<0x111, 0xf>(~0ull, lo), dpp64<0x111, 0xf>(0ull, hi));  // row_shr:1
    step(dpp64<0x112, 0xf>(~0ull, lo), dpp64<0x112, 0xf>(0ull, hi));  // row_shr:2
    step(dpp64<0x114, 0xf>(~0ull, lo), dpp64<0x114, 0xf>(0ull, hi));  // row_shr:4
    step(dpp64<0x118, 0xf>(~0ull, lo), dpp64<0x118, 0xf>(0ull, hi));  // row_shr:8
    step(dpp64<0x142, 0xa>(~0ull, lo), dpp64<0x142, 0xa>(0ull, hi));  // row_bcast:15 -> rows 1, 3
    step(dpp64<0x143, 0xc>(~0ull, lo), dpp64<0x143, 0xc>(0ull, hi));  // row_bcast:31 -> rows 2, 3
}

// Min of a 64-bit value over the wave (DPP prefix, lane 63 read back): uniform.
__device__ __forceinline__ uint64_t wave_min64(uint64_t x) {
    uint64_t hi = 0;
    wave_prefix_minmax(x, hi);
    return ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(x >> 32), 63) << 32) |
           (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)x, 63);
}

// Inclusive wave scan of 32-bit values through DPP (row shifts, then the row broadcasts of gfx9):
// six VALU steps instead of six dependent cross-lane LDS round trips (ds_bpermute) of the 64-bit
// scan below.
__device__ __forceinline__ uint32_t wave_incl_scan32(uint32_t x) {
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xf, 0xf, false);  // row_shr:1
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xf, 0xf, false);  // row_shr:2
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xf, 0xf, false);  // row_shr:4
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xf, 0xf, false);  // row_shr:8
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xa, 0xf, false);  // row_bcast:15 -> rows 1, 3
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xc, 0xf, false);  // row_bcast:31 -> rows 2, 3
    return x;
}

// Min and max of a 32-bit value over the wave (DPP prefix, lane 63 read back): uniform.
__device__ __forceinline__ uint32_t wave_min32(uint32_t x) {
    auto st = [&](uint32_t o) { x = o < x ? o : x; };
    st((uint32_t)__builtin_amdgcn_update_dpp(-1, (int)x, 0x111, 0xf, 0xf, false));
    st((uint32_t)__builtin_amdgcn_update_dpp(-1, (int)x, 0x112, 0xf, 0xf, false));
    st((uint32_t)__builtin_amdgcn_update_dpp(-1, (int)x, 0x114, 0xf, 0xf, false));
    st((uint32_t)__builtin_amdgcn_update_dpp(-1, (int)x, 0x118, 0xf, 0xf, false));
    st((uint32_t)__builtin_amdgcn_update_dpp(-1, (int)x, 0x142, 0xa, 0xf, false));
    st((uint32_t)__builtin_amdgcn_update_dpp(-1, (int)x, 0x143, 0xc, 0xf, false));
    return (uint32_t)__builtin_amdgcn_readlane((int)x, 63);
}
__device__ __forceinline__ uint32_t wave_max32(uint32_t x) {
    auto st = [&](uint32_t o) { x = o > x ? o : x; };
    st((uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xf, 0xf, false));
    st((uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xf, 0xf, false));
    st((uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xf, 0xf, false));
    st((uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xf, 0xf, false));
    st((uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xa, 0xf, false));
    st((uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xc, 0xf, false));
    return (uint32_t)__builtin_amdgcn_readlane((int)x, 63);
}

// OR of a 32-bit value over the wave (DPP prefix, lane 63 read back): uniform.
__device__ __forceinline__ uint32_t wave_or32(uint32_t x) {
    x |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xf, 0xf, false);
    x |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xf, 0xf, false);
    x |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xf, 0xf, false);
    x |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xf, 0xf, false);
    x |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xa, 0xf, false);
    x |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xc, 0xf, false);
    return (uint32_t)__builtin_amdgcn_readlane((int)x, 63);
}

struct StgBatch {
    uintptr_t p;    // this lane's record
    uint32_t n, init;
    bool vi;
    uintptr_t lo;   // the batch's aligned extent (wave-uniform); hi == 0: no live record
    uintptr_t hi;
};

__device__ __forceinline__ StgBatch stg_meta(const RaggedArgs& A, uint64_t n_rec, uint64_t base, uint32_t lane) {
    StgBatch B;
    const uint64_t ri = base + lane;
    B.vi = ri < n_rec;
    B.p = B.vi ? reinterpret_cast<uintptr_t>(A.arena + A.off[ri]) : 0;
    B.n = B.vi ? A.len[ri] : 0u;
    B.init = B.vi ? (A.init ? A.init[ri] : A.init_scalar) : 0u;
    const bool live = B.vi && B.n;
    uint64_t lo = live ? (B.p & ~uintptr_t(15)) : ~0ull, hi = live ? ((B.p + B.n + 15) & ~uintptr_t(15)) : 0ull;
    wave_prefix_minmax(lo, hi);  // lane 63: the whole wave's
    B.lo = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(lo >> 32), 63) << 32) |
           (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)lo, 63);
    B.hi = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(hi >> 32), 63) << 32) |
           (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)hi, 63);
    return B;
}
__device__ __forceinline__ bool stg_fits(const StgBatch& B) { return B.hi != 0 && B.hi - B.lo <= kStgBytes; }

__device__ __forceinline__ void stg_issue(const StgBatch& B, uint32_t lane, u32x4 (&v)[kStgVecs]) {
    const uint32_t nv = (uint32_t)((B.hi - B.lo) / 16);
#pragma unroll
    for (int q = 0; q < kStgVecs; ++q) {
        const uint32_t j = lane + 64u * q;  // past the extent: its first block again (no branch)
        v[q] = ldg<true>(reinterpret_cast<const uint8_t*>(B.lo + 16ull * (j < nv ? j : 0u)));
    }
}
__device__ __forceinline__ void stg_store(const StgBatch& B, uint32_t lane, const u32x4 (&v)[kStgVecs], uint8_t* stage) {
#pragma unroll
    for (int q = 0; q < kStgVecs; ++q) {
        const uint32_t j = lane + 64u * q;  // every slot of the stage (past the extent: unused)
        *reinterpret_cast<u32x4*>(stage + 16u * j) = v[q];
    }
}

// The staged kernels' table image: the lane blob's Z_16 stride tables in 16 copies, Z4 and the
// byte table.
template <int THREADS>
__device__ __forceinline__ void load_stg_tables(uint32_t* lds, const uint32_t* __restrict__ blob) {
    load_rep16_stride<THREADS>(lds, blob, [&] {
        copy_to_lds<1024, THREADS>(lds + kStgZ4, blob + kBlobZ4);
        copy_to_lds<256, THREADS>(lds + kStgT8, blob + kBlobT8);
    });
}

// Records in lane order (this lane's: [p, p + n), live = a record with bytes): the longest
// prefix of lanes whose aligned extent fits kStgBytes -- cnt lanes (wave-uniform, >= 1) and
// the extent [lo, hi).  cnt == 1 with hi == 0 and a live lane 0: that one record alone does
// not fit (it is read from global memory).  Lanes whose prefix holds no live record fit
// with an empty extent.
struct StgSpan {
    uintptr_t lo, hi;
    uint32_t cnt;
};
__device__ __forceinline__ StgSpan stg_prefix(uintptr_t p, uint32_t n, bool live, uint32_t lane) {
    uint64_t lo = live ? (p & ~uintptr_t(15)) : ~0ull, hi = live ? ((p + n + 15) & ~uintptr_t(15)) : 0ull;
    wave_prefix_minmax(lo, hi);  // inclusive prefix min / max
    const bool fits = hi == 0 || hi - lo <= kStgBytes;  // monotonic in the lane
    const uint32_t cnt = (uint32_t)__popcll(__ballot(fits));
    StgSpan S;
    if (cnt == 0) {
        S.lo = S.hi = 0;
        S.cnt = 1;
        return S;
    }
    S.lo = uniform64((uint64_t)__shfl((long long)lo, (int)cnt - 1));
    S.hi = uniform64((uint64_t)__shfl((long long)hi, (int)cnt - 1));
    S.cnt = cnt;
    if (S.hi == 0) S.lo = 0;
    return S;
}
// Copy [lo, hi) (hi - lo <= kStgBytes, 16-aligned) into the wave's stage: every load issued
// before the first store.
__device__ __forceinline__ void stg_copy(uintptr_t lo, uintptr_t hi, uint32_t lane, uint8_t* stage) {
    const uint32_t nv = (uint32_t)((hi - lo) / 16);
    u32x4 v[kStgVecs];
#pragma unroll
    for (int q = 0; q < kStgVecs; ++q) {
        const uint32_t j = lane + 64u * q;
        v[q] = ldg<true>(reinterpret_cast<const uint8_t*>(lo + 16ull * (j < nv ? j : 0u)));
    }
#pragma unroll
    for (int q = 0; q < kStgVecs; ++q) {
        const uint32_t j = lane + 64u * q;  // every slot of the stage (past the extent: unused)
        *reinterpret_cast<u32x4*>(stage + 16u * j) = v[q];
    }
}

// One record per lane out of the LDS stage, its 16-byte windows aligned to the record's END:
// the record [sp, sp + n) of the stage (byte offsets; 16 <= sp is not required, but the 15
// bytes before sp must be stage bytes too) is read as W = ceil(n / 16) windows ending at
// sp + n, the first window front-padded with h0 = 16 W - n bytes that are masked to zero.
// Zero bytes entering a zero register leave it zero, so the padded span steps from a zero
// register once ~init is xored into the record's first 4 bytes (the register a word step
// xors in, crc32c.cc:293-299): no head or tail byte steps, one dependent chain of W stride
// steps and the STEP4W fold.  Needs n >= 4 (the injected word lies inside the record).
// rd(q): dword q of the stage (q = byte offset / 4; the windows are read as dwords and
// funnel-shifted, v_alignbyte_b32).
template <int SMODE = 24, typename Rd>
__device__ __forceinline__ uint32_t lane_record_end(const uint32_t* lds, uint32_t X, int z4, uint32_t sp, uint32_t n,
                                                    uint32_t init, Rd&& rd) {
    const uint32_t W = (n + 15) >> 4, h0 = 16 * W - n;
    const uint32_t s0 = sp - h0, sh = s0 & 3;
    uint32_t q = s0 >> 2;
    uint32_t d0 = rd(q), d1 = rd(q + 1), d2 = rd(q + 2), d3 = rd(q + 3), d4 = rd(q + 4);
    uint32_t w0 = __builtin_amdgcn_alignbyte(d1, d0, sh), w1 = __builtin_amdgcn_alignbyte(d2, d1, sh);
    uint32_t w2 = __builtin_amdgcn_alignbyte(d3, d2, sh), w3 = __builtin_amdgcn_alignbyte(d4, d3, sh);
    // window 0: bytes [0, h0) are not the record's
    auto keep = [&](uint32_t k) {
        const int r = (int)h0 - 4 * (int)k;
        return r <= 0 ? ~0u : r >= 4 ? 0u : (~0u << (8 * r));
    };
    w0 &= keep(0);
    w1 &= keep(1);
    w2 &= keep(2);
    w3 &= keep(3);
    // ~init into bytes [h0, h0 + 4): word k0 and (unaligned) the next one, or window 1's first
    const uint32_t inj = ~init, b = h0 & 3, k0 = h0 >> 2;
    const uint32_t lo32 = inj << (8 * b), hi32 = b ? inj >> (32 - 8 * b) : 0u;
    w0 ^= k0 == 0 ? lo32 : 0u;
    w1 ^= (k0 == 1 ? lo32 : 0u) ^ (k0 == 0 ? hi32 : 0u);
    w2 ^= (k0 == 2 ? lo32 : 0u) ^ (k0 == 1 ? hi32 : 0u);
    w3 ^= (k0 == 3 ? lo32 : 0u) ^ (k0 == 2 ? hi32 : 0u);
    uint32_t carry = k0 == 3 ? hi32 : 0u;
    uint32_t a0 = w0, a1 = w1, a2 = w2, a3 = w3;
    if constexpr ((SMODE & 88) == 88) {
        // SMODE bit 6 (with the 16-copy image in swapped lane order): each window in three
        // phases kept apart by scheduling barriers -- the 16 lookup indices; every LDS read of the
        // window (the next window's stage dwords, then the 16 lookups) in flight together; the
        // xors.  (Left to itself the compiler issues the lookups of two accumulators, waits for
        // them, then issues the other two's: two LDS round trips per window.)
        const bool swp = (threadIdx.x & 16u) != 0;
        const uint32_t s0 = swp ? 0x0c0c0105u : 0x0c0c0004u, s1 = swp ? 0x0c0c0004u : 0x0c0c0105u;
        const uint32_t s2 = swp ? 0x0c0c0307u : 0x0c0c0206u, s3 = swp ? 0x0c0c0206u : 0x0c0c0307u;
        // SMODE bit 7: when every active lane's windows are dword-aligned (sh == 0: payload sizes and
        // strides that are multiples of 4), the windows are the stage dwords themselves, no funnel shifts
        if ((SMODE & 128) != 0 && __ballot(sh != 0u) == 0) {
            for (uint32_t j = 1; j < W; ++j) {
                q += 4;
                const uint32_t acc[4] = {a0, a1, a2, a3};
                uint32_t ix[16], l[16];
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    ix[4 * k] = __builtin_amdgcn_perm(X, acc[k], s0);
                    ix[4 * k + 1] = __builtin_amdgcn_perm(X, acc[k], s1);
                    ix[4 * k + 2] = __builtin_amdgcn_perm(X, acc[k], s2);
                    ix[4 * k + 3] = __builtin_amdgcn_perm(X, acc[k], s3);
                }
                __builtin_amdgcn_sched_barrier(0);
                const uint32_t e0 = rd(q), e1 = rd(q + 1), e2 = rd(q + 2), e3 = rd(q + 3);
#pragma unroll
                for (int k = 0; k < 16; ++k) l[k] = lds_at_byte(lds, ix[k]);
                __builtin_amdgcn_sched_barrier(0);
                a0 = xor3(xor3(l[0], l[1], e0 ^ carry), l[2], l[3]);
                carry = 0u;
                a1 = xor3(xor3(l[4], l[5], e1), l[6], l[7]);
                a2 = xor3(xor3(l[8], l[9], e2), l[10], l[11]);
                a3 = xor3(xor3(l[12], l[13], e3), l[14], l[15]);
            }
        } else
        for (uint32_t j = 1; j < W; ++j) {
            q += 4;
            const uint32_t acc[4] = {a0, a1, a2, a3};
            uint32_t ix[16], l[16];
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                ix[4 * k] = __builtin_amdgcn_perm(X, acc[k], s0);
                ix[4 * k + 1] = __builtin_amdgcn_perm(X, acc[k], s1);
                ix[4 * k + 2] = __builtin_amdgcn_perm(X, acc[k], s2);
                ix[4 * k + 3] = __builtin_amdgcn_perm(X, acc[k], s3);
            }
            __builtin_amdgcn_sched_barrier(0);
            d0 = d4;
            d1 = rd(q + 1);
            d2 = rd(q + 2);
            d3 = rd(q + 3);
            d4 = rd(q + 4);
#pragma unroll
            for (int k = 0; k < 16; ++k) l[k] = lds_at_byte(lds, ix[k]);
            __builtin_amdgcn_sched_barrier(0);
            const uint32_t vx = __builtin_amdgcn_alignbyte(d1, d0, sh) ^ carry;
            carry = 0u;
            a0 = xor3(xor3(l[0], l[1], vx), l[2], l[3]);
            a1 = xor3(xor3(l[4], l[5], __builtin_amdgcn_alignbyte(d2, d1, sh)), l[6], l[7]);
            a2 = xor3(xor3(l[8], l[9], __builtin_amdgcn_alignbyte(d3, d2, sh)), l[10], l[11]);
            a3 = xor3(xor3(l[12], l[13], __builtin_amdgcn_alignbyte(d4, d3, sh)), l[14], l[15]);
        }
    } else
    for (uint32_t j = 1; j < W; ++j) {
        q += 4;
        d0 = d4;
        d1 = rd(q + 1);
        d2 = rd(q + 2);
        d3 = rd(q + 3);
        d4 = rd(q + 4);
        u32x4 v;
        v.x = __builtin_amdgcn_alignbyte(d1, d0, sh) ^ carry;
        v.y = __builtin_amdgcn_alignbyte(d2, d1, sh);
        v.z = __builtin_amdgcn_alignbyte(d3, d2, sh);
        v.w = __builtin_amdgcn_alignbyte(d4, d3, sh);
        carry = 0u;
        step4<SMODE>(lds, X, a0, a1, a2, a3, v);
    }
    // the STEP4W fold Z4(a3 ^ Z4(a2 ^ Z4(a1 ^ Z4(a0)))) as Z16(a0) ^ Z4(a3 ^ Z4(a2 ^ Z4(a1))): Z16 is
    // the stride map, read from the replicated image beside the three-step chain
    const uint32_t z16 = (SMODE & 32) ? stride_step8(lds, a0, 0u)
                         : (SMODE & 16) ? stride_step16s(lds, X, a0, 0u)
                                        : stride_step16(lds, X, a0, 0u);
    uint32_t c = zmap(lds, z4, a1);
    c = zmap(lds, z4, c ^ a2);
    return ~(z16 ^ zmap(lds, z4, c ^ a3));
}

// LDS writes of a wave visible to its own later LDS reads (and its reads done before its
// next writes): the wave's LDS operations complete in order, so a wait for them and a
// compiler barrier suffice (no workgroup barrier).
__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0)
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// One record per lane: [p, p + n) with init, its aligned 16-byte blocks read through
// src(address) (16-aligned absolute address; LDS staging or global memory).  The reference's
// own structure (crc32c.cc:323-370): the unaligned head byte steps, four word slots striding
// 16 bytes through the aligned body (Z_16 stride tables in the 16-copy image: stride_step16),
// the STEP4W lane fold and the unaligned tail; records with no aligned 16-byte block inside
// are stepped word by word.  n must be > 0 (an empty record's CRC is init).
template <int MODE = 8, typename Src>
__device__ __forceinline__ uint32_t lane_record(const uint32_t* lds, uint32_t X, int z4, int t8, uintptr_t p,
                                                uint32_t n, uint32_t init, Src&& src) {
    uint32_t r = ~init;
    const uintptr_t e = p + n;
    const uintptr_t a = (p + 15) & ~uintptr_t(15), b = e & ~uintptr_t(15);
    if (b < a + 16) {  // short: the one or two blocks it touches, step by step
        for (uintptr_t blk = p & ~uintptr_t(15); blk < e; blk += 16) {
            const uint32_t from = p > blk ? (uint32_t)(p - blk) : 0u;
            const uint32_t to = e - blk < 16 ? (uint32_t)(e - blk) : 16u;
            r = steps_in_vec(lds, z4, t8, r, src(blk), from, to);
        }
        return ~r;
    }
    if (p < a) r = steps_in_vec(lds, z4, t8, r, src(a - 16), (uint32_t)(p - (a - 16)), 16u);
    const u32x4 v0 = src(a);
    uint32_t a0 = v0.x ^ r, a1 = v0.y, a2 = v0.z, a3 = v0.w;
    for (uintptr_t w = a + 16; w < b; w += 16) step4<MODE>(lds, X, a0, a1, a2, a3, src(w));
    r = lane_fold_at(lds, z4, a0, a1, a2, a3);
    if (e > b) r = steps_in_vec(lds, z4, t8, r, src(b), 0u, (uint32_t)(e - b));
    return ~r;
}

}  // namespace dev
}  // namespace engine
}  // namespace karma
