// karma_amd/csrc/crc_fixed.hip -- fixed-size record batches on MI355X (gfx950).
//
// Batched form of segment_file::append_record's per-record crc32c::Value
// (karma-store/segment_file.cc:22; algorithm karma-util/crc32c.cc:275-376).
// Record r = arena + r*rec_bytes.  Each record body is cut into k units
// (k = 1, or k = KW = 2 folded inside the wave, for batches large enough to fill
// the GPU), one unit per group of 8 lanes; otherwise the unit
// contributions are folded by the wave (8 units) and then k_combine_block or
// k_combine_fixed, one level per factor of 64, with maps Z_{D*2^d}.
#include <hip/hip_runtime.h>

#include "ab.h"
#include "crc_device.h"
#include "engine.h"
#include "wavelog.h"

namespace karma {
namespace engine {
namespace {

using namespace dev;

// Per-lane plan of unit u of a fixed-layout batch (arithmetic only, no memory
// access).  Records hold an aligned 16-byte block (rec_bytes >= 31), so the
// body start g.a is a safe address for every load of an empty or out-of-range
// unit.
struct FixedPlan {
    LaneUnit L;
    const uint8_t* hblk;  // 16-byte block with the unaligned head bytes [hfrom, 16)
    const uint8_t* tblk;  // 16-byte block with the unaligned tail bytes [0, tto)
    const uint8_t* inj_at;  // the body start when this unit holds it, else nullptr
    uint64_t r;
    uint32_t hfrom, tto;
    bool valid;
};

// ONE: a single record (no 64-bit division: r = 0).
template <bool ONE = false>
__device__ __forceinline__ FixedPlan fixed_plan(const FixedArgs& A, uint64_t u, uint64_t U, uint32_t l) {
    FixedPlan P;
    const uint64_t k = A.units_per_rec;
    P.valid = u < U;
    const uint64_t uu = P.valid ? u : 0;
    P.r = ONE ? 0 : k == 1 ? uu : uu / k;
    const uint64_t j = uu - P.r * k;
    const uint8_t* p = A.arena + P.r * A.rec_bytes;
    const Geom g = geom(p, A.rec_bytes);
    // unit j of the body [a, b), end-aligned at b: [b - (k-j)*U, b - (k-1-j)*U) clipped to a
    const uint8_t* ue = g.b - (int64_t)((k - 1 - j) * A.unit_bytes);
    const uint8_t* us_raw = ue - (int64_t)A.unit_bytes;
    const uint8_t* us = pmax(us_raw, g.a);
    const bool first = P.valid && g.a >= us_raw && g.a < ue;
    if (!P.valid || ue <= g.a) us = ue = g.a;  // empty: safe addresses, no steps
    P.L = lane_unit(us, ue, l);
    P.inj_at = first ? g.a : nullptr;
    const bool head = first && p < g.a;
    P.hblk = head ? g.a - 16 : g.a;
    P.hfrom = head ? (uint32_t)(p - (g.a - 16)) : 16u;
    const bool tail = P.valid && j == k - 1 && g.e > g.b;
    P.tblk = tail ? g.b : g.a;
    P.tto = tail ? (uint32_t)(g.e - g.b) : 0u;
    return P;
}

// Fixed records with rec_bytes >= 31: every lane streams its groups' units
// back to back; the loads of unit u + step (chunk 0, PF chunks, the head and
// tail blocks, the init value) are issued before unit u's last chunks are
// consumed (stream_unit), so no wave waits on a fresh load at a unit boundary.
// The first unit's loads are issued before the LDS table fill, which then
// costs no separate memory round trip.  WAVE_COMB (k % 8 == 0): the 8 groups of
// a wave hold units 8i..8i+7 of one record, end-aligned; a 3-level tree over
// the groups (Z_U, Z_2U, Z_4U) leaves one state per 8 units, so the combine
// kernels start one level up (a 64 MiB segment: 32768 -> 4096 states here).
// The fused combine of FUSE (one record, its wave states folded by the grid's last workgroup):
// thread t folds states [t m, t m + m) with Z_D (leading zero states pad k_in to 1024 m), reading
// each tagged state with an agent-scope atomic load until it carries this call's tag (a state
// whose store is not visible yet is waited for; no release fence or L2 write-back is needed);
// then the 64-lane tree and thread 0's fold of the 16 wave results, as k_combine_block.
__device__ void fused_record_fold(const FixedArgs& A, uint32_t* lds, uint32_t* wv, uint64_t k_in, uint32_t tag) {
    const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
    const uint64_t m = A.comb_m;
    const int64_t pad = (int64_t)(m * 1024 - k_in);
    const int64_t i0 = (int64_t)(threadIdx.x * m) - pad;
    unsigned long long* st = reinterpret_cast<unsigned long long*>(A.partial);
    // 8 states per thread in flight at once (the first 8 before the table copy), then checked
    constexpr int kQ = 8;
    auto load8 = [&](uint64_t q0, unsigned long long (&w)[kQ]) {
#pragma unroll
        for (int q = 0; q < kQ; ++q)
            w[q] = q0 + q < m && i0 + (int64_t)(q0 + q) >= 0
                       ? __hip_atomic_load(st + i0 + q0 + q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                       : ((unsigned long long)tag << 32);
    };
    unsigned long long w[kQ];
    load8(0, w);
    copy_to_lds<kBlockCombWords, kBlockThreads>(lds, A.block_blob);
    __syncthreads();
    uint32_t acc = 0;
    for (uint64_t q0 = 0; q0 < m; q0 += kQ) {
        if (q0) load8(q0, w);
#pragma unroll
        for (int q = 0; q < kQ; ++q) {
            if (q0 + q >= m) break;
            while ((uint32_t)(w[q] >> 32) != tag) {  // a store not visible yet: wait for it
                __builtin_amdgcn_s_sleep(1);
                w[q] = __hip_atomic_load(st + i0 + q0 + q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
            acc = zmap(lds, kBcZD, acc) ^ (uint32_t)w[q];
        }
    }
    acc = wave_tree(lds + kBcTree, acc);
    if (lane == 0) wv[wave] = acc;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t v = wv[0];
        for (int w = 1; w < 16; ++w) v = zmap(lds, kBcWave, v) ^ wv[w];
        A.out[0] = ~tail_register(lds, kBcZ4, kBcT8, v, geom(A.arena, A.rec_bytes));
    }
}

// (KARMA_FIXED_STEP_MODE / KARMA_SEGMENT_STEP_WIDE: a build's default window step -- step4 MODE 64 / 88,
// the phased step, for a whole-build A/B through tools/ragged_study.py LIBS; the shipped build: 0)
#ifndef KARMA_FIXED_STEP_MODE
#define KARMA_FIXED_STEP_MODE 0
#endif
#ifndef KARMA_SEGMENT_STEP_WIDE
#define KARMA_SEGMENT_STEP_WIDE false
#endif
template <int PF, bool NT, bool HAS_INIT, bool WAVE_COMB, int MODE = KARMA_FIXED_STEP_MODE, bool BAL = true, int KW = 1, bool FUSE = false>
__global__ __launch_bounds__(kBlockThreads) void k_units_fixed(FixedArgs A) {
    static_assert(!FUSE || WAVE_COMB, "the fused combine folds wave states");
    KB_SET_ARENA(reinterpret_cast<uintptr_t>(A.arena) & ~uintptr_t(15),
                 (reinterpret_cast<uintptr_t>(A.arena + A.n_rec * A.rec_bytes) + 15) & ~uintptr_t(15));
    constexpr bool kMaps = WAVE_COMB || KW > 1;
    __shared__ __attribute__((aligned(16))) uint32_t lds[kMaps ? kLdsWordsComb : kLdsWords];
    __shared__ uint32_t blk_next;  // BAL: the block's next wave-step (an LDS counter, lgkmcnt only)
    __shared__ uint32_t s_tag;  // FUSE: this call's tag
    if (FUSE && threadIdx.x == 0) {
        const uint32_t t = (uint32_t)__hip_atomic_load(A.fctl + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1u;
        s_tag = t ? t : 1u;
    }
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t l = lane & (kGroupLanes - 1);
    const uint32_t grp = lane / kGroupLanes;
    const uint32_t X = lane_const();
    const uint64_t k = A.units_per_rec;
    const uint64_t U = A.n_rec * k;
    const uint64_t nwaves = (uint64_t)gridDim.x * kWavesPerBlock;
    const uint64_t step = nwaves * kGroupsPerWave;
    uint64_t wb = (uint64_t)blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6);
    uint64_t u = wb * kGroupsPerWave + grp;
    // BAL: the block owns wave-steps b*16 + j + r*nwaves (j < 16, r < rounds) and its 16 waves
    // take them in that order from an LDS counter, so a wave that the CU's memory pipe serves
    // faster does more of them (static: the waves of one CU ended up to 60 us apart;
    // 128 GiB slice 19.81 vs 20.69 ms).
    const uint64_t nws = (U + kGroupsPerWave - 1) / kGroupsPerWave;
    const uint64_t bw0 = (uint64_t)blockIdx.x * kWavesPerBlock;
    if (BAL && threadIdx.x == 0) blk_next = kWavesPerBlock;  // steps 0..15 go to waves 0..15
    // (a dynamic tail -- the last steps taken from a global counter -- measured no gain here:
    // 1M x 4 KiB 0.6041 vs 0.6023 ms, 256K x 16 KiB 0.6224 vs 0.6144, profiles/r04_fixed_dyn_tail_ab.txt)
    const uint64_t S = nws;
    const uint32_t nidx = (uint32_t)((S + nwaves - 1) / nwaves) * kWavesPerBlock;
    // unit u's head block and init value, then its chunk loads, then the tables
    FixedPlan P = fixed_plan(A, u, U, l);
    u32x4 hv = ld16(P.hblk), tv = ld16(P.tblk);
    uint32_t iv = HAS_INIT ? *(const __attribute__((address_space(1))) uint32_t*)(A.init + P.r) : A.init_scalar;
    UnitLoads<PF> Ld;
    issue_unit_loads<PF, NT>(P.L, Ld);
    load_stream_tables(lds, A.blob);
    if constexpr (kMaps) copy_to_lds<3 * 1024, kBlockThreads>(lds + kCombLdsBase, A.comb_maps);
    __syncthreads();
    WLOG_DECL;
    WLOG_START();
    const uint64_t wlog_id = wb;
    (void)wlog_id;
    for (; wb < nws; ) {
        uint32_t inj = 0;
        if (P.inj_at) inj = P.hfrom < 16 ? steps_in_vec(lds, kLZ4, kLT8, ~iv, hv, P.hfrom, 16u) : ~iv;
        // Every load is issued ahead of unit boundaries, with the next unit's
        // chunks (a load issued just before the main loop would be waited on by
        // its first batch: vmcnt counts in order).
        const u32x4 tcur = tv;
        FixedPlan N;
        uint64_t wb_next = wb + nwaves;
        uint32_t R = stream_unit<PF, NT, MODE>(lds, X, l, P.L, Ld, P.inj_at, inj, [&](UnitLoads<PF>& nx) {
            if constexpr (BAL) {
                uint32_t i = 0;
                if (lane == 0) i = atomicAdd(&blk_next, 1u);
                i = __builtin_amdgcn_readfirstlane(__shfl(i, 0));
                wb_next = i < nidx ? bw0 + (i % kWavesPerBlock) + (uint64_t)(i / kWavesPerBlock) * nwaves : nws;
            }
            N = fixed_plan(A, wb_next * kGroupsPerWave + grp, U, l);
            hv = ld16(N.hblk);
            tv = ld16(N.tblk);
            if constexpr (HAS_INIT) iv = *(const __attribute__((address_space(1))) uint32_t*)(A.init + N.r);
            issue_unit_loads<PF, NT>(N.L, nx);
        });
        if constexpr (WAVE_COMB) {  // unit states sit in lanes 8g; fold g = 0..7 (g = 7 ends last)
            R = zmap(lds, kCombLdsBase, R) ^ tree_down<8>(R);
            R = zmap(lds, kCombLdsBase + 1024, R) ^ tree_down<16>(R);
            R = zmap(lds, kCombLdsBase + 2048, R) ^ tree_down<32>(R);
            if constexpr (FUSE) {  // tagged, visible to the last workgroup without a fence
                if (P.valid && lane == 0)
                    __hip_atomic_store(reinterpret_cast<unsigned long long*>(A.partial) + wb,
                                       ((unsigned long long)s_tag << 32) | R, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            } else if (P.valid && lane == 0) {
                A.partial[wb] = R;  // state wb = units 8wb .. 8wb+7
            }
        } else if constexpr (KW > 1) {
            // the record's KW units sit in groups KW*i .. KW*i+KW-1 of this wave (end-aligned: all
            // but the first are full); fold them into the last group, whose lanes hold the tail:
            // level d, group g takes group g - 2^d's state shifted over 2^d units (Z_{2^d U})
            uint32_t t = __shfl_up(R, 8, 64);
            R = zmap(lds, kCombLdsBase, t) ^ R;
            if constexpr (KW >= 4) {
                t = __shfl_up(R, 16, 64);
                R = zmap(lds, kCombLdsBase + 1024, t) ^ R;
            }
            if constexpr (KW == 8) {
                t = __shfl_up(R, 32, 64);
                R = zmap(lds, kCombLdsBase + 2048, t) ^ R;
            }
            if (P.valid && l == 0 && (grp & (KW - 1)) == KW - 1)
                A.out[P.r] = ~steps_in_vec(lds, kLZ4, kLT8, R, tcur, 0u, P.tto);
        } else if (P.valid && l == 0) {
            if (k == 1)
                A.out[P.r] = ~steps_in_vec(lds, kLZ4, kLT8, R, tcur, 0u, P.tto);
            else
                A.partial[u] = R;
        }
        WLOG_STEP();
        WLOG_UNIT(P.valid && l == 0, A.unit_bytes);
        P = N;
        wb = wb_next;
        u = wb * kGroupsPerWave + grp;
    }
    WLOG_END(wlog_id);
    if constexpr (FUSE) {  // the grid's last workgroup folds the record's wave states
        // (no completion counter: 256 workgroups' atomics on one word serialise at the memory
        // side; the fold waits on each state's tag instead.  Every workgroup reads the tag at
        // its start, before its states exist, so the fold -- which waits for all of them --
        // retires the tag only after every workgroup has read it.)
        if (blockIdx.x + 1 != gridDim.x) return;
        __syncthreads();  // this workgroup's waves are done with the stream tables
        __shared__ uint32_t wv[16];
        fused_record_fold(A, lds, wv, A.units_per_rec / kGroupsPerWave, s_tag);
        if (threadIdx.x == 0)  // retired: the next call (stream order) takes the next tag
            __hip_atomic_store(A.fctl + 1, (unsigned long long)s_tag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

// ---- one segment, one wave-step per wave (karma_crc32c_stream up to grid x 16 x 8 units) ------
// DESIGN.md Appendix B "One segment (round 4)": a 64 MiB scan is 4,096 wave-steps of 8 x 2 KiB units, one per
// wave of a 256-workgroup grid, so the looping kernel above spends its time in latency: the LDS
// table fill behind the first chunk loads (~4.7 us), four batches of chunk loads one round trip
// each, and a last-workgroup fold of 4,096 wave states (~4.8 us).  Here every lane issues the
// table words it fills first and then all of its unit's chunk loads (<= 16, 64 VGPRs), so the
// fill overlaps the stream and the stream is one round trip; the 16-copy stride image (64 KiB,
// read conflict-free by stride_step16s) leaves LDS for the fold maps.  Each workgroup folds its
// 16 wave states in LDS and publishes one tagged state; the grid's last workgroup folds those
// (at most 1024: a 64-lane tree per wave, then a Horner step per wave) and writes the CRC.
// Forward progress: as the FUSE kernel (include/karma_crc32c.h: grid <= CUs, in-order dispatch).
constexpr int kSegZ4 = kRep16Words;                        // Z4, Z16, Z32, Z64, byte table (the blob's)
constexpr int kSegComb = kSegZ4 + kSmallWords;             // comb_maps: Z_{U 2^k}, k = 0..6
constexpr int kSegGrid = kSegComb + kCombMaps * 1024;      // block_blob: Z_{128 U 2^k}, k = 0..6
constexpr int kSegLdsWords = kSegGrid + kCombMaps * 1024;  // 140,288 bytes
static_assert(kSegLdsWords * 4 <= 160 * 1024, "LDS of one workgroup");
constexpr int kSegMaxChunks = 16;                          // units of at most 2 KiB

#ifdef KARMA_AB  // tools build: per-workgroup phase stamps of k_segment_once (karma_ab_seg_log)
__device__ uint64_t* g_seg_log;
#define SEG_STAMP(i)                                                                  \
    do {                                                                              \
        if (g_seg_log && threadIdx.x == 0) g_seg_log[blockIdx.x * 8 + (i)] = wall_clock64(); \
    } while (0)
#else
#define SEG_STAMP(i) ((void)0)
#endif


// ARRIVE: the workgroup that arrives last folds (one ticket per workgroup from fctl[0] after its
// state is published; the last ticket resets the counter), instead of the grid's highest-index
// workgroup waiting for the others: no workgroup waits on one that may not have been scheduled, so
// the forward-progress contract of include/karma_crc32c.h is not needed.  Every workgroup then
// loads the grid fold maps (any may fold).
// R8 (tools build A/B, round 6): the 8-copy stride image (32 KiB, stride_step8) instead of the
// 16-copy one (64 KiB): half the table fill the chunk loads queue behind.
// LATE (tools build A/B, round 6): the comb maps only the workgroup fold uses (Z_8U .. Z_64U, 16 of
// the fill's 49 KiB) loaded after the chunk loads and stored after the steps.
template <bool NT, bool ARRIVE = false, bool R8 = false, bool LATE = false, bool WIDE = KARMA_SEGMENT_STEP_WIDE>
__global__ __launch_bounds__(kBlockThreads) void k_segment_once(FixedArgs A) {
    constexpr int TW = R8 ? kRep8Words : kRep16Words;
    constexpr int kSegZ4 = TW, kSegComb = kSegZ4 + kSmallWords, kSegGrid = kSegComb + kCombMaps * 1024;
    constexpr int kSegLdsWords = kSegGrid + kCombMaps * 1024;
    KB_SET_ARENA(reinterpret_cast<uintptr_t>(A.arena) & ~uintptr_t(15),
                 (reinterpret_cast<uintptr_t>(A.arena + A.rec_bytes) + 15) & ~uintptr_t(15));
    __shared__ __attribute__((aligned(16))) uint32_t lds[kSegLdsWords];
    __shared__ uint32_t wst[kWavesPerBlock];
    const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
    const uint32_t l = lane & (kGroupLanes - 1), grp = lane / kGroupLanes;
    const bool last_wg = blockIdx.x + 1 == gridDim.x;
    SEG_STAMP(0);
    // The tables first, into LDS, and only then the chunk loads: issued together, the table loads
    // (L2 misses after the previous call's stream) queued at the memory channels behind the whole
    // grid's 64 MiB of chunk requests and landed ~10 us in, after the data, so no step overlapped
    // the stream.  (Round 5: the chunk loads issued after the table loads but before the table
    // stores -- the stores then wait for the table loads alone -- measured 2 us slower per isolated
    // 64 MiB call, profiles/r05_segment_early_ab.json.)  The call's tag, the grid's fold maps and the tail block are read after the steps.
    // 1. the table words this thread fills
    constexpr int NV16 = TW / 4, IT16 = NV16 / kBlockThreads;
    uint32_t e16[IT16];
#pragma unroll
    for (int q = 0; q < IT16; ++q) {
        const int v = (int)threadIdx.x + q * kBlockThreads;
        // (16-copy: row e = v >> 4, table k; 8-copy, load_rep8_stride's layout: entry v >> 3, table (v >> 1) & 3)
        const int row = R8 ? v >> 3 : v >> 4, k = R8 ? (v >> 1) & 3 : (v >> 2) & 3;
        e16[q] = *(const __attribute__((address_space(1))) uint32_t*)(A.blob + kBlobStride + k * 256 + row);
    }
    LdsCopy<kSmallWords, kBlockThreads> small;
    small.load(A.blob + 1024);
    constexpr int kEarlyMaps = LATE ? 3 : kCombMaps;  // (the wave trees use Z_U, Z_2U, Z_4U)
    LdsCopy<kEarlyMaps * 1024, kBlockThreads> comb;
    comb.load(A.comb_maps);
    SEG_STAMP(6);
    // 2. this lane's unit (arithmetic only: it runs while the table loads are in flight)
    const uint64_t U = A.units_per_rec;
    const uint64_t u = ((uint64_t)blockIdx.x * kWavesPerBlock + wave) * kGroupsPerWave + grp;
    const FixedPlan P = fixed_plan<true>(A, u, U, l);
    const LaneUnit& L = P.L;
    const bool ok0 = L.nch > 0 && L.w >= L.us && L.w < L.ue;
    // 3. the tables into LDS
    u32x4* l4 = reinterpret_cast<u32x4*>(lds);
#pragma unroll
    for (int q = 0; q < IT16; ++q) l4[(int)threadIdx.x + q * kBlockThreads] = u32x4{e16[q], e16[q], e16[q], e16[q]};
    small.store(lds + kSegZ4);
    comb.store(lds + kSegComb);
    __syncthreads();
    SEG_STAMP(1);
    // 4. every chunk load of the unit and its head block, consumed in issue order (vmcnt counts)
    const u32x4 hv = ld16(P.hblk);
    asm volatile("" ::: "memory");  // (issued before the chunks: the first step needs it)
    u32x4 v[kSegMaxChunks];
    v[0] = ldg<NT>(ok0 ? L.w : L.lclamp);
#pragma unroll
    for (int q = 1; q < kSegMaxChunks; ++q) v[q] = ldg<NT>(pmin(L.w + q * kChunk, L.lclamp));
    LdsCopy<LATE ? (kCombMaps - 3) * 1024 : 1024, kBlockThreads> comb_late;  // (LATE: behind the chunks)
    if constexpr (LATE) comb_late.load(A.comb_maps + 3 * 1024);
    SEG_STAMP(7);
    // 5. the unit's windows (stride_step16s: the 16-copy image in swapped lane order), the lane
    //    fold and the 8-lane tree
    const uint32_t X = lane_const16();
    uint32_t inj = 0;
    if (P.inj_at) {  // (a per-record init array holds one value: the record's)
        const uint32_t init = A.init ? *(const __attribute__((address_space(1))) uint32_t*)A.init : A.init_scalar;
        inj = P.hfrom < 16 ? steps_in_vec(lds, kSegZ4, kSegZ4 + 4096, ~init, hv, P.hfrom, 16u) : ~init;
    }
    u32x4 x0 = ok0 ? v[0] : u32x4{0u, 0u, 0u, 0u};
    if (ok0 && L.w == P.inj_at) x0.x ^= inj;
    uint32_t a0 = x0.x, a1 = x0.y, a2 = x0.z, a3 = x0.w;
#pragma unroll
    for (int q = 1; q < kSegMaxChunks; ++q)
        if (q < L.nch - 1 || (q == L.nch - 1 && L.lok)) step4<R8 ? 32 : WIDE ? 88 : 24>(lds, X, a0, a1, a2, a3, v[q]);
    LdsCopy<kCombMaps * 1024, kBlockThreads> grid;  // the last workgroup's fold maps, in flight meanwhile
    if (ARRIVE || last_wg) grid.load(A.block_blob);
    uint32_t tag = 0;  // wave 0 publishes the workgroup's state, tagged with the call's tag
    if (wave == 0)
        tag = __hip_atomic_load(reinterpret_cast<const uint32_t*>(A.fctl + 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1u;
    uint32_t c = lane_fold_at(lds, kSegZ4, a0, a1, a2, a3);
    c = __shfl(c, (int)((lane & ~(kGroupLanes - 1u)) | ((l + L.m + 1) & (kGroupLanes - 1))), 64);
    // (the tree levels through DPP / readlane, tree_down: no LDS round trip between levels)
    c = zmap(lds, kSegZ4 + 1024, c) ^ tree_down<1>(c);
    c = zmap(lds, kSegZ4 + 2048, c) ^ tree_down<2>(c);
    c = zmap(lds, kSegZ4 + 3072, c) ^ tree_down<4>(c);
    // 6. the wave's 8 units (Z_U, Z_2U, Z_4U), the workgroup's 16 waves (Z_8U .. Z_64U)
    c = zmap(lds, kSegComb, c) ^ tree_down<8>(c);
    c = zmap(lds, kSegComb + 1024, c) ^ tree_down<16>(c);
    c = zmap(lds, kSegComb + 2048, c) ^ tree_down<32>(c);
    if (lane == 0) wst[wave] = c;
    if (ARRIVE || last_wg) grid.store(lds + kSegGrid);
    if constexpr (LATE) comb_late.store(lds + kSegComb + 3 * 1024);
    SEG_STAMP(2);
    __syncthreads();
    __shared__ uint32_t s_tag;
    __shared__ uint32_t s_last;
    if (wave == 0) {
        const uint32_t my_tag = tag ? tag : 1u;
        uint32_t s = lane < kWavesPerBlock ? wst[lane] : 0u;
        s = zmap(lds, kSegComb + 3 * 1024, s) ^ tree_down<1>(s);
        s = zmap(lds, kSegComb + 4 * 1024, s) ^ tree_down<2>(s);
        s = zmap(lds, kSegComb + 5 * 1024, s) ^ tree_down<4>(s);
        s = zmap(lds, kSegComb + 6 * 1024, s) ^ tree_down<8>(s);
        if (lane == 0)  // tagged: visible to the last workgroup without a fence
            __hip_atomic_store(reinterpret_cast<unsigned long long*>(A.partial) + blockIdx.x,
                               ((unsigned long long)my_tag << 32) | s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (lane == 0) s_tag = my_tag;
        if (ARRIVE && lane == 0)  // the ticket: taken after the state's store was issued
            s_last = __hip_atomic_fetch_add(A.fctl, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1 == gridDim.x;
    }
    SEG_STAMP(3);
    if (ARRIVE) {
        __syncthreads();  // s_last, s_tag
        if (!s_last) return;
    } else {
        if (!last_wg) return;
        __syncthreads();  // s_tag
    }
    const uint32_t my_tag = s_tag;
    // 7. the grid's last workgroup: its states, end-aligned (leading zeros pad them to whole waves),
    //    a 64-lane tree per wave (Z_{128U 2^d}), the wave results by Horner (Z_{64 128U}), the tail
    const uint32_t G = gridDim.x, nw = (G + 63) / 64, pad = nw * 64 - G;
    const Geom g0 = geom(A.arena, A.rec_bytes);  // the record's tail block (thread 0), in flight during the wait
    const u32x4 tv = ld16(threadIdx.x == 0 && g0.e > g0.b ? g0.b : g0.a);
    uint32_t s = 0;
    if (threadIdx.x < nw * 64 && threadIdx.x >= pad) {
        unsigned long long* st = reinterpret_cast<unsigned long long*>(A.partial) + (threadIdx.x - pad);
        unsigned long long w = __hip_atomic_load(st, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        while ((uint32_t)(w >> 32) != my_tag) {  // a workgroup whose state is not visible yet
            __builtin_amdgcn_s_sleep(1);
            w = __hip_atomic_load(st, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        s = (uint32_t)w;
    }
    if (wave < nw) {
        s = zmap(lds, kSegGrid, s) ^ tree_down<1>(s);
        s = zmap(lds, kSegGrid + 1024, s) ^ tree_down<2>(s);
        s = zmap(lds, kSegGrid + 2 * 1024, s) ^ tree_down<4>(s);
        s = zmap(lds, kSegGrid + 3 * 1024, s) ^ tree_down<8>(s);
        s = zmap(lds, kSegGrid + 4 * 1024, s) ^ tree_down<16>(s);
        s = zmap(lds, kSegGrid + 5 * 1024, s) ^ tree_down<32>(s);
        if (lane == 0) wst[wave] = s;
    }
    __syncthreads();
    SEG_STAMP(4);
    if (threadIdx.x == 0) {
        uint32_t r = wst[0];
        for (uint32_t w = 1; w < nw; ++w) r = zmap(lds, kSegGrid + 6 * 1024, r) ^ wst[w];
        A.out[0] = ~steps_in_vec(lds, kSegZ4, kSegZ4 + 4096, r, tv, 0u, g0.e > g0.b ? (uint32_t)(g0.e - g0.b) : 0u);
        __hip_atomic_store(A.fctl + 1, (unsigned long long)my_tag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (ARRIVE)  // every ticket of this call is taken: the next call on the stream starts from 0
            __hip_atomic_store(A.fctl, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    SEG_STAMP(5);
}

// Records of fewer than 31 bytes may hold no aligned 16-byte block (and tiny
// batches need no streaming): the general kernel, one unit per group, each
// unit's loads issued when the unit starts.  Also the A/B baseline (variant 1).
template <int PF, bool NT>
__global__ __launch_bounds__(kBlockThreads) void k_units_fixed_v1(FixedArgs A) {
    KB_SET_ARENA(reinterpret_cast<uintptr_t>(A.arena) & ~uintptr_t(15),
                 (reinterpret_cast<uintptr_t>(A.arena + A.n_rec * A.rec_bytes) + 15) & ~uintptr_t(15));
    __shared__ __attribute__((aligned(16))) uint32_t lds[kLdsWords];
    load_stream_tables(lds, A.blob);
    __syncthreads();
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t l = lane & (kGroupLanes - 1);
    const uint32_t grp = lane / kGroupLanes;
    const uint32_t X = lane_const();
    const uint64_t k = A.units_per_rec;
    const uint64_t U = A.n_rec * k;
    const uint64_t nwaves = (uint64_t)gridDim.x * kWavesPerBlock;
    WLOG_DECL;
    WLOG_START();
    for (uint64_t wb = (uint64_t)blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6); wb * kGroupsPerWave < U;
         wb += nwaves) {
        WLOG_STEP();
        const uint64_t u = wb * kGroupsPerWave + grp;
        const bool valid = u < U;
        uint64_t r = 0, j = 0;
        if (valid) {
            if (k == 1) {
                r = u;
            } else {
                r = u / k;
                j = u - r * k;
            }
        }
        const uint8_t* p = A.arena + r * A.rec_bytes;
        const uint32_t init = valid ? (A.init ? A.init[r] : A.init_scalar) : 0u;
        const Geom g = geom(p, A.rec_bytes);
        // unit j of the body [a, b), end-aligned at b: [b - (k-j)*U, b - (k-1-j)*U) clipped to a
        const uint8_t* us = nullptr;
        const uint8_t* ue = nullptr;
        const uint8_t* inj_at = nullptr;
        uint32_t inj = 0;
        if (valid && !g.is_short) {
            ue = g.b - (int64_t)((k - 1 - j) * A.unit_bytes);
            const uint8_t* us_raw = ue - (int64_t)A.unit_bytes;
            us = pmax(us_raw, g.a);
            if (us > ue) us = ue;
            if (g.a >= us_raw && g.a < ue) {  // this unit holds the body start
                inj_at = g.a;
                inj = head_register(lds, kLZ4, kLT8, p, g, init);
            }
        }
        uint32_t R = group_unit<PF, NT>(lds, X, l, us, ue, inj_at, inj);
        WLOG_UNIT(valid && l == 0, ue - us);
        if (valid && l == 0) {
            if (g.is_short) {
                A.out[r] = short_record(lds, kLZ4, kLT8, p, A.rec_bytes, init);
            } else if (k == 1) {
                A.out[r] = ~tail_register(lds, kLZ4, kLT8, R, g);
            } else {
                A.partial[u] = R;
            }
        }
    }
    WLOG_END((uint64_t)blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6));
}

// One combine level: record r's k_in states (end-aligned, D bytes each) ->
// k_out = ceil(k_in / 64) states of 64*D bytes; the last level (k_out == 1)
// adds the record tail and writes the CRC.  One wave per output state.
__global__ __launch_bounds__(256) void k_combine_fixed(FixedArgs A, const uint32_t* in, uint64_t k_in, uint32_t* outs,
                                                      uint64_t k_out, const uint32_t* comb) {
    KB_SET_ARENA(reinterpret_cast<uintptr_t>(A.arena) & ~uintptr_t(15),
                 (reinterpret_cast<uintptr_t>(A.arena + A.n_rec * A.rec_bytes) + 15) & ~uintptr_t(15));
    __shared__ __attribute__((aligned(16))) uint32_t lds[kCombCoreWords];
    load_comb_tables<kCombCoreWords, 256>(lds, comb);
    __syncthreads();
    const uint32_t lane = threadIdx.x & 63u;
    const uint64_t nwaves = (uint64_t)gridDim.x * (blockDim.x >> 6);
    const uint64_t total = A.n_rec * k_out;
    const int64_t pad = (int64_t)(k_out * 64 - k_in);
    for (uint64_t t = (uint64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); t < total; t += nwaves) {
        const uint64_t r = t / k_out;
        const uint64_t o = t - r * k_out;
        const int64_t idx = (int64_t)(o * 64 + lane) - pad;
        uint32_t v = idx >= 0 ? in[r * k_in + idx] : 0u;
        v = wave_tree(lds, v);
        if (lane == 0) {
            if (k_out == 1) {
                const uint8_t* p = A.arena + r * A.rec_bytes;
                A.out[r] = ~tail_register(lds, kCombZ4, kCombT8, v, geom(p, A.rec_bytes));
            } else {
                outs[r * k_out + o] = v;
            }
        }
    }
}

// Every state of one record (blockIdx.x) folded in one block: thread t folds
// states [t*m, t*m + m) (leading zero states pad k_in to 1024 m) with Z_D, the
// 64-lane tree (Z_{mD*2^d}) folds each wave, thread 0 folds the 16 wave
// results with Z_{64mD}, adds the record tail and writes the CRC.
__global__ __launch_bounds__(1024) void k_combine_block(FixedArgs A, const uint32_t* in, uint64_t k_in, uint64_t m,
                                                        const uint32_t* bc) {
    KB_SET_ARENA(reinterpret_cast<uintptr_t>(A.arena) & ~uintptr_t(15),
                 (reinterpret_cast<uintptr_t>(A.arena + A.n_rec * A.rec_bytes) + 15) & ~uintptr_t(15));
    __shared__ __attribute__((aligned(16))) uint32_t lds[kBlockCombWords];
    __shared__ uint32_t wv[16];
    const uint64_t r = blockIdx.x;
    const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
    const int64_t pad = (int64_t)(m * 1024 - k_in);
    const int64_t i0 = (int64_t)(threadIdx.x * m) - pad;
    const uint32_t* rs = in + r * k_in;
    uint32_t first[8];  // the first states are issued before the table fill
#pragma unroll
    for (int q = 0; q < 8; ++q) first[q] = (uint64_t)q < m && i0 + q >= 0 ? rs[i0 + q] : 0u;
    copy_to_lds<kBlockCombWords, 1024>(lds, bc);
    __syncthreads();
    uint32_t acc = 0;
#pragma unroll
    for (int q = 0; q < 8; ++q)
        if ((uint64_t)q < m) acc = zmap(lds, kBcZD, acc) ^ first[q];
    for (uint64_t i = 8; i < m; i += 8) {
        uint32_t sv[8];
#pragma unroll
        for (int q = 0; q < 8; ++q) sv[q] = i + q < m && i0 + (int64_t)(i + q) >= 0 ? rs[i0 + i + q] : 0u;
#pragma unroll
        for (int q = 0; q < 8; ++q)
            if (i + q < m) acc = zmap(lds, kBcZD, acc) ^ sv[q];
    }
    acc = wave_tree(lds + kBcTree, acc);
    if (lane == 0) wv[wave] = acc;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t v = wv[0];
        for (int w = 1; w < 16; ++w) v = zmap(lds, kBcWave, v) ^ wv[w];
        const uint8_t* p = A.arena + r * A.rec_bytes;
        A.out[r] = ~tail_register(lds, kBcZ4, kBcT8, v, geom(p, A.rec_bytes));
    }
}

#ifdef KARMA_AB
// Tools build only (ab.h): the alternatives measured in DESIGN.md §4, chosen per
// call by KARMA_CRC_VARIANT (1 = v1 kernel, 2 = 2 chunks in flight, 6 = timing
// only with WRONG CRCs, 7 = static wave-steps).  Returns false for the shipped
// kernel (variant 0, or a plan shape the variant does not cover).
bool launch_fixed_ab(const FixedArgs& a, dim3 grid, dim3 blk, hipStream_t s) {
    const long v = KARMA_AB_KNOB("KARMA_CRC_VARIANT", 0);
    if (v == 0 || a.rec_bytes < 31 || (!a.fold_k && !a.comb_maps && a.unit_bytes < 2048)) return false;
    if (a.fold_k) {
        if (v != 7) return false;
#define KARMA_FOLD_STATIC(KW)                                                                              \
    if (a.init) hipLaunchKernelGGL((k_units_fixed<4, true, true, false, 0, false, KW>), grid, blk, 0, s, a); \
    else hipLaunchKernelGGL((k_units_fixed<4, true, false, false, 0, false, KW>), grid, blk, 0, s, a);
        if (a.fold_k == 2) { KARMA_FOLD_STATIC(2) } else if (a.fold_k == 4) { KARMA_FOLD_STATIC(4) } else { KARMA_FOLD_STATIC(8) }
#undef KARMA_FOLD_STATIC
        return true;
    }
    if (a.comb_maps) {
        if (v != 7) return false;
        if (a.init) hipLaunchKernelGGL((k_units_fixed<4, true, true, true, 0, false>), grid, blk, 0, s, a);
        else hipLaunchKernelGGL((k_units_fixed<4, true, false, true, 0, false>), grid, blk, 0, s, a);
        return true;
    }
    switch (v) {
        case 1: hipLaunchKernelGGL((k_units_fixed_v1<4, true>), grid, blk, 0, s, a); return true;
        case 2:
            if (a.init) hipLaunchKernelGGL((k_units_fixed<2, true, true, false>), grid, blk, 0, s, a);
            else hipLaunchKernelGGL((k_units_fixed<2, true, false, false>), grid, blk, 0, s, a);
            return true;
        case 6: hipLaunchKernelGGL((k_units_fixed<4, true, false, false, 1>), grid, blk, 0, s, a); return true;
        case 7:
            if (a.init) hipLaunchKernelGGL((k_units_fixed<4, true, true, false, 0, false>), grid, blk, 0, s, a);
            else hipLaunchKernelGGL((k_units_fixed<4, true, false, false, 0, false>), grid, blk, 0, s, a);
            return true;
        default: return false;
    }
}
#endif

}  // namespace

hipError_t launch_fixed(const FixedArgs& a, int grid_blocks, hipStream_t s) {
    if (a.n_rec == 0) return hipSuccess;
    const uint64_t units = a.n_rec * a.units_per_rec;
    const uint64_t need = (units + kGroupsPerWave * kWavesPerBlock - 1) / (kGroupsPerWave * kWavesPerBlock);
    const dim3 grid((unsigned)(need < (uint64_t)grid_blocks ? need : (uint64_t)grid_blocks));
    units_timer_begin(s);
    const dim3 blk(kBlockThreads);
#ifdef KARMA_AB
    if (launch_fixed_ab(a, grid, blk, s)) {
        units_timer_end(s);
        return hipGetLastError();
    }
#endif
    // Records of < 31 bytes may hold no aligned 16-byte block.  Units under 2 KiB:
    // the pipelined kernel's extra per-unit work outweighs its hidden latency
    // (1 KiB units: 0.700 vs 0.669 ms per 4 GiB; 4 KiB: 0.628 vs 0.641).
    if (a.fold_k) {  // k = fold_k units per record folded in the wave, units >= 2 KiB (planner)
#define KARMA_FOLD(KW)                                                                                \
    if (a.init) hipLaunchKernelGGL((k_units_fixed<4, true, true, false, KARMA_FIXED_STEP_MODE, true, KW>), grid, blk, 0, s, a); \
    else hipLaunchKernelGGL((k_units_fixed<4, true, false, false, KARMA_FIXED_STEP_MODE, true, KW>), grid, blk, 0, s, a);
        if (a.fold_k == 2) { KARMA_FOLD(2) } else if (a.fold_k == 4) { KARMA_FOLD(4) } else { KARMA_FOLD(8) }
#undef KARMA_FOLD
    } else if (a.comb_maps && a.fctl) {  // one record, its wave states folded by the last workgroup
        if (a.n_rec != 1 || !a.block_blob || a.comb_m == 0 || a.units_per_rec / kGroupsPerWave > a.comb_m * 1024)
            return hipErrorInvalidValue;
        if (a.init) hipLaunchKernelGGL((k_units_fixed<4, true, true, true, KARMA_FIXED_STEP_MODE, true, 1, true>), grid, blk, 0, s, a);
        else hipLaunchKernelGGL((k_units_fixed<4, true, false, true, KARMA_FIXED_STEP_MODE, true, 1, true>), grid, blk, 0, s, a);
    } else if (a.comb_maps) {  // k % 8 == 0, units >= 2 KiB (planner)
        if (a.init) hipLaunchKernelGGL((k_units_fixed<4, true, true, true>), grid, blk, 0, s, a);
        else hipLaunchKernelGGL((k_units_fixed<4, true, false, true>), grid, blk, 0, s, a);
    } else if (a.rec_bytes < 31 || a.unit_bytes < 2048) {
        hipLaunchKernelGGL((k_units_fixed_v1<4, true>), grid, blk, 0, s, a);
    } else {
        if (a.init) hipLaunchKernelGGL((k_units_fixed<4, true, true, false>), grid, blk, 0, s, a);
        else hipLaunchKernelGGL((k_units_fixed<4, true, false, false>), grid, blk, 0, s, a);
    }
    units_timer_end(s);
    return hipGetLastError();
}

hipError_t launch_segment_once(const FixedArgs& a, int grid_blocks, hipStream_t s, bool arrive) {
    // one record; units_per_rec = 8 units x 16 waves x grid_blocks of at most 2 KiB; fctl, partial,
    // comb_maps (comb blob of the unit) and block_blob (comb blob of 128 units) bound
    if (a.n_rec != 1 || !a.fctl || !a.partial || !a.comb_maps || !a.block_blob || a.rec_bytes < 31 ||
        a.units_per_rec != (uint64_t)grid_blocks * kWavesPerBlock * kGroupsPerWave ||
        a.unit_bytes > segment_once_max_unit(a.arena, a.rec_bytes) || a.unit_bytes % kChunk || grid_blocks > 1024)
        return hipErrorInvalidValue;
    units_timer_begin(s);
    if (arrive)
        hipLaunchKernelGGL((k_segment_once<true, true>), dim3(grid_blocks), dim3(kBlockThreads), 0, s, a);
#ifdef KARMA_AB
    else if (KARMA_AB_KNOB("KARMA_SEGMENT_R8", 0))  // (A/B: the 8-copy stride image)
        hipLaunchKernelGGL((k_segment_once<true, false, true>), dim3(grid_blocks), dim3(kBlockThreads), 0, s, a);
    else if (KARMA_AB_KNOB("KARMA_SEGMENT_WIDE", 0))  // (A/B: the phased window step, step4 MODE 88)
        hipLaunchKernelGGL((k_segment_once<true, false, false, false, true>), dim3(grid_blocks), dim3(kBlockThreads), 0, s, a);
    else if (KARMA_AB_KNOB("KARMA_SEGMENT_LATE", 0))  // (A/B: the workgroup fold's maps behind the chunks)
        hipLaunchKernelGGL((k_segment_once<true, false, false, true>), dim3(grid_blocks), dim3(kBlockThreads), 0, s, a);
#endif
    else
        hipLaunchKernelGGL((k_segment_once<true, false>), dim3(grid_blocks), dim3(kBlockThreads), 0, s, a);
    units_timer_end(s);
    return hipGetLastError();
}

hipError_t launch_combine_fixed(const FixedArgs& a, const uint32_t* in_states, uint64_t k_in, uint32_t* out_states,
                                uint64_t k_out, const uint32_t* comb_blob, hipStream_t s) {
    const uint64_t waves = a.n_rec * k_out;
    uint64_t blocks = (waves + 3) / 4;
    if (blocks > 8192) blocks = 8192;
    hipLaunchKernelGGL(k_combine_fixed, dim3((unsigned)blocks), dim3(256), 0, s, a, in_states, k_in, out_states,
                       k_out, comb_blob);
    return hipGetLastError();
}

hipError_t launch_combine_block(const FixedArgs& a, const uint32_t* in_states, uint64_t k_in, uint64_t m,
                                const uint32_t* block_blob, hipStream_t s) {
    if (a.n_rec == 0) return hipSuccess;
    if (m == 0 || m > kBlockCombMaxPerThread || k_in > m * 1024) return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_combine_block, dim3((unsigned)a.n_rec), dim3(1024), 0, s, a, in_states, k_in, m, block_blob);
    return hipGetLastError();
}

KB_DEFINE_COLLECT(fixed)
#ifdef KARMA_AB
WLOG_SETTER(fixed)
hipError_t set_seg_log(void* p) {
    uint64_t* q = static_cast<uint64_t*>(p);
    return hipMemcpyToSymbol(HIP_SYMBOL(g_seg_log), &q, sizeof(q));
}
#endif

}  // namespace engine
}  // namespace karma
