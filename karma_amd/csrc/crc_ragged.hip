// karma_amd/csrc/crc_ragged.hip -- ragged record batches (offsets + lengths).
//
// Batched form of wal::scan_record's payload check crc32c::Value
// (karma-store/wal.cc:60) and of any Extend over a list of buffers.  Records
// are cut into units of <= unit_bytes (end-aligned to the record's aligned
// body end) so every group of 8 lanes gets at most one unit's worth of work
// regardless of how skewed the record sizes are:
//
//   k_ragged_plan      one thread per record, one pass: unit counts, the slots
//                      of each block of records (a decoupled look-back over the
//                      blocks' unit counts), the entering register over the
//                      unaligned head (crc32c.cc:323-329 analogue) and one
//                      16-byte descriptor {span start, span length, inj} per unit
//                      (round 1's k_ragged_scan + k_ragged_desc in one launch)
//   k_units_ragged     the streaming kernel over the descriptor list: every
//                      wave streams 8 units of (nearly) equal length
//   k_ragged_finalize  one lane per record: Horner fold of its unit
//                      contributions with Z_unit, unaligned tail bytes, ~R;
//                      records with > 64 units are folded by the whole wave
#include <hip/hip_runtime.h>

#include "ab.h"
#include "crc_device.h"
#include "engine.h"
#include "wavelog.h"

namespace karma {
namespace engine {
namespace {

using namespace dev;

constexpr int kRaggedPF = 4;       // chunk loads in flight per lane: small-record and pipelined kernels
constexpr int kRaggedUnitsPF = 6;  // ... and the shipped units kernel (k_units_ragged)
constexpr bool kRaggedNT = true;
// Where a ragged record's unaligned head and tail bytes are stepped (the EM template argument of
// k_ragged_plan / k_units_ragged / k_ragged_finalize): bit 0 = the head in the plan, bit 1 = the
// tail in finalize, bit 2 = the head in finalize; 0 = both in the units kernel (ragged_unit, from the lines it loads).  3 is
// shipped: the units-kernel form saves the plan and finalize 15 us of scattered reads on
// configs[2] but costs the units kernel as much.
constexpr int kShipEM = 3;

static_assert(kScanBlock % 64 == 0 && kScanBlock <= 1024 && kScanBlock >= kBuckets, "scan block shape");
constexpr uint64_t kU = kDefaultUnit;  // ragged units: absolute kU-byte boundaries
constexpr int kUShift = __builtin_ctzll(kDefaultUnit);
static_assert((kU & (kU - 1)) == 0, "unit size is a power of two");

// Unit layout of one record: the aligned body [a, b) cut at absolute multiples
// of U = unit_bytes.  Unit j = [max(a, (A0+j)U), min(b, (A0+j+1)U)), A0 = a/U,
// k = ceil(b/U) - A0.  Only the first and the last unit can be partial.
struct RecUnits {
    Geom g;
    uint64_t k;      // units (0 for short records: finalize does them alone)
    uint64_t full;   // full units
    uint32_t part0;  // 1 if unit 0 is partial
    uint32_t part1;  // 1 if unit k-1 (k >= 2) is partial
    uint32_t c0, c1; // cache lines (chunks) of those partial units
    uint32_t last;   // bytes of the last unit (the last Horner step's distance)
};

__device__ __forceinline__ uint32_t lines_of(const uint8_t* us, const uint8_t* ue) {
    return (uint32_t)((ue - floor128(us) + kChunk - 1) / kChunk);
}

__device__ __forceinline__ RecUnits rec_units(const RaggedArgs& A, uint64_t r) {
    RecUnits u;
    u.g = geom(A.arena + A.off[r], A.len[r]);
    u.k = u.full = 0;
    u.part0 = u.part1 = u.c0 = u.c1 = u.last = 0;
    if (!u.g.is_short) {
        constexpr uint64_t U = kU;
        const uintptr_t a = reinterpret_cast<uintptr_t>(u.g.a), b = reinterpret_cast<uintptr_t>(u.g.b);
        const uint64_t A0 = a >> kUShift, A1 = (b + U - 1) >> kUShift;
        u.k = A1 - A0;
        const uintptr_t e0 = (A0 + 1) * U < b ? (A0 + 1) * U : b;
        u.part0 = (e0 - a) < U ? 1u : 0u;
        if (u.part0) u.c0 = lines_of(u.g.a, reinterpret_cast<const uint8_t*>(e0));
        if (u.k >= 2) {
            const uintptr_t s1 = (A1 - 1) * U;
            u.part1 = (b - s1) < U ? 1u : 0u;
            if (u.part1) u.c1 = lines_of(reinterpret_cast<const uint8_t*>(s1), u.g.b);
            u.last = (uint32_t)(b - s1);
        } else {
            u.last = (uint32_t)(b - a);
        }
        u.full = u.k - u.part0 - u.part1;
    }
    return u;
}

// Inclusive wave scan of 64-bit values.
__device__ __forceinline__ uint64_t wave_incl_scan(uint64_t x) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint64_t t = __shfl_up(x, d);
        if (lane >= d) x += t;
    }
    return x;
}

// Exclusive block scan (blockDim.x a multiple of 64, <= 1024).
__device__ uint64_t block_excl_scan(uint64_t v, uint64_t* sm, uint64_t& total) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
    const uint64_t inc = wave_incl_scan(v);
    if (lane == 63) sm[wave] = inc;
    __syncthreads();
    if (wave == 0) {
        uint64_t s = lane < nw ? sm[lane] : 0;
        s = wave_incl_scan(s);
        if (lane < nw) sm[lane] = s;
    }
    __syncthreads();
    const uint64_t pre = wave ? sm[wave - 1] : 0;
    total = sm[nw - 1];
    __syncthreads();
    return pre + inc - v;
}

// The unit descriptors of the block's records (one thread per record, every lane of the wave
// calls this).  fb: the slot of the record's first full unit; cnt: the block's partial-run
// cursors by chunk count (LDS); full slots at or past full_cap and any slot at or past
// unit_cap are dropped (a caller's total_len too low: k_ragged_finalize steps those records
// alone).  The first unit carries the record's init and head offset, the last its tail length
// (UnitDesc): the plan reads no record bytes.
// (EM, the tools build's KARMA_RAGGED_EDGES: bit 0 = the head in the plan -- the entering
// register h stepped here from the record's head bytes and stored as inj, no kDescFirst --; bit
// 1 = the tail in finalize (no kDescLast).  The shipped library has EM = 0.)
template <int EM = 0>
__device__ void write_unit_descs(const RaggedArgs& A, const RecUnits& u, bool valid, uint64_t r, uint64_t fb,
                                 unsigned long long* cnt, uint64_t full_cap, uint32_t h = 0) {
    const uint32_t lane = threadIdx.x & 63u;
    const uintptr_t a = reinterpret_cast<uintptr_t>(u.g.a), b = reinterpret_cast<uintptr_t>(u.g.b);
    const uint64_t A0 = a >> kUShift;
    uint32_t init = 0, hoff = 0, t = 0;
    if (valid) {
        A.fbase[r] = fb;
        init = A.init ? A.init[r] : A.init_scalar;
        hoff = (uint32_t)(reinterpret_cast<uintptr_t>(A.arena + A.off[r]) & 15u);
        t = (uint32_t)(u.g.e - u.g.b);
        if (EM & 1) {
            init = h;
            hoff = 0;
        }
        if (EM & 4) {  // the head is finalize's: no entering register in the units
            init = 0;
            hoff = 0;
        }
        if (EM & 2) t = 0;
        if (u.part0) {
            const uint64_t slot = atomicAdd(&cnt[u.c0], 1ull);
            A.pslot[2 * r] = slot;
            const uintptr_t e0 = ((A0 + 1) << kUShift) < b ? ((A0 + 1) << kUShift) : b;
            if (slot < A.unit_cap)
                A.desc[slot] = UnitDesc{(uint64_t)a, (uint32_t)(e0 - a) | desc_flags(!(EM & 5), hoff, !(EM & 2) && u.k == 1, t), init};
        }
        if (u.part1) {
            const uint64_t slot = atomicAdd(&cnt[u.c1], 1ull);
            A.pslot[2 * r + 1] = slot;
            const uintptr_t s1 = (A0 + u.k - 1) << kUShift;
            if (slot < A.unit_cap)
                A.desc[slot] = UnitDesc{(uint64_t)s1, (uint32_t)(b - s1) | desc_flags(false, 0, !(EM & 2), t), 0u};
        }
    }
    // Full units of the wave's 64 records are consecutive slots: the wave writes them together,
    // lane i taking slot F0 + i and finding its record by a search over the lanes' inclusive
    // unit counts, so the stores are coalesced and balanced however skewed the record sizes are.
    const uint64_t nfull = valid ? u.full : 0;
    const uint64_t incl = wave_incl_scan(nfull);
    const uint64_t T = __shfl(incl, 63);
    const uint64_t F0 = __shfl(fb, 0);
    for (uint64_t base = 0; base < T; base += 64) {  // uniform trip count: shuffles see every lane
        const uint64_t i = base + lane;
        int o = 0;  // owner: the first lane whose inclusive count exceeds i
#pragma unroll
        for (int s = 32; s > 0; s >>= 1)
            if (__shfl(incl, o + s - 1) <= i) o += s;
        o = o < 63 ? o : 63;
        const uint64_t incl_o = __shfl(incl, o), full_o = __shfl(nfull, o), A0_o = __shfl(A0, o), k_o = __shfl(u.k, o);
        const uint32_t part0_o = __shfl(u.part0, o), part1_o = __shfl(u.part1, o);
        const uint32_t init_o = __shfl(init, o), hoff_o = __shfl(hoff, o), t_o = __shfl(t, o);
        const uint64_t j = i - (incl_o - full_o) + part0_o;  // unit index within the owner's record
        const uint64_t slot = F0 + i;
        if (i < T && slot < full_cap)
            A.desc[slot] = UnitDesc{(A0_o + j) << kUShift,
                                    (uint32_t)kU | desc_flags(!(EM & 5) && j == 0, hoff_o, !(EM & 2) && !part1_o && j + 1 == k_o, t_o),
                                    j == 0 ? init_o : 0u};
    }
}

// Per scan block: exclusive scan of full units (record order), and the
// block's totals of full and partial units (block_sums / block_psums).
// k_ragged_desc turns the block totals into slots: full units take [0, F) in
// record order; block b's partial units take the run [F + P_b, F + P_b +
// parts_b), sorted by chunk count, longest first (a wave's 8 units then have
// nearly equal length).
__global__ __launch_bounds__(kScanBlock) void k_ragged_scan(RaggedArgs A) {
    __shared__ uint64_t sm[16];
    const uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    RecUnits u{};
    if (r < A.n_rec) u = rec_units(A, r);
    uint64_t total, parts;
    const uint64_t ex = block_excl_scan(r < A.n_rec ? u.full : 0, sm, total);  // has barriers
    (void)block_excl_scan(r < A.n_rec ? u.part0 + u.part1 : 0, sm, parts);
    if (r < A.n_rec) A.fbase[r] = ex;
    if (threadIdx.x == 0) {
        A.block_sums[blockIdx.x] = total;
        A.block_psums[blockIdx.x] = parts;
    }
}

#ifdef KARMA_AB  // the two-pass plan (k_ragged_scan + k_ragged_desc): tools build, KARMA_RAGGED_PLAN=2
// Block b's full-unit prefix, its partial-unit prefix and the grand totals,
// reduced from the scan's block totals by every desc block (nb loads per
// block: cheaper than another launch or a grid-wide fence).
struct BlockBase {
    uint64_t full_pre, part_pre, F, P;
};

__device__ BlockBase block_base(const RaggedArgs& A, uint64_t* sm) {
    const uint64_t nb = gridDim.x, b = blockIdx.x;
    uint64_t fp = 0, pp = 0, ft = 0, pt = 0;
    for (uint64_t i = threadIdx.x; i < nb; i += blockDim.x) {
        const uint64_t f = A.block_sums[i], p = A.block_psums[i];
        ft += f;
        pt += p;
        if (i < b) {
            fp += f;
            pp += p;
        }
    }
    uint64_t v[4] = {fp, pp, ft, pt};
#pragma unroll
    for (int k = 0; k < 4; ++k)
#pragma unroll
        for (int d = 32; d > 0; d >>= 1) v[k] += __shfl_xor(v[k], d);
    const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
    if (lane < 4) sm[wave * 4 + lane] = lane == 0 ? v[0] : lane == 1 ? v[1] : lane == 2 ? v[2] : v[3];
    __syncthreads();
    BlockBase B{0, 0, 0, 0};
    for (uint32_t w = 0; w < nw; ++w) {
        B.full_pre += sm[w * 4 + 0];
        B.part_pre += sm[w * 4 + 1];
        B.F += sm[w * 4 + 2];
        B.P += sm[w * 4 + 3];
    }
    return B;
}

// One thread per record (block b = scan block b): final slots, the entering
// register over the unaligned head, and the unit descriptors.  The block's
// partial units fill its run from k_ragged_scan sorted by chunk count (a
// counting sort in LDS); each lane writes its record's (at most two).  The full units of a
// wave's 64 records are consecutive slots: the wave writes them together, lane
// t taking slot F0 + t and finding its record by a search over the lanes'
// inclusive unit counts, so the descriptor stores are coalesced and balanced
// however skewed the record sizes are.
__global__ __launch_bounds__(kScanBlock) void k_ragged_desc(RaggedArgs A) {
    __shared__ unsigned long long cnt[kBuckets];
    __shared__ uint32_t hist[kBuckets];
    __shared__ uint64_t sm[4 * (kScanBlock / 64)];
    if (threadIdx.x < kBuckets) hist[threadIdx.x] = 0;
    const BlockBase B = block_base(A, sm);  // has a barrier
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        A.fbase[A.n_rec] = B.F + B.P;  // total units
        A.fbase[A.n_rec + 1] = B.F;
    }
    const uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const bool valid = r < A.n_rec;
    RecUnits u{};
    if (valid) {
        u = rec_units(A, r);
        if (u.part0) atomicAdd(&hist[u.c0], 1u);
        if (u.part1) atomicAdd(&hist[u.c1], 1u);
    }
    __syncthreads();
    if (threadIdx.x == 0) {  // the block's partial run, longest bucket first
        unsigned long long s = B.F + B.part_pre;
        for (int c = kBuckets - 1; c >= 0; --c) {
            cnt[c] = s;
            s += hist[c];
        }
    }
    __syncthreads();
    const uint64_t fb = valid ? A.fbase[r] + B.full_pre : 0;
    write_unit_descs(A, u, valid, r, fb, cnt, A.unit_cap);
}

#endif  // KARMA_AB

// ---- the single-pass plan ----------------------------------------------------
// Block status words for the decoupled look-back (RaggedArgs::lb): seq << 42 | flag << 40 |
// value.  The words are read and written with agent-scope atomics (cache-coherent across
// the XCDs); nothing else a block writes is read by another block of the same launch, so no
// release fence is needed (on gfx950 one would write back the XCD's L2).
constexpr uint64_t kLbValueMask = (1ull << 40) - 1;
constexpr uint64_t kLbAgg = 1ull << 40, kLbIncl = 2ull << 40;

__device__ __forceinline__ void lb_store(unsigned long long* p, uint64_t v) {
    __hip_atomic_store(p, (unsigned long long)v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint64_t lb_load(unsigned long long* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// One look-back step for one status array: lane l holds the word of block j - l (blocks
// before 0: an inclusive total of 0).  Adds the values of lanes 0..k, k the first lane holding
// an inclusive total (all 64 if none), to excl; true when one was found.
__device__ __forceinline__ bool lb_take(uint64_t w, uint64_t& excl) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint64_t incl = __ballot(((w >> 40) & 3u) == 2u);
    const uint32_t k = incl ? (uint32_t)(__ffsll((long long)incl) - 1) : 63u;
    uint64_t v = lane <= k ? (w & kLbValueMask) : 0;
#pragma unroll
    for (int d = 32; d > 0; d >>= 1) v += __shfl_xor(v, d);
    excl += v;
    return incl != 0;
}

__device__ __forceinline__ uint64_t lb_wait(unsigned long long* p, uint32_t seq) {
    uint64_t w = lb_load(p);
    while ((w >> 42) != seq) {  // not published yet (this call's tag)
        __builtin_amdgcn_s_sleep(1);
        w = lb_load(p);
    }
    return w;
}

// Wave 0 of plan block b: publish the block's full and partial unit counts, sum the counts
// of the blocks before it (256 per step, newest first, each array until the first block that
// has published its inclusive total there), publish the inclusive totals and return the
// exclusive ones (uniform).  Every block it waits for has started (ids are taken in start
// order) and publishes its own counts before waiting on anything, so the wait ends.
__device__ void lookback(const RaggedArgs& A, uint32_t seq, uint64_t b, uint64_t full_b, uint64_t part_b,
                         uint64_t& exF, uint64_t& exP) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint64_t tag = (uint64_t)seq << 42;
    unsigned long long* lf = A.lb + 1;
    unsigned long long* lp = A.lbp;
    exF = exP = 0;
    if (b > 0) {
        if (lane == 0) {
            lb_store(lf + b, tag | kLbAgg | full_b);
            lb_store(lp + b, tag | kLbAgg | part_b);
        }
        // 256 blocks per step: every lane's 4 loads go out together (an inclusive total
        // travels back 256 blocks per memory round trip instead of 64), then the windows are
        // taken nearest first; a word is waited for only if its window is reached.
        constexpr int kLbWin = 4;
        bool doneF = false, doneP = false;
        for (int64_t j = (int64_t)b - 1; !(doneF && doneP); j -= 64 * kLbWin) {
            uint64_t wf[kLbWin], wp[kLbWin];
#pragma unroll
            for (int q = 0; q < kLbWin; ++q) {
                const int64_t i = j - (int64_t)lane - 64 * q;
                wf[q] = wp[q] = tag | kLbIncl;  // before block 0: an inclusive total of 0
                if (i >= 0) {
                    if (!doneF) wf[q] = lb_load(lf + i);
                    if (!doneP) wp[q] = lb_load(lp + i);
                }
            }
#pragma unroll
            for (int q = 0; q < kLbWin; ++q) {
                const int64_t i = j - (int64_t)lane - 64 * q;
                if (!doneF) {
                    if (i >= 0 && (wf[q] >> 42) != seq) wf[q] = lb_wait(lf + i, seq);
                    doneF = lb_take(wf[q], exF);
                }
                if (!doneP) {
                    if (i >= 0 && (wp[q] >> 42) != seq) wp[q] = lb_wait(lp + i, seq);
                    doneP = lb_take(wp[q], exP);
                }
            }
        }
    }
    if (lane == 0) {
        lb_store(lf + b, tag | kLbIncl | (exF + full_b));
        lb_store(lp + b, tag | kLbIncl | (exP + part_b));
    }
}

// The single-pass plan's look-back words after the call (the first thing k_ragged_finalize
// does; the plan has finished, stream order): the block counter back to 0 and the finished
// call's tag into lb_ctl[0], so the next plan -- also a replay of a captured graph -- takes
// fresh ids and the next tag.  When the tags run out every status word is cleared (each
// finalize thread a stride of them) and they restart at 1.  Every block writes the same values.
__device__ void lookback_retire(const RaggedArgs& A) {
    const uint32_t seq = (uint32_t)lb_load(A.lb_ctl + 1);
    const bool wrap = seq + 1u >= A.lb_seq_max;
    if (wrap) {
        const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
        for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < A.lb_words; i += stride)
            lb_store(A.lb + 1 + i, 0ull);
    }
    // one workgroup writes the control words: hundreds of workgroups storing the same words
    // queue at the memory side (it cost the call ~30 us)
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        lb_store(A.lb, 0ull);
        lb_store(A.lb_ctl, wrap ? 0ull : (unsigned long long)seq);
        lb_store(A.lb_ctl + 2, 0ull);  // the longest partial run (the tools build's rank-major order)
    }
}

// One pass over the records (one thread per record, plan block b = kScanBlock records):
// unit counts, the slots of the block's units from the look-back, the entering register
// over each record's unaligned head, and one 16-byte descriptor per unit.  Full units take
// slots [0, F) in record order; partial units [part_base, part_base + P), each block's run
// sorted by chunk count, longest first (the two-pass plan's order, which the units kernel
// streams 3 % faster on configs[2] than block-interleaved runs).  Replaces k_ragged_scan +
// k_ragged_desc: one launch, and no block reads every other block's totals.
template <int EM = 0>
__global__ __launch_bounds__(kScanBlock) void k_ragged_plan(RaggedArgs A) {
    KB_SET_ARENA(A.kb_lo, A.kb_hi);
    constexpr bool HP = (EM & 1) != 0;
    __shared__ __attribute__((aligned(16))) uint32_t lds[HP ? kCombCoreWords - kCombZ4 : 4];  // HP: Z4, byte table
    __shared__ unsigned long long cnt[kBuckets];
    __shared__ uint32_t hist[kBuckets];
    __shared__ uint64_t sm[kScanBlock / 64];
    __shared__ uint64_t s_id, s_fbase;
    __shared__ uint32_t s_seq;
    if (threadIdx.x == 0) {
        s_id = atomicAdd(A.lb, 1ull);  // ids in start order (k_ragged_finalize resets the counter)
        s_seq = (uint32_t)lb_load(A.lb_ctl) + 1u;  // this call's tag (RaggedArgs::lb_ctl)
        if (s_id == 0) lb_store(A.lb_ctl + 1, s_seq);
    }
    if constexpr (HP) copy_to_lds<kCombCoreWords - kCombZ4, kScanBlock>(lds, A.comb_blob + kCombZ4);
    if (threadIdx.x < kBuckets) hist[threadIdx.x] = 0;
    __syncthreads();
    const uint64_t b = s_id;
    const uint64_t r = b * kScanBlock + threadIdx.x;
    const bool valid = r < A.n_rec;
    RecUnits u{};
    if (valid) {
        u = rec_units(A, r);
        if (u.part0) atomicAdd(&hist[u.c0], 1u);
        if (u.part1) atomicAdd(&hist[u.c1], 1u);
    }
    // full units (high bits) and partial units (low 16 bits: at most 2 per record) in one scan
    const uint64_t packed = valid ? (u.full << 16) | (u.part0 + u.part1) : 0;
    uint64_t tot;
    const uint64_t ex = block_excl_scan(packed, sm, tot) >> 16;  // has barriers (hist complete after)
    const uint64_t full_b = tot >> 16, part_b = tot & 0xffffu;
    if (threadIdx.x < 64) {
        uint64_t exF, exP;
        lookback(A, s_seq, b, full_b, part_b, exF, exP);
        if (threadIdx.x == 0) {
            s_fbase = exF;
            unsigned long long s = A.part_base + exP;  // the block's partial run, longest bucket first
            for (int c = kBuckets - 1; c >= 0; --c) {
                cnt[c] = s;
                s += hist[c];
            }
            if (b + 1 == gridDim.x) {
                A.fbase[A.n_rec] = exF + full_b + exP + part_b;  // total units
                A.fbase[A.n_rec + 1] = exF + full_b;             // full units
            }
            // the block's partial run (first slot after part_base, length) and the longest run:
            // the units kernel's rank-major order (k_units_ragged_pipe, RM)
            A.block_psums[b] = (exP << 16) | part_b;
#ifdef KARMA_AB  // (the rank-major variants' longest run: one atomic per plan block, tools build only)
            atomicMax(A.lb_ctl + 2, (unsigned long long)part_b);
#endif
        }
    }
    uint32_t h = 0;
    if (HP && valid && u.k) h = head_register(lds, 0, 1024, A.arena + A.off[r], u.g, A.init ? A.init[r] : A.init_scalar);
    __syncthreads();
    write_unit_descs<EM>(A, u, valid, r, s_fbase + ex, cnt, A.part_base, h);
}

// Units of the batch in streaming order: u in [0, U).  Full units are slots [0, F); the
// partial units follow at part_base (the single-pass plan; 0 = the two-pass plan, whose
// partial units follow the full ones directly).  Slots past the table (a caller's total_len
// too low) are left out; k_ragged_finalize steps their records alone.
struct UnitMap {
    uint64_t U, Fc, shift;
    __device__ __forceinline__ uint64_t slot(uint64_t u) const { return u < Fc ? u : u + shift; }
};
__device__ __forceinline__ UnitMap unit_map(const RaggedArgs& A) {
    UnitMap m;
    const uint64_t all = A.fbase[A.n_rec];
    if (!A.part_base) {
        m.U = m.Fc = all < A.unit_cap ? all : A.unit_cap;
        m.shift = 0;
    } else {
        const uint64_t F = A.fbase[A.n_rec + 1], P = all - F, pcap = A.unit_cap - A.part_base;
        m.Fc = F < A.part_base ? F : A.part_base;
        m.U = m.Fc + (P < pcap ? P : pcap);
        m.shift = A.part_base - m.Fc;
    }
    return m;
}

// Descriptor load through address space 1 (global_load_dwordx4, vmcnt only): a
// flat load would also count on lgkmcnt and stall the LDS lookups behind it.
__device__ __forceinline__ UnitDesc load_desc(const UnitDesc* d) {
    const u32x4 v = ldmeta16(d);
    return UnitDesc{v.x | ((uint64_t)v.y << 32), v.z, v.w};
}

// Register contribution of one ragged unit (d, UnitDesc) to its record: group_unit's
// streaming loop, plus the record's edges taken from the lines the unit loads anyway.
//   head (kDescFirst): the lane whose chunk-0 window is the body's first one loads the
//     16-byte block before it (the same cache line unless the body starts on a line), steps
//     ~init over the head bytes and xors the result into the body's first word;
//   tail (kDescLast): group lane 0 loads the block at the body end (usually in the unit's
//     last line) and steps a zero register over the tail bytes: tail (valid where tail_here)
//     = that register, and
//     the record's CRC is ~(Z_t(R_b) ^ *tail), R_b its register at the body end
//     (k_ragged_finalize applies Z_t).
// The edge loads are issued before the body's, by the lanes that need them, and the edge
// steps depend on them only, so they run while the body's loads are in flight (vmcnt counts
// in issue order); the epilogue after the group tree has no extra work.  The contribution is
// valid in group lane 0; every lane of the wave must call this.
template <int PF, bool NT, bool HP = false>  // HP: the plan stepped the head (inj = the register)
__device__ __forceinline__ uint32_t ragged_unit(const uint32_t* lds, uint32_t X, uint32_t l, const UnitDesc& d,
                                                uint32_t& tail, bool& tail_here) {
    const uint8_t* us = reinterpret_cast<const uint8_t*>(d.us);
    const uint8_t* ue = us + (d.span & kDescBytes);
    const bool first = (d.span & kDescFirst) != 0, last = (d.span & kDescLast) != 0;
    const uint32_t hoff = (d.span >> 17) & 15u, t = (d.span >> 22) & 15u;
    uint32_t a0 = 0, a1 = 0, a2 = 0, a3 = 0;
    uint32_t m = kGroupLanes - 1;
    tail = 0;
    tail_here = false;
    if (ue > us) {
        const uint8_t* base = floor128(us);
        const int64_t nch = (ue - base + kChunk - 1) / kChunk;
        m = (uint32_t)((reinterpret_cast<uintptr_t>(ue) - 16) >> 4) & (kGroupLanes - 1);
        const uint8_t* w = base + 16 * l;
        const uint8_t* const w0 = w;  // this lane's chunk-0 window
        const uint8_t* wl = base + (nch - 1) * kChunk + 16 * l;
        const bool lok = wl < ue;
        const uint8_t* lclamp = lok ? wl : ue - 16;
        // The head lane holds the body's first window, the tail lane is group lane 0.  (Putting
        // the tail 4 lanes from the head, so that one load and one divergent step loop serve
        // both edges, measured slower: 0.821 vs 0.797 ms units on 1-1.5 KiB records.  The loads
        // are lane-masked: an unmasked pair at safe addresses costs every lane two 16-byte
        // requests per unit, 2.5 % of the kernel on 4 KiB records.)
        const bool hl = first && hoff != 0 && w == us;
        const bool tl = last && t != 0 && l == 0;
        tail_here = tl;
        u32x4 hv = {0u, 0u, 0u, 0u}, tv = {0u, 0u, 0u, 0u};
        if (hl) hv = ld16(us - 16);
        if (tl) tv = ld16(ue);
        const bool ok = w >= us && w < ue;
        u32x4 v = ok ? ldg<NT>(w) : u32x4{0u, 0u, 0u, 0u};
        int64_t rem = nch - 1;
        w += kChunk;
        u32x4 nb[PF];
#pragma unroll
        for (int q = 0; q < PF; ++q) nb[q] = ldg<NT>(pmin(w + q * kChunk, lclamp));
        // The edge steps and chunk 0's registers are taken after the next batch's loads are
        // issued: waiting for chunk 0 (or an edge block) before that issue would leave one
        // batch fewer in flight at every unit start (measured: 1.7 % on 4 KiB records).
        auto edges = [&]() {
            uint32_t h = ~d.inj;
            if (hl) h = steps_in_vec(lds, kLZ4, kLT8, h, hv, hoff, 16u);
            if (tl) tail = steps_in_vec(lds, kLZ4, kLT8, 0u, tv, 0u, t);
            if (HP) {
                if (w0 == us) v.x ^= d.inj;  // (0 for all but a record's first unit)
            } else if (first && w0 == us) {
                v.x ^= h;
            }
            a0 = v.x;
            a1 = v.y;
            a2 = v.z;
            a3 = v.w;
        };
        auto batch = [&]() {  // step the PF chunks in flight, with the next PF issued first
            u32x4 cur[PF];
#pragma unroll
            for (int q = 0; q < PF; ++q) cur[q] = nb[q];
            w += PF * kChunk;
#pragma unroll
            for (int q = 0; q < PF; ++q) nb[q] = ldg<NT>(pmin(w + q * kChunk, lclamp));
            return [&, cur]() {
#pragma unroll
                for (int q = 0; q < PF; ++q) step4(lds, X, a0, a1, a2, a3, cur[q]);
                rem -= PF;
            };
        };
        if (rem > PF) {  // the first batch, peeled: the edges go between its issue and its steps
            auto steps = batch();
            __builtin_amdgcn_sched_barrier(0);
            edges();
            steps();
        } else {
            edges();
        }
        while (rem > PF) batch()();
#pragma unroll
        for (int q = 0; q < PF; ++q) {
            if (q < rem - 1 || (q == rem - 1 && lok)) step4(lds, X, a0, a1, a2, a3, nb[q]);
        }
    }
    uint32_t c = lane_fold(lds, a0, a1, a2, a3);
    const uint32_t lane = threadIdx.x & 63u;
    c = __shfl(c, (int)((lane & ~(kGroupLanes - 1u)) | ((l + m + 1) & (kGroupLanes - 1))), 64);
    uint32_t t1 = __shfl_down(c, 1, kGroupLanes);
    c = zmap(lds, kLZ16, c) ^ t1;
    t1 = __shfl_down(c, 2, kGroupLanes);
    c = zmap(lds, kLZ32, c) ^ t1;
    t1 = __shfl_down(c, 4, kGroupLanes);
    c = zmap(lds, kLZ64, c) ^ t1;
    return c;
}

// The units kernel: each unit's loads are issued when the unit starts (ragged_unit), the
// next descriptor is in flight meanwhile.  (A software-pipelined form, stream_unit's, measured
// 0.3-0.8 % slower on config 3 in round 2, unlike the fixed layout, where it wins 2.7 %:
// DESIGN.md §4.)
// PF = 6 chunk loads in flight per lane (4: config 3 units 0.6736 vs 0.6680 ms, aligned 4 KiB
// records 0.6656 vs 0.6525; 8: no better than 4 -- profiles/r02_ragged_pf_ab.txt).  With one
// 1024-thread workgroup per CU (the 145 KiB LDS image) the chunks in flight per CU are what
// keeps HBM busy across the unit boundaries this kernel does not pipeline.
template <bool BAL = true, int PF = kRaggedUnitsPF, int EM = kShipEM>
__global__ __launch_bounds__(kBlockThreads) void k_units_ragged(RaggedArgs A) {
    KB_SET_ARENA(A.kb_lo, A.kb_hi);
    __shared__ __attribute__((aligned(16))) uint32_t lds[kLdsWords];
    __shared__ uint32_t blk_next;  // BAL: the block's next wave-step (an LDS counter)
    if (BAL && threadIdx.x == 0) blk_next = kWavesPerBlock;
    load_stream_tables(lds, A.blob);
    __syncthreads();
    WLOG_DECL;
    WLOG_START();
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t l = lane & (kGroupLanes - 1);
    const uint32_t grp = lane / kGroupLanes;
    const uint32_t X = lane_const();
    const UnitMap M = unit_map(A);
    const uint64_t U = M.U;
    const uint64_t nwaves = (uint64_t)gridDim.x * kWavesPerBlock;
    // BAL: as k_units_fixed, the block's wave-steps b*16 + j + r*nwaves are taken in order from
    // an LDS counter, one step ahead (the next descriptor is loaded while a unit streams).
    const uint64_t nws = (U + kGroupsPerWave - 1) / kGroupsPerWave;
    const uint32_t nidx = (uint32_t)((nws + nwaves - 1) / nwaves) * kWavesPerBlock;
    const uint64_t bw0 = (uint64_t)blockIdx.x * kWavesPerBlock;
    uint64_t wb = bw0 + (threadIdx.x >> 6);
    uint64_t u = wb * kGroupsPerWave + grp;
    UnitDesc d = u < U ? load_desc(A.desc + M.slot(u)) : UnitDesc{0, 0, 0};
    while (wb < nws) {
        const UnitDesc cur = d;
        const bool valid = u < U;
        uint64_t wb_next = wb + nwaves;
        if constexpr (BAL) {
            uint32_t i = 0;
            if (lane == 0) i = atomicAdd(&blk_next, 1u);
            i = __builtin_amdgcn_readfirstlane(__shfl(i, 0));
            wb_next = i < nidx ? bw0 + (i % kWavesPerBlock) + (uint64_t)(i / kWavesPerBlock) * nwaves : nws;
        }
        const uint64_t un = wb_next * kGroupsPerWave + grp;
        d = un < U ? load_desc(&KB_READ(A.desc, M.slot(un), A.unit_cap, kKbUnit)) : UnitDesc{0, 0, 0};
        uint32_t tail = 0, R;
        bool tail_here = false;
        if constexpr ((EM & 2) && (EM & 5)) {  // neither edge in the units kernel
            const uint8_t* us = reinterpret_cast<const uint8_t*>(cur.us);
            R = group_unit<PF, kRaggedNT>(lds, X, l, us, us + cur.span, us, cur.inj);
        } else {
            R = ragged_unit<PF, kRaggedNT, (EM & 1) != 0>(lds, X, l, cur, tail, tail_here);
        }
        if (valid && l == 0) KB_WRITE(A.partial, M.slot(u), A.unit_cap, kKbUnit, R);
        if (valid && tail_here) KB_WRITE(A.tailc, M.slot(u), A.unit_cap, kKbUnit, tail);
        WLOG_STEP();
        WLOG_UNIT(valid && l == 0, cur.span & kDescBytes);
        wb = wb_next;
        u = un;
    }
    WLOG_END(bw0 + (threadIdx.x >> 6));
}


// The units kernel, software-pipelined across units (stream_unit, as k_units_fixed): the
// next wave-step's descriptor is loaded when the current unit starts (its slot taken from
// the block's LDS counter), and that unit's first chunk loads go out before the current
// unit's last batch is stepped, so a wave never drains its loads at a unit boundary.  The
// per-wave log (tools/ragged_gap.py) showed the unpipelined kernel streaming configs[2] at
// 6.85 TB/s in steady state against 7.52 for the pipelined fixed kernel (and 6.73 for the
// fixed kernel without pipelining, k_units_fixed_v1).  Edges as kShipEM: the plan steps each
// record's head (desc.inj), finalize its tail.  Units past the table point at the table blob
// (always mapped, 16-byte aligned): every load is issued unconditionally.
// Rank-major order of the partial units (RM): the plan leaves each plan block's partial run
// sorted longest first; the units kernel takes rank 0 of every block's run, then rank 1, ...
// (unit Fc + k is rank k / nb of block k % nb; ranks past a run's end are empty), so the
// wave-steps come in nearly descending cost and the static round robin over the CUs ends
// with the shortest units everywhere.  In slot order (block after block) the last steps held
// the last plan blocks' longest partial units: the per-wave log on configs[2] showed the wave
// end times spread over 126 us against 51 for fixed records (tools/ragged_gap.py).
// RM 2 (tail only): slot order up to the partial runs of the last `tail_blocks` plan blocks,
// rank-major over those (b0 = their first block, T0 = the partial slots before them, L their
// longest run): the locality of slot order everywhere but in the last few percent of the work.
struct RankMap {
    uint64_t Fc, nb, U;  // full units streamed, plan blocks in the rank-major part, units in streaming order
    uint64_t b0, T0;     // first rank-major block, partial units before it (slot order)
    __device__ __forceinline__ bool slot(const RaggedArgs& A, uint64_t u, uint64_t& s) const {
        if (u < Fc + T0) {
            s = u < Fc ? u : A.part_base + (u - Fc);
            return u < Fc || s < A.unit_cap;
        }
        const uint64_t k = u - Fc - T0, i = k / nb, b = b0 + (k - i * nb);
        const uint64_t run = __ldg(reinterpret_cast<const unsigned long long*>(A.block_psums) + b);
        s = A.part_base + (run >> 16) + i;
        return i < (run & 0xffffu) && s < A.unit_cap;
    }
};
template <int RM>
__device__ __forceinline__ RankMap rank_map(const RaggedArgs& A, uint64_t tail_blocks) {
    RankMap m;
    const uint64_t F = A.fbase[A.n_rec + 1];
    m.Fc = F < A.part_base ? F : A.part_base;
    const uint64_t nb = (A.n_rec + kScanBlock - 1) / kScanBlock;
    if (RM == 1 || tail_blocks >= nb) {
        m.b0 = 0;
        m.T0 = 0;
        m.nb = nb;
        m.U = m.Fc + m.nb * __hip_atomic_load(A.lb_ctl + 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        return m;
    }
    m.nb = tail_blocks;
    m.b0 = nb - tail_blocks;
    const unsigned long long* pr = reinterpret_cast<const unsigned long long*>(A.block_psums);
    m.T0 = pr[m.b0] >> 16;
    uint64_t L = 0;
    for (uint64_t b = m.b0; b < nb; ++b) L = (pr[b] & 0xffffu) > L ? (pr[b] & 0xffffu) : L;  // uniform: scalar loads
    m.U = m.Fc + m.T0 + m.nb * L;
    return m;
}

template <int PF = kRaggedPF, int RM = 0>
__global__ __launch_bounds__(kBlockThreads) void k_units_ragged_pipe(RaggedArgs A) {
    KB_SET_ARENA_SAFE(A.kb_lo, A.kb_hi, A.blob, A.blob + kBlobWords);
    __shared__ __attribute__((aligned(16))) uint32_t lds[kLdsWords];
    __shared__ uint32_t blk_next;
    if (threadIdx.x == 0) blk_next = kWavesPerBlock;
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t l = lane & (kGroupLanes - 1);
    const uint32_t grp = lane / kGroupLanes;
    const uint32_t X = lane_const();
    const UnitMap M = unit_map(A);
    const RankMap RMap = RM ? rank_map<RM>(A, A.tail_blocks) : RankMap{0, 1, 0, 0, 0};
    const uint64_t U = RM ? RMap.U : M.U;
    const uint64_t nwaves = (uint64_t)gridDim.x * kWavesPerBlock;
    const uint64_t nws = (U + kGroupsPerWave - 1) / kGroupsPerWave;
    const uint32_t nidx = (uint32_t)((nws + nwaves - 1) / nwaves) * kWavesPerBlock;
    const uint64_t bw0 = (uint64_t)blockIdx.x * kWavesPerBlock;
    const uint8_t* safe = reinterpret_cast<const uint8_t*>(A.blob);
    uint64_t wb = bw0 + (threadIdx.x >> 6);
    uint64_t u = wb * kGroupsPerWave + grp;
    auto unit_of = [&](const UnitDesc& d, bool valid) {
        const uint8_t* us = valid ? reinterpret_cast<const uint8_t*>(d.us) : safe;
        return lane_unit(us, valid ? us + d.span : safe, l);
    };
    // unit u's slot (valid: a unit of the table, else an empty step)
    auto slot_of = [&](uint64_t uu, uint64_t& s) {
        if (uu >= U) return false;
        if constexpr (RM) return RMap.slot(A, uu, s);
        s = M.slot(uu);
        return true;
    };
    // the first unit: its descriptor, then its loads in flight over the table fill
    uint64_t su = 0;
    bool valid = slot_of(u, su);
    UnitDesc d = valid ? load_desc(A.desc + su) : UnitDesc{0, 0, 0};
    LaneUnit L = unit_of(d, valid);
    UnitLoads<PF> Ld;
    issue_unit_loads<PF, kRaggedNT>(L, Ld);
    load_stream_tables(lds, A.blob);
    __syncthreads();
    WLOG_DECL;
    WLOG_START();
    while (wb < nws) {
        uint64_t wb_next;
        {
            uint32_t i = 0;
            if (lane == 0) i = atomicAdd(&blk_next, 1u);
            i = __builtin_amdgcn_readfirstlane(__shfl(i, 0));
            wb_next = i < nidx ? bw0 + (i % kWavesPerBlock) + (uint64_t)(i / kWavesPerBlock) * nwaves : nws;
        }
        const uint64_t un = wb_next * kGroupsPerWave + grp;
        uint64_t sn = 0;
        const bool vn = slot_of(un, sn);
        const UnitDesc dn = vn ? load_desc(&KB_READ(A.desc, sn, A.unit_cap, kKbUnit)) : UnitDesc{0, 0, 0};
        LaneUnit N = L;
        const uint32_t R = stream_unit<PF, kRaggedNT>(lds, X, l, L, Ld, L.us, d.inj, [&](UnitLoads<PF>& nx) {
            N = unit_of(dn, vn);
            issue_unit_loads<PF, kRaggedNT>(N, nx);
        });
        if (valid && l == 0) KB_WRITE(A.partial, su, A.unit_cap, kKbUnit, R);
        WLOG_STEP();
        WLOG_UNIT(valid && l == 0, d.span);
        wb = wb_next;
        u = un;
        su = sn;
        valid = vn;
        d = dn;
        L = N;
    }
    WLOG_END(bw0 + (threadIdx.x >> 6));
}

// Slot of unit j of a record (full units from fb in order, partial ones bucketed).
__device__ __forceinline__ uint64_t unit_slot(uint64_t j, uint64_t k, uint64_t fb, uint64_t ps0, uint64_t ps1,
                                              uint32_t part0, uint32_t part1) {
    if (j == 0 && part0) return ps0;
    if (j == k - 1 && part1) return ps1;
    return fb + j - part0;
}

// Last Horner step over a unit of `last` bytes (== U: the table of Z_U).
__device__ __forceinline__ uint32_t shift_last(const uint32_t* lds, uint32_t x, uint32_t last, uint64_t U) {
    return last == U ? zmap(lds, 0, x) : zshift16(lds, x, last / 16);
}

// One lane per record: Horner fold of the unit contributions (Z_U between unit
// ends, Z_last before the last unit), the unaligned tail, ~R.  Records of more
// than 64 units: the whole wave folds all but the last unit with the 64-lane tree.
template <int EM = 0>
__global__ __launch_bounds__(1024) void k_ragged_finalize(RaggedArgs A) {
    KB_SET_ARENA(A.kb_lo, A.kb_hi);
    __shared__ __attribute__((aligned(16))) uint32_t lds[kCombWords];
    if (A.lb) lookback_retire(A);
    load_comb_tables<kCombWords, 1024>(lds, A.comb_blob);
    __syncthreads();
    const uint32_t lane = threadIdx.x & 63u;
    constexpr uint64_t U = kU;
    const uint64_t nwaves = (uint64_t)gridDim.x * (blockDim.x >> 6);
    for (uint64_t r0 = ((uint64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6)) * 64; r0 < A.n_rec;
         r0 += nwaves * 64) {
        const uint64_t r = r0 + lane;
        const bool valid = r < A.n_rec;
        RecUnits u{};
        uint64_t fb = 0, ps0 = 0, ps1 = 0;
        uint32_t init = 0;
        const uint8_t* p = A.arena;
        if (valid) {
            u = rec_units(A, r);
            fb = A.fbase[r];
            if (u.part0) ps0 = A.pslot[2 * r];
            if (u.part1) ps1 = A.pslot[2 * r + 1];
            init = A.init ? A.init[r] : A.init_scalar;
            p = A.arena + A.off[r];
        }
        const bool ok = valid && fb + u.full <= (A.part_base ? A.part_base : A.unit_cap) &&
                        (!u.part0 || ps0 < A.unit_cap) &&
                        (!u.part1 || ps1 < A.unit_cap);
        uint32_t acc = 0;
        bool huge = false;
        // (EM bit 2: the head here -- its register moved to the first unit's end, Z_len0(h))
        uint32_t hs = 0;
        if ((EM & 4) && ok && u.k > 0) {
            const uintptr_t a0 = reinterpret_cast<uintptr_t>(u.g.a);
            const uint32_t len0 = u.k == 1 ? u.last : u.part0 ? (uint32_t)((((a0 >> kUShift) + 1) << kUShift) - a0) : (uint32_t)U;
            hs = shift_last(lds, head_register(lds, kCombZ4, kCombT8, p, u.g, init), len0, U);
        }
        if (ok && u.k > 0) {
            if (u.k <= 64) {
                acc = A.partial[unit_slot(0, u.k, fb, ps0, ps1, u.part0, u.part1)] ^ hs;
                for (uint64_t j = 1; j + 1 < u.k; j += 8) {  // middle units: Z_U steps, 8 loads in flight
                    uint32_t s[8];
#pragma unroll
                    for (int q = 0; q < 8; ++q) s[q] = j + q + 1 < u.k ? A.partial[fb + j + q - u.part0] : 0u;
#pragma unroll
                    for (int q = 0; q < 8; ++q)
                        if (j + q + 1 < u.k) acc = zmap(lds, 0, acc) ^ s[q];
                }
            } else {
                huge = true;
            }
        }
        uint64_t hm = __ballot(huge);
        while (hm) {
            const int h = __ffsll((long long)hm) - 1;
            hm &= hm - 1;
            const uint64_t hk = __shfl(u.k, h) - 1;  // all units but the last
            const uint64_t hfb = __shfl(fb, h), hps0 = __shfl(ps0, h);
            const uint32_t hp0 = __shfl(u.part0, h), hhs = __shfl(hs, h);
            const uint64_t nb = (hk + 63) / 64;
            const int64_t pad = (int64_t)(nb * 64 - hk);
            uint32_t w = 0;
            for (uint64_t blk = 0; blk < nb; ++blk) {
                const int64_t idx = (int64_t)(blk * 64 + lane) - pad;
                uint32_t v = 0;
                if (idx >= 0) v = A.partial[idx == 0 && hp0 ? hps0 : hfb + idx - hp0];
                if (idx == 0) v ^= hhs;
                v = wave_tree(lds, v);
                w = zmap(lds, 6 * 1024, w) ^ v;
            }
            w = __shfl(w, 0);
            if ((int)lane == h) acc = w;
        }
        if (ok && u.k >= 2)  // the last unit: shift by its own length
            acc = shift_last(lds, acc, u.last, U) ^ A.partial[unit_slot(u.k - 1, u.k, fb, ps0, ps1, u.part0, u.part1)];
        if ((EM & 2) && ok && u.k > 0)
            acc = tail_register(lds, kCombZ4, kCombT8, acc, u.g);
        else if (ok && u.k > 0 && u.g.e > u.g.b)  // the tail: Z_t, and the tail bytes' register from the units kernel
            acc = steps_in_vec(lds, kCombZ4, kCombT8, acc, u32x4{0u, 0u, 0u, 0u}, 0u, (uint32_t)(u.g.e - u.g.b)) ^
                  A.tailc[unit_slot(u.k - 1, u.k, fb, ps0, ps1, u.part0, u.part1)];
        if (valid) {
            uint32_t res;
            if (ok && u.k > 0)
                res = ~acc;
            else  // a short record, or (the caller's total_len was low) one whose units did not
                  // fit the table: this lane steps it alone -- slow, but never a wrong CRC
                res = short_record(lds, kCombZ4, kCombT8, p, A.len[r], init);
            A.out[r] = res;
        }
    }
}

// Batches of small records (WAL replay of short records, the bounded ragged ABI, the
// writer's CRC blocks): one record per group of G = 4 lanes, its whole body one unit, no
// plan kernels (scan, descriptors and finalize cost more than the CRCs of 180-byte
// records).  Chunks are 64 bytes on the absolute 64-byte grid, read with the quad blob's
// Z_64 stride tables; the group tree has two levels.  The head and tail byte steps are
// serial LDS lookups with a per-record trip count, so a wave does them for 64 records at
// once (lane i: record base + i), then streams the 64 bodies in 4 rounds of 16 groups,
// passing each record's entering register in and its body register out by shuffles.
// The rounds are software-pipelined (stream_unit): round r + 1's loads are issued before
// round r's last chunks are stepped, and each record's tail block is loaded with its
// extent.  A group with no body in a round (a short record, or past the batch) streams an
// empty unit at a valid address (the table blob): every load is issued unconditionally.
// Correct for any length; balanced when every record is small.
// Why 4 lanes: the kernel is instruction-bound on small records, and the per-round set-up,
// lane fold and tree are shared by 16 records instead of 8 (8-lane groups: 0.237 ms per
// replay call of 1M x 180 B, 4: 0.202, 2: 0.222 -- their loads then spread over 32 cache
// lines per instruction; one record per lane: 0.327).  G = 2 is the tools
// build's KARMA_DIRECT_VARIANT=5 (the pair blob, Z_32).
template <int G, int MODE = 0, int PF = kRaggedPF, bool ALL = false>  // MODE != 0: timing-only variants of the
                                 // tools build (bits 0-1: stream_unit's, crc_device.h; bit 2: no head / tail steps)
__global__ __launch_bounds__(kBlockThreads) void k_ragged_direct4(RaggedArgs A) {
    uint64_t n_rec = A.n_rec;
    if (A.n_dev) {  // a device-sized batch: the count is known on the device only
        if (*A.gate_len > A.gate_max || *A.gate_len < A.gate_min) return;
        n_rec = *A.n_dev;
    }
    KB_SET_ARENA_SAFE(A.kb_lo, A.kb_hi, A.blob, A.blob + kBlobWords);  // the blob: empty units' address
    __shared__ __attribute__((aligned(16))) uint32_t lds[kLdsWords];
    load_stream_tables(lds, A.blob);
    __syncthreads();
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t X = lane_const();
    const uint8_t* safe = reinterpret_cast<const uint8_t*>(A.blob);  // 16-aligned, always mapped
    const uint64_t nwaves = (uint64_t)gridDim.x * kWavesPerBlock;
    for (uint64_t base = ((uint64_t)blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6)) * 64; base < n_rec;
         base += nwaves * 64) {
        const uint64_t ri = base + lane;
        const bool vi = ri < n_rec;
        const uint8_t* pi = vi ? A.arena + A.off[ri] : A.arena;
        const uint32_t ni = vi ? A.len[ri] : 0u;
        const uint32_t initi = vi ? (A.init ? A.init[ri] : A.init_scalar) : 0u;
        const uint32_t res = direct_batch<G, PF, kRaggedNT, MODE, ALL>(lds, X, safe, pi, ni, initi, vi);
        if (vi) {
            A.out[ri] = res;
            if (A.cmp_stored && ni && res != A.cmp_stored[ri]) atomicMin(A.cmp_bad, (unsigned long long)ri);
        }
    }
}

// Batches of small records staged through LDS, one record per lane: a wave takes 64 records,
// and when their aligned extent [lo, hi) fits its kStgBytes of LDS (64 WAL records of up to
// ~190 bytes; consecutive records of any smaller size) it copies that extent in with whole
// 1 KiB wave loads (every cache line read once, by one instruction), then each lane steps its
// own record out of LDS with the reference's 4-slot structure (lane_record: no shuffles, no
// per-round unit geometry, no group tree).  A batch whose extent does not fit (records far
// apart or long) reads its blocks from global memory instead -- exact, only slower.
// PIPE: the next batch's extent is loaded into registers while this batch is stepped.
template <bool PIPE, int MODE = 0>  // MODE (tools build timing only, wrong CRCs): 1 no CRC steps, 2 no staging copy
__global__ __launch_bounds__(kStgWaves * 64) void k_ragged_staged(RaggedArgs A) {
    uint64_t n_rec = A.n_rec;
    if (A.n_dev) {  // a device-sized batch (as k_ragged_direct4)
        if (*A.gate_len > A.gate_max || *A.gate_len < A.gate_min) return;
        n_rec = *A.n_dev;
    }
    KB_SET_ARENA(A.kb_lo, A.kb_hi);
    __shared__ __attribute__((aligned(16))) uint32_t lds[kStgLdsWords];
    load_stg_tables<kStgWaves * 64>(lds, A.blob);
    __syncthreads();
    const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
    const uint32_t X = lane_const16();
    uint8_t* stage = reinterpret_cast<uint8_t*>(lds + kStgBuf) + wave * kStgBytes;
    const uint64_t step = (uint64_t)gridDim.x * kStgWaves * 64;
    uint64_t base = ((uint64_t)blockIdx.x * kStgWaves + wave) * 64;
    if (base >= n_rec) return;
    auto one = [&](const StgBatch& B, bool staged) {
        uint32_t res = B.init;
        if constexpr ((MODE & 1) != 0) {
            if (B.vi && B.n && staged) res ^= *reinterpret_cast<const uint32_t*>(stage + (uint32_t)((B.p & ~uintptr_t(15)) - B.lo));
        } else if (B.vi && B.n) {
            if (staged)
                res = lane_record(lds, X, kStgZ4, kStgT8, B.p, B.n, B.init,
                                  [&](uintptr_t a) { return *reinterpret_cast<const u32x4*>(stage + (uint32_t)(a - B.lo)); });
            else
                res = lane_record(lds, X, kStgZ4, kStgT8, B.p, B.n, B.init,
                                  [&](uintptr_t a) { return ld16(reinterpret_cast<const uint8_t*>(a)); });
        }
        if (B.vi) {
            const uint64_t ri = base + lane;
            A.out[ri] = res;
            if (A.cmp_stored && B.n && res != A.cmp_stored[ri]) atomicMin(A.cmp_bad, (unsigned long long)ri);
        }
    };
    u32x4 v[kStgVecs];
    if constexpr (!PIPE) {
        for (; base < n_rec; base += step) {
            const StgBatch B = stg_meta(A, n_rec, base, lane);
            const bool staged = stg_fits(B);
            if (staged && (MODE & 2) == 0) {
                stg_issue(B, lane, v);
                stg_store(B, lane, v, stage);
                wave_lds_sync();
            }
            one(B, staged);
            wave_lds_sync();  // this batch's reads before the next batch's stores
        }
    } else {
        StgBatch B = stg_meta(A, n_rec, base, lane);
        bool staged = stg_fits(B);
        if (staged) stg_issue(B, lane, v);
        for (;;) {
            if (staged) {
                stg_store(B, lane, v, stage);
                wave_lds_sync();
            }
            const uint64_t nb = base + step;
            const bool more = nb < n_rec;
            StgBatch N = B;
            bool nstaged = false;
            if (more) {  // the next batch's extent in flight while this one is stepped
                N = stg_meta(A, n_rec, nb, lane);
                nstaged = stg_fits(N);
                if (nstaged) stg_issue(N, lane, v);
            }
            one(B, staged);
            wave_lds_sync();
            if (!more) break;
            base = nb;
            B = N;
            staged = nstaged;
        }
    }
}

// The staged kernel software-pipelined across batches: batch k + 1's extent and batch k + 2's
// offsets / lengths are in flight while batch k is stepped (a wave's batches are otherwise one
// chain of three memory latencies and the steps: DESIGN.md §8a), plain scalars across the loop.
// END: the records' windows aligned to their ends (lane_record_end: no head or tail steps);
// the stage then holds the extent 16 bytes in, after a slack the first window may read.
// SKEW (with END): the stage is bank-skewed, one pad dword after every 128 bytes (dword q at
// q + q / 32), so records whose stride is a multiple of 32 bytes (120-B payloads + 8-B headers
// put every lane on one bank) read their windows without conflicts; stores go out as dwords.
template <bool END, int SMODE = 24, int NW = kStgWaves, bool SKEW = true>  // SMODE 8: the 16-copy image in plain lane order
                                                         // (2-way conflicts); NW < kStgWaves: fewer waves (A/B)
__global__ __launch_bounds__(NW * 64) void k_ragged_staged_pipe(RaggedArgs A) {
    // SMODE 32: the 8-copy stride image (32 KiB), so more waves fit beside their stages
    constexpr int TW = (SMODE & 32) ? kRep8Words : kRep16Words, Z4 = TW, T8 = TW + 1024, BUF = TW + 1280;
    constexpr uint32_t kLead = END ? 16u : 0u, kFit = END ? kStgBytes - 32u : kStgBytes;
    constexpr bool SK = END && SKEW;
    constexpr uint32_t kStride = SK ? kStgBytes + kStgBytes / 32 : kStgBytes;  // bytes per wave's stage
    uint64_t n_rec = A.n_rec;
    if (A.n_dev) {
        if (*A.gate_len > A.gate_max || *A.gate_len < A.gate_min) return;
        n_rec = *A.n_dev;
    }
    KB_SET_ARENA(A.kb_lo, A.kb_hi);
    __shared__ __attribute__((aligned(16))) uint32_t lds[BUF + NW * (int)(kStride / 4)];
    if constexpr ((SMODE & 32) != 0) {
        load_rep8_stride<NW * 64>(lds, A.blob);
        copy_to_lds<1024, NW * 64>(lds + Z4, A.blob + kBlobZ4);
        copy_to_lds<256, NW * 64>(lds + T8, A.blob + kBlobT8);
    } else {
        load_stg_tables<NW * 64>(lds, A.blob);
    }
    __syncthreads();
    const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
    const uint32_t X = lane_const16();
    uint8_t* stage = reinterpret_cast<uint8_t*>(lds + BUF) + wave * kStride;
    uint32_t* stage32 = reinterpret_cast<uint32_t*>(stage);
    const uint64_t step = (uint64_t)gridDim.x * NW * 64;
    uint64_t base = ((uint64_t)blockIdx.x * NW + wave) * 64;
    if (base >= n_rec) return;
    auto ld_meta = [&](uint64_t b, uint64_t& o, uint32_t& n, uint32_t& ini) {
        const uint64_t ri = b + lane;
        const bool v = ri < n_rec;
        o = v ? A.off[ri] : 0;
        n = v ? A.len[ri] : 0u;
        ini = v ? (A.init ? A.init[ri] : A.init_scalar) : 0u;
    };
    auto extent = [&](uint64_t o, uint32_t n, uintptr_t& lo, uintptr_t& hi) {
        const uintptr_t p = reinterpret_cast<uintptr_t>(A.arena) + o;
        uint64_t l = n ? (p & ~uintptr_t(15)) : ~0ull, h = n ? ((p + n + 15) & ~uintptr_t(15)) : 0ull;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const uint64_t ol = (uint64_t)__shfl_xor((long long)l, d), oh = (uint64_t)__shfl_xor((long long)h, d);
            l = ol < l ? ol : l;
            h = oh > h ? oh : h;
        }
        lo = uniform64(l);
        hi = uniform64(h);
    };
    u32x4 v[kStgVecs];
    auto issue = [&](uintptr_t lo, uintptr_t hi) {
        const uint32_t nv = (uint32_t)((hi - lo) / 16);
#pragma unroll
        for (int q = 0; q < kStgVecs; ++q) {
            const uint32_t j = lane + 64u * q;  // past the extent: its first block again (no branch)
            v[q] = ldg<true>(reinterpret_cast<const uint8_t*>(lo + 16ull * (j < nv ? j : 0u)));
        }
    };
    // batch `base`: meta (o, n, ini), extent; batch base + step: meta (o2, n2, ini2)
    uint64_t o, o2;
    uint32_t n, ini, n2, ini2;
    uintptr_t lo, hi;
    ld_meta(base, o, n, ini);
    ld_meta(base + step, o2, n2, ini2);
    extent(o, n, lo, hi);
    bool fits = hi != 0 && hi - lo <= kFit;
    // does the batch at (o, n, lo) need the skewed stage?  (banks of the records' first dwords)
    auto skewed = [&](uint64_t o, uint32_t n, uintptr_t lo) {
        if constexpr (!SK) return false;
        const uintptr_t p = reinterpret_cast<uintptr_t>(A.arena) + o;
        uint32_t bits = n ? 1u << (((uint32_t)(p - lo) >> 2) & 31u) : 0u;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) bits |= (uint32_t)__shfl_xor((int)bits, d);
        return __builtin_popcount(__builtin_amdgcn_readfirstlane(bits)) < 12;
    };
    bool sk = fits && skewed(o, n, lo);
    if (fits) issue(lo, hi);
    for (;;) {
        if (fits) {
#pragma unroll
            for (int q = 0; q < kStgVecs; ++q) {
                uint32_t at = kLead + 16u * (lane + 64u * q);
                at = at >= kStgBytes ? 0u : at;  // (END) the last slot, past any extent, into the slack
                if (sk) {  // 4 dwords in one 128-byte line: contiguous after the skew
                    const uint32_t d = at / 4 + at / 128;
                    stage32[d] = v[q].x;
                    stage32[d + 1] = v[q].y;
                    stage32[d + 2] = v[q].z;
                    stage32[d + 3] = v[q].w;
                } else {
                    *reinterpret_cast<u32x4*>(stage + at) = v[q];
                }
            }
            wave_lds_sync();
        }
        const uint64_t nb = base + step;
        const bool more = nb < n_rec;
        uintptr_t lo2 = 0, hi2 = 0;
        bool fits2 = false, sk2 = false;
        uint64_t o3 = 0;
        uint32_t n3 = 0, ini3 = 0;
        if (more) {
            extent(o2, n2, lo2, hi2);
            fits2 = hi2 != 0 && hi2 - lo2 <= kFit;
            sk2 = fits2 && skewed(o2, n2, lo2);
            if (fits2) issue(lo2, hi2);
            ld_meta(nb + step, o3, n3, ini3);
        }
        const uint64_t ri = base + lane;
        if (ri < n_rec) {
            uint32_t res = ini;
            const uintptr_t p = reinterpret_cast<uintptr_t>(A.arena) + o;
            if (n) {
                if (fits && END && n >= 4 && sk)
                    res = lane_record_end<SMODE>(lds, X, Z4, kLead + (uint32_t)(p - lo), n, ini,
                                                 [&](uint32_t q) { return stage32[q + (q >> 5)]; });
                else if (fits && END && n >= 4)
                    res = lane_record_end<SMODE>(lds, X, Z4, kLead + (uint32_t)(p - lo), n, ini, [&](uint32_t q) {
                        return *reinterpret_cast<const uint32_t*>(stage + 4u * q);
                    });
                else if (fits)
                    res = lane_record(lds, X, Z4, T8, p, n, ini, [&](uintptr_t a) {
                        const uint32_t at = kLead + (uint32_t)(a - lo);
                        if (sk) {
                            const uint32_t d = at / 4 + at / 128;
                            return u32x4{stage32[d], stage32[d + 1], stage32[d + 2], stage32[d + 3]};
                        }
                        return *reinterpret_cast<const u32x4*>(stage + at);
                    });
                else
                    res = lane_record(lds, X, Z4, T8, p, n, ini,
                                      [&](uintptr_t a) { return ld16(reinterpret_cast<const uint8_t*>(a)); });
            }
            A.out[ri] = res;
            if (A.cmp_stored && n && res != A.cmp_stored[ri]) atomicMin(A.cmp_bad, (unsigned long long)ri);
        }
        wave_lds_sync();
        if (!more) break;
        base = nb;
        o = o2; n = n2; ini = ini2;
        o2 = o3; n2 = n3; ini2 = ini3;
        lo = lo2; hi = hi2; fits = fits2; sk = sk2;
    }
}

#ifdef KARMA_AB
// Pairs of lanes per record (tools build, KARMA_DIRECT_VARIANT=21): half the stage per wave
// (32 records, 6 KiB) so twice the waves per CU, and half the dependent chain per lane.  The
// windows are aligned to the record's end (lane_record_end) and dealt from the end: lane 1 of
// the pair takes windows W-1, W-3, ..., lane 0 takes W-2, W-4, ..., each striding 32 bytes
// (the pair blob's Z_32 tables); the record's register is R1 ^ Z16(R0).
constexpr int kPairWaves = 14;
constexpr uint32_t kPairStg = 6144;                     // extent bytes per wave (32 records)
constexpr uint32_t kPairStride = kPairStg + 16;         // + the first window's lead-in slack
constexpr int kPairVecs = (int)(kPairStg / 1024);
constexpr int kPairZ4 = kRep16Words, kPairZ16 = kPairZ4 + 1024, kPairT8 = kPairZ16 + 1024, kPairBuf = kPairT8 + 256;
constexpr int kPairLdsWords = kPairBuf + kPairWaves * (int)(kPairStride / 4);
static_assert(kPairLdsWords * 4 <= 160 * 1024, "LDS of one workgroup");

// This lane's half of the record [sp, sp + n) of the stage (n >= 4): its windows' register,
// ending at the record end (l = 1) or 16 bytes before it (l = 0; 0 when it has none).
template <typename Rd>
__device__ __forceinline__ uint32_t pair_record_end(const uint32_t* lds, uint32_t X, uint32_t sp, uint32_t n,
                                                    uint32_t init, uint32_t l, Rd&& rd) {
    const uint32_t W = (n + 15) >> 4, h0 = 16 * W - n;
    const uint32_t s0 = sp - h0, sh = s0 & 3, q0 = s0 >> 2;
    const uint32_t inj = ~init, b = h0 & 3, k0 = h0 >> 2;
    const uint32_t lo32 = inj << (8 * b), hi32 = b ? inj >> (32 - 8 * b) : 0u;
    auto keep = [&](uint32_t k) {
        const int r = (int)h0 - 4 * (int)k;
        return r <= 0 ? ~0u : r >= 4 ? 0u : (~0u << (8 * r));
    };
    auto window = [&](uint32_t j) {
        const uint32_t q = q0 + 4 * j;
        const uint32_t d0 = rd(q), d1 = rd(q + 1), d2 = rd(q + 2), d3 = rd(q + 3), d4 = rd(q + 4);
        u32x4 v;
        v.x = __builtin_amdgcn_alignbyte(d1, d0, sh);
        v.y = __builtin_amdgcn_alignbyte(d2, d1, sh);
        v.z = __builtin_amdgcn_alignbyte(d3, d2, sh);
        v.w = __builtin_amdgcn_alignbyte(d4, d3, sh);
        if (j == 0) {  // the lead-in bytes masked, ~init into the record's first 4 bytes
            v.x = (v.x & keep(0)) ^ (k0 == 0 ? lo32 : 0u);
            v.y = (v.y & keep(1)) ^ (k0 == 1 ? lo32 : 0u) ^ (k0 == 0 ? hi32 : 0u);
            v.z = (v.z & keep(2)) ^ (k0 == 2 ? lo32 : 0u) ^ (k0 == 1 ? hi32 : 0u);
            v.w = (v.w & keep(3)) ^ (k0 == 3 ? lo32 : 0u) ^ (k0 == 2 ? hi32 : 0u);
        } else if (j == 1 && k0 == 3) {
            v.x ^= hi32;
        }
        return v;
    };
    uint32_t j = l ? ((W - 1) & 1u) : (W & 1u);
    uint32_t a0 = 0, a1 = 0, a2 = 0, a3 = 0;
    if (j < W) {
        const u32x4 v = window(j);
        a0 = v.x;
        a1 = v.y;
        a2 = v.z;
        a3 = v.w;
        j += 2;
    }
    for (; j < W; j += 2) step4<8>(lds, X, a0, a1, a2, a3, window(j));
    return lane_fold_at(lds, kPairZ4, a0, a1, a2, a3);
}

__global__ __launch_bounds__(kPairWaves * 64) void k_ragged_staged_pair(RaggedArgs A) {
    uint64_t n_rec = A.n_rec;
    if (A.n_dev) {
        if (*A.gate_len > A.gate_max || *A.gate_len < A.gate_min) return;
        n_rec = *A.n_dev;
    }
    KB_SET_ARENA(A.kb_lo, A.kb_hi);
    __shared__ __attribute__((aligned(16))) uint32_t lds[kPairLdsWords];
    load_rep16_stride<kPairWaves * 64>(lds, A.blob, [&] {  // the pair blob: Z_32 stride tables
        copy_to_lds<1024, kPairWaves * 64>(lds + kPairZ4, A.blob + kBlobZ4);
        copy_to_lds<1024, kPairWaves * 64>(lds + kPairZ16, A.blob + kBlobZ16);
        copy_to_lds<256, kPairWaves * 64>(lds + kPairT8, A.blob + kBlobT8);
    });
    __syncthreads();
    const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6, l = lane & 1u, rl = lane >> 1;
    const uint32_t X = lane_const16();
    uint8_t* stage = reinterpret_cast<uint8_t*>(lds + kPairBuf) + wave * kPairStride;  // data from stage + 16
    const uint64_t step = (uint64_t)gridDim.x * kPairWaves * 32;
    uint64_t base = ((uint64_t)blockIdx.x * kPairWaves + wave) * 32;
    if (base >= n_rec) return;
    auto ld_meta = [&](uint64_t b, uint64_t& o, uint32_t& n, uint32_t& ini) {
        const uint64_t ri = b + rl;
        const bool v = ri < n_rec;
        o = v ? A.off[ri] : 0;
        n = v ? A.len[ri] : 0u;
        ini = v ? (A.init ? A.init[ri] : A.init_scalar) : 0u;
    };
    auto extent = [&](uint64_t o, uint32_t n, uintptr_t& lo, uintptr_t& hi) {
        const uintptr_t p = reinterpret_cast<uintptr_t>(A.arena) + o;
        uint64_t lw = n ? (p & ~uintptr_t(15)) : ~0ull, h = n ? ((p + n + 15) & ~uintptr_t(15)) : 0ull;
#pragma unroll
        for (int d = 2; d < 64; d <<= 1) {  // (the two lanes of a pair hold the same record)
            const uint64_t ol = (uint64_t)__shfl_xor((long long)lw, d), oh = (uint64_t)__shfl_xor((long long)h, d);
            lw = ol < lw ? ol : lw;
            h = oh > h ? oh : h;
        }
        lo = uniform64(lw);
        hi = uniform64(h);
    };
    u32x4 v[kPairVecs];
    auto issue = [&](uintptr_t lo, uintptr_t hi) {
        const uint32_t nv = (uint32_t)((hi - lo) / 16);
#pragma unroll
        for (int q = 0; q < kPairVecs; ++q) {
            const uint32_t j = lane + 64u * q;
            v[q] = ldg<true>(reinterpret_cast<const uint8_t*>(lo + 16ull * (j < nv ? j : 0u)));
        }
    };
    constexpr uint32_t kFit = kPairStg - 16u;  // the last window may read 3 bytes past the extent
    uint64_t o, o2;
    uint32_t n, ini, n2, ini2;
    uintptr_t lo, hi;
    ld_meta(base, o, n, ini);
    ld_meta(base + step, o2, n2, ini2);
    extent(o, n, lo, hi);
    bool fits = hi != 0 && hi - lo <= kFit;
    if (fits) issue(lo, hi);
    for (;;) {
        if (fits) {
#pragma unroll
            for (int q = 0; q < kPairVecs; ++q) *reinterpret_cast<u32x4*>(stage + 16u + 16u * (lane + 64u * q)) = v[q];
            wave_lds_sync();
        }
        const uint64_t nb = base + step;
        const bool more = nb < n_rec;
        uintptr_t lo2 = 0, hi2 = 0;
        bool fits2 = false;
        uint64_t o3 = 0;
        uint32_t n3 = 0, ini3 = 0;
        if (more) {
            extent(o2, n2, lo2, hi2);
            fits2 = hi2 != 0 && hi2 - lo2 <= kFit;
            if (fits2) issue(lo2, hi2);
            ld_meta(nb + step, o3, n3, ini3);
        }
        const uint64_t ri = base + rl;
        const uintptr_t p = reinterpret_cast<uintptr_t>(A.arena) + o;
        uint32_t part = 0;
        const bool pair = fits && n >= 4 && ri < n_rec;
        if (pair)
            part = pair_record_end(lds, X, 16u + (uint32_t)(p - lo), n, ini, l, [&](uint32_t q) {
                return *reinterpret_cast<const uint32_t*>(stage + 4u * q);
            });
        const uint32_t other = __shfl_xor(part, 1);
        if (l == 1 && ri < n_rec) {
            uint32_t res;
            if (pair)
                res = ~(part ^ zmap(lds, kPairZ16, other));
            else if (n)  // a short record or an extent that does not fit: byte / word steps from memory
                res = short_record(lds, kPairZ4, kPairT8, reinterpret_cast<const uint8_t*>(p), n, ini);
            else
                res = ini;
            A.out[ri] = res;
            if (A.cmp_stored && n && res != A.cmp_stored[ri]) atomicMin(A.cmp_bad, (unsigned long long)ri);
        }
        wave_lds_sync();
        if (!more) break;
        base = nb;
        o = o2; n = n2; ini = ini2;
        o2 = o3; n2 = n3; ini2 = ini3;
        lo = lo2; hi = hi2; fits = fits2;
    }
}

// Tools build (KARMA_DIRECT_VARIANT=1, ab.h): small records one per group of 8 lanes, the
// shipped kernel before k_ragged_direct4 (0.237 vs 0.202 ms per 1M x 180 B replay call,
// DESIGN.md §8a).  Batches of small records: one record per group, its whole body one unit, no plan kernels (scan, descriptors and
// finalize cost more than the CRCs of 180-byte records).  The head and tail byte steps are
// serial LDS lookups with a per-record trip count, so a wave does them for 64 records at
// once (lane i: record base + i), and streams the 64 bodies in 8 rounds of 8 groups,
// passing each record's entering register in and its body register out by shuffles.
// The rounds are software-pipelined (stream_unit): round r + 1's loads are issued before
// round r's last chunks are stepped, and each record's tail block is loaded with its
// extent, so a wave waits on memory about once per 64 records instead of once per round.
// A group with no body in a round (a short record, or past the batch) streams an empty
// unit at a valid address (the table blob): every load is issued unconditionally.
// Correct for any length; balanced when every record is small.
__global__ __launch_bounds__(kBlockThreads) void k_ragged_direct(RaggedArgs A) {
    KB_SET_ARENA_SAFE(A.kb_lo, A.kb_hi, A.blob, A.blob + kBlobWords);  // the blob: empty units' address
    __shared__ __attribute__((aligned(16))) uint32_t lds[kLdsWords];
    load_stream_tables(lds, A.blob);
    __syncthreads();
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t l = lane & (kGroupLanes - 1);
    const uint32_t grp = lane / kGroupLanes;
    const uint32_t X = lane_const();
    const uint8_t* safe = reinterpret_cast<const uint8_t*>(A.blob);  // 16-aligned, always mapped
    const uint64_t nwaves = (uint64_t)gridDim.x * kWavesPerBlock;
    for (uint64_t base = ((uint64_t)blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6)) * 64; base < A.n_rec;
         base += nwaves * 64) {
        // lane i: record base + i -- its extent, entering register and tail block
        const uint64_t ri = base + lane;
        const bool vi = ri < A.n_rec;
        const uint8_t* pi = vi ? A.arena + A.off[ri] : A.arena;
        const uint32_t ni = vi ? A.len[ri] : 0u;
        const uint32_t initi = vi ? (A.init ? A.init[ri] : A.init_scalar) : 0u;
        const Geom gi = geom(pi, ni);
        const bool body = vi && !gi.is_short;
        const uint64_t ai = reinterpret_cast<uintptr_t>(body ? gi.a : safe);
        const uint64_t bi = reinterpret_cast<uintptr_t>(body ? gi.b : safe);
        // round r's unit of this group: record base + 8 r + grp (shuffles with every lane active)
        auto unit_of = [&](uint32_t r) {
            const int src = (int)(r * kGroupsPerWave + grp);
            const uint8_t* us = reinterpret_cast<const uint8_t*>((uintptr_t)__shfl((long long)ai, src));
            const uint8_t* ue = reinterpret_cast<const uint8_t*>((uintptr_t)__shfl((long long)bi, src));
            return lane_unit(us, ue, l);
        };
        LaneUnit L = unit_of(0);
        UnitLoads<kRaggedPF> Ld;
        issue_unit_loads<kRaggedPF, kRaggedNT>(L, Ld);
        const bool tail = body && gi.e > gi.b;
        const u32x4 tv = ld16(tail ? gi.b : safe);
        const uint32_t hi = body ? head_register(lds, kLZ4, kLT8, pi, gi, initi) : 0u;
        uint32_t Ri = 0;
#pragma unroll 1
        for (uint32_t round = 0; round < 8; ++round) {
            const uint32_t sh = __shfl(hi, (int)(round * kGroupsPerWave + grp));
            LaneUnit N = L;
            const uint32_t R = stream_unit<kRaggedPF, kRaggedNT>(lds, X, l, L, Ld, L.us, sh, [&](UnitLoads<kRaggedPF>& nx) {
                if (round + 1 < 8) {
                    N = unit_of(round + 1);
                    issue_unit_loads<kRaggedPF, kRaggedNT>(N, nx);
                }
            });
            const uint32_t Rr = __shfl(R, (int)((lane & 7u) * kGroupLanes));  // group (lane & 7)'s register
            if (lane / kGroupsPerWave == round) Ri = Rr;
            L = N;
        }
        if (vi)
            A.out[ri] = gi.is_short ? short_record(lds, kLZ4, kLT8, pi, ni, initi)
                                    : ~steps_in_vec(lds, kLZ4, kLT8, Ri, tv, 0u, tail ? (uint32_t)(gi.e - gi.b) : 0u);
    }
}

// Tools build (KARMA_DIRECT_VARIANT=3, ab.h): small records one per LANE, measured slower
// than k_ragged_direct on the WAL replay's 180-byte records (0.327 vs 0.240 ms per replay
// call): a lane's 16-byte loads of its own record make every load
// instruction touch 64 cache lines.  Each lane runs the
// reference's own structure over its record (crc32c.cc:323-370): the unaligned head byte
// steps, four word slots striding 16 bytes through the aligned body (Z_16 from the
// bank-replicated LDS tables of the lane blob, one v_perm_b32 per lookup address), the
// STEP4W lane fold and the unaligned tail.  There is no cross-lane work at all (no group
// tree, no rounds, no shuffles), which is what bounds the one-record-per-group kernel on
// 180-byte records (k_ragged_direct: ~110 VALU instructions per record, mostly fold, tree
// and unit set-up for two chunks of data).  A lane loads up to kLaneWindows 16-byte
// windows of its body at once: the 8 windows of one cache line are in flight together, so
// each line is requested from L2 once.
constexpr int kLaneWindows = 16;

__global__ __launch_bounds__(kBlockThreads) void k_ragged_lanes(RaggedArgs A) {
    KB_SET_ARENA_SAFE(A.kb_lo, A.kb_hi, A.blob, A.blob + kBlobWords);
    __shared__ __attribute__((aligned(16))) uint32_t lds[kLdsWords];
    load_stream_tables(lds, A.blob);  // the lane blob: Z_16 replicated, Z4, the byte table
    __syncthreads();
    const uint32_t X = lane_const();
    const uint8_t* safe = reinterpret_cast<const uint8_t*>(A.blob);
    const uint64_t nthr = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; r < A.n_rec; r += nthr) {
        const uint8_t* p = A.arena + A.off[r];
        const uint32_t n = A.len[r];
        const uint32_t init = A.init ? A.init[r] : A.init_scalar;
        const Geom g = geom(p, n);
        if (g.is_short) {
            A.out[r] = short_record(lds, kLZ4, kLT8, p, n, init);
            continue;
        }
        const uint64_t nw = (uint64_t)(g.b - g.a) / 16;  // aligned body windows (>= 1)
        const bool tail = g.e > g.b;
        // first batch of windows, the head and the tail blocks: all in flight at once
        u32x4 v[kLaneWindows];
        uint64_t m = nw < kLaneWindows ? nw : kLaneWindows;
#pragma unroll
        for (int q = 0; q < kLaneWindows; ++q) v[q] = ldg<true>(g.a + 16 * ((uint64_t)q < m ? q : m - 1));
        const u32x4 tv = ld16(tail ? g.b : safe);
        const uint32_t h = head_register(lds, kLZ4, kLT8, p, g, init);
        uint32_t a0 = v[0].x ^ h, a1 = v[0].y, a2 = v[0].z, a3 = v[0].w;
#pragma unroll
        for (int q = 1; q < kLaneWindows; ++q)
            if ((uint64_t)q < m) step4(lds, X, a0, a1, a2, a3, v[q]);
        for (uint64_t c = kLaneWindows; c < nw; c += kLaneWindows) {  // longer bodies: further batches
            m = nw - c < kLaneWindows ? nw - c : kLaneWindows;
            const uint8_t* w = g.a + 16 * c;
#pragma unroll
            for (int q = 0; q < kLaneWindows; ++q) v[q] = ldg<true>(w + 16 * ((uint64_t)q < m ? q : m - 1));
#pragma unroll
            for (int q = 0; q < kLaneWindows; ++q)
                if ((uint64_t)q < m) step4(lds, X, a0, a1, a2, a3, v[q]);
        }
        const uint32_t R = lane_fold(lds, a0, a1, a2, a3);  // the register at the body end
        A.out[r] = ~steps_in_vec(lds, kLZ4, kLT8, R, tv, 0u, tail ? (uint32_t)(g.e - g.b) : 0u);
    }
}

// The first form of k_ragged_direct (tools build, KARMA_DIRECT_VARIANT=2, ab.h): each round's
// loads issued when the round starts.  Batches of small records: one record per group,
// its whole body one unit, no plan kernels (scan, descriptors and finalize cost
// more than the CRCs of 180-byte records).  The head and tail byte steps are
// serial LDS lookups with a per-record trip count, so a wave does them for 64
// records at once (lane i: record base + i), then streams the 64 bodies in 8
// rounds of 8 groups, passing each record's entering register in and its body
// register out by shuffles.  Correct for any length; balanced when every record
// is small.
__global__ __launch_bounds__(kBlockThreads) void k_ragged_direct_v1(RaggedArgs A) {
    KB_SET_ARENA(A.kb_lo, A.kb_hi);
    __shared__ __attribute__((aligned(16))) uint32_t lds[kLdsWords];
    load_stream_tables(lds, A.blob);
    __syncthreads();
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t l = lane & (kGroupLanes - 1);
    const uint32_t grp = lane / kGroupLanes;
    const uint32_t X = lane_const();
    const uint64_t nwaves = (uint64_t)gridDim.x * kWavesPerBlock;
    for (uint64_t base = ((uint64_t)blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6)) * 64; base < A.n_rec;
         base += nwaves * 64) {
        // lane i: record base + i -- its extent and entering register
        const uint64_t ri = base + lane;
        const bool vi = ri < A.n_rec;
        const uint8_t* pi = vi ? A.arena + A.off[ri] : A.arena;
        const uint32_t ni = vi ? A.len[ri] : 0u;
        const uint32_t initi = vi ? (A.init ? A.init[ri] : A.init_scalar) : 0u;
        const Geom gi = geom(pi, ni);
        const bool body = vi && !gi.is_short;
        const uint32_t hi = body ? head_register(lds, kLZ4, kLT8, pi, gi, initi) : 0u;
        const uint64_t ai = reinterpret_cast<uintptr_t>(gi.a), bi = reinterpret_cast<uintptr_t>(gi.b);
        uint32_t Ri = 0;
#pragma unroll 1
        for (uint32_t round = 0; round < 8; ++round) {  // 8 records per round, one per group
            // shuffles with every lane active (a source lane outside EXEC would read as 0)
            const int src = (int)(round * kGroupsPerWave + grp);
            const bool has = __shfl((int)body, src) != 0;
            const uint64_t sa = (uint64_t)__shfl((long long)ai, src), sb = (uint64_t)__shfl((long long)bi, src);
            const uint32_t sh = __shfl(hi, src);
            const uint8_t* us = has ? reinterpret_cast<const uint8_t*>((uintptr_t)sa) : nullptr;
            const uint8_t* ue = has ? reinterpret_cast<const uint8_t*>((uintptr_t)sb) : nullptr;
            const uint8_t* inj_at = us;
            const uint32_t inj = has ? sh : 0u;
            const uint32_t R = group_unit<kRaggedPF, kRaggedNT>(lds, X, l, us, ue, inj_at, inj);
            const uint32_t Rr = __shfl(R, (int)((lane & 7u) * kGroupLanes));  // group (lane & 7)'s register
            if (lane / kGroupsPerWave == round) Ri = Rr;
        }
        if (vi)
            A.out[ri] = gi.is_short ? short_record(lds, kLZ4, kLT8, pi, ni, initi) : ~tail_register(lds, kLZ4, kLT8, Ri, gi);
    }
}

#endif

}  // namespace

hipError_t launch_ragged_direct(const RaggedArgs& a, int grid_blocks, hipStream_t s) {
    if (a.n_rec == 0) return hipSuccess;
    units_timer_begin(s);
#ifdef KARMA_AB
    const long v = KARMA_AB_KNOB("KARMA_DIRECT_VARIANT", 0);
    if (v == 1)
        hipLaunchKernelGGL(k_ragged_direct, dim3(grid_blocks), dim3(kBlockThreads), 0, s, a);
    else if (v == 2)
        hipLaunchKernelGGL(k_ragged_direct_v1, dim3(grid_blocks), dim3(kBlockThreads), 0, s, a);
    else if (v == 3)
        hipLaunchKernelGGL(k_ragged_lanes, dim3(grid_blocks), dim3(kBlockThreads), 0, s, a);
    else if (v == 5)
        hipLaunchKernelGGL(k_ragged_direct4<2>, dim3(grid_blocks), dim3(kBlockThreads), 0, s, a);
    else if (v == 6)  // timing only (wrong CRCs): no body lookups / no fold and tree / neither
        hipLaunchKernelGGL((k_ragged_direct4<4, 1>), dim3(grid_blocks), dim3(kBlockThreads), 0, s, a);
    else if (v == 7)
        hipLaunchKernelGGL((k_ragged_direct4<4, 2>), dim3(grid_blocks), dim3(kBlockThreads), 0, s, a);
    else if (v == 8)
        hipLaunchKernelGGL((k_ragged_direct4<4, 3>), dim3(grid_blocks), dim3(kBlockThreads), 0, s, a);
    else if (v == 9)  // timing only: no head / tail steps; 10: none of the three
        hipLaunchKernelGGL((k_ragged_direct4<4, 4>), dim3(grid_blocks), dim3(kBlockThreads), 0, s, a);
    else if (v == 10)
        hipLaunchKernelGGL((k_ragged_direct4<4, 7>), dim3(grid_blocks), dim3(kBlockThreads), 0, s, a);
    else if (v == 11)  // every round's first loads at once (direct_batch ALL), 2 / 4 chunks each
        hipLaunchKernelGGL((k_ragged_direct4<4, 0, 2, true>), dim3(grid_blocks), dim3(kBlockThreads), 0, s, a);
    else if (v == 12)
        hipLaunchKernelGGL((k_ragged_direct4<4, 0, 4, true>), dim3(grid_blocks), dim3(kBlockThreads), 0, s, a);
    else if (v == 13)  // one round ahead (the shipped form) with 2 chunks
        hipLaunchKernelGGL((k_ragged_direct4<4, 0, 2, false>), dim3(grid_blocks), dim3(kBlockThreads), 0, s, a);
    else if (v == 14)  // staged through LDS, one record per lane (the lane blob)
        hipLaunchKernelGGL(k_ragged_staged<false>, dim3(grid_blocks), dim3(kStgWaves * 64), 0, s, a);
    else if (v == 15)  // ... with the next batch's extent loaded while this one is stepped
        hipLaunchKernelGGL(k_ragged_staged<true>, dim3(grid_blocks), dim3(kStgWaves * 64), 0, s, a);
    else if (v == 19)  // staged, software-pipelined across batches (k_ragged_staged_pipe)
        hipLaunchKernelGGL(k_ragged_staged_pipe<false>, dim3(grid_blocks), dim3(kStgWaves * 64), 0, s, a);
    else if (v == 20)  // ... with the windows aligned to the record ends (no head / tail steps)
        hipLaunchKernelGGL(k_ragged_staged_pipe<true>, dim3(grid_blocks), dim3(kStgWaves * 64), 0, s, a);
    else if (v == 22)  // variant 20 with the plain lane order of the 16-copy image (2-way bank conflicts)
        hipLaunchKernelGGL((k_ragged_staged_pipe<true, 8>), dim3(grid_blocks), dim3(kStgWaves * 64), 0, s, a);
    else if (v == 23)  // variant 20 with 4 / 5 waves per CU (LDS left for other kernels' workgroups)
        hipLaunchKernelGGL((k_ragged_staged_pipe<true, 24, 4>), dim3(grid_blocks), dim3(4 * 64), 0, s, a);
    else if (v == 24)
        hipLaunchKernelGGL((k_ragged_staged_pipe<true, 24, 5>), dim3(grid_blocks), dim3(5 * 64), 0, s, a);
    else if (v == 27)  // variant 20 without the bank-skewed stage
        hipLaunchKernelGGL((k_ragged_staged_pipe<true, 24, kStgWaves, false>), dim3(grid_blocks), dim3(kStgWaves * 64), 0, s, a);
    else if (v == 25)  // variant 20 on the 8-copy stride image, 10 / 9 waves per CU
        hipLaunchKernelGGL((k_ragged_staged_pipe<true, 32, 10, false>), dim3(grid_blocks), dim3(10 * 64), 0, s, a);
    else if (v == 26)
        hipLaunchKernelGGL((k_ragged_staged_pipe<true, 32, 9, false>), dim3(grid_blocks), dim3(9 * 64), 0, s, a);
    else if (v == 21)  // ... and two lanes per record (32 records per wave, 14 waves per CU)
        hipLaunchKernelGGL(k_ragged_staged_pair, dim3(grid_blocks), dim3(kPairWaves * 64), 0, s, a);
    else if (v == 16)  // timing only: staging copy without the CRC steps / 17 the steps without the copy / 18 neither
        hipLaunchKernelGGL((k_ragged_staged<false, 1>), dim3(grid_blocks), dim3(kStgWaves * 64), 0, s, a);
    else if (v == 17)
        hipLaunchKernelGGL((k_ragged_staged<false, 2>), dim3(grid_blocks), dim3(kStgWaves * 64), 0, s, a);
    else if (v == 18)
        hipLaunchKernelGGL((k_ragged_staged<false, 3>), dim3(grid_blocks), dim3(kStgWaves * 64), 0, s, a);
    else
#endif
        hipLaunchKernelGGL(k_ragged_direct4<4>, dim3(grid_blocks), dim3(kBlockThreads), 0, s, a);
    units_timer_end(s);
    return hipGetLastError();
}

hipError_t launch_ragged_staged_dev(const RaggedArgs& a, int grid_blocks, hipStream_t s) {
    if (a.n_rec == 0 || !a.n_dev || !a.gate_len) return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_ragged_staged_pipe<true>, dim3(grid_blocks), dim3(kStgWaves * 64), 0, s, a);
    return hipGetLastError();
}

hipError_t launch_ragged_direct_dev(const RaggedArgs& a, int grid_blocks, hipStream_t s) {
    if (a.n_rec == 0 || !a.n_dev || !a.gate_len) return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_ragged_direct4<4>, dim3(grid_blocks), dim3(kBlockThreads), 0, s, a);
    return hipGetLastError();
}

hipError_t launch_ragged_scan(const RaggedArgs& a, hipStream_t s) {
    if (a.n_rec == 0) return hipSuccess;
    if (a.unit_bytes != kU) return hipErrorInvalidValue;
    const uint64_t nb = ragged_scan_blocks(a.n_rec);
    hipLaunchKernelGGL(k_ragged_scan, dim3((unsigned)nb), dim3(kScanBlock), 0, s, a);
    return hipGetLastError();
}

hipError_t launch_ragged_main(const RaggedArgs& a, int grid_blocks, hipStream_t s, bool two_pass) {
    if (a.n_rec == 0) return hipSuccess;
    const uint64_t nb = ragged_scan_blocks(a.n_rec);
    // Where the record edges are stepped: kShipEM (the plan steps each record's head, finalize
    // its tail).  The tools build's KARMA_RAGGED_EDGES: 1 = that, 0 = both in the units kernel
    // (ragged_unit), 2 = head in the plan only, 3 = tail in finalize only, 4 = both in finalize.
    int em = kShipEM;
#ifdef KARMA_AB
    {
        const long ev = KARMA_AB_KNOB("KARMA_RAGGED_EDGES", 1);
        em = two_pass ? 0 : ev == 1 ? 3 : ev == 2 ? 1 : ev == 3 ? 2 : ev == 4 ? 6 : 0;
    }
    if (two_pass) {
        hipLaunchKernelGGL(k_ragged_desc, dim3((unsigned)nb), dim3(kScanBlock), 0, s, a);  // after launch_ragged_scan
    } else
#endif
    {
        if (two_pass || !a.lb || !a.lb_ctl || a.lb_seq_max < 2 || a.lb_seq_max > (1u << 22)) return hipErrorInvalidValue;
#ifdef KARMA_AB
        if (em == 0)
            hipLaunchKernelGGL(k_ragged_plan<0>, dim3((unsigned)nb), dim3(kScanBlock), 0, s, a);
        else if (em == 1)
            hipLaunchKernelGGL(k_ragged_plan<1>, dim3((unsigned)nb), dim3(kScanBlock), 0, s, a);
        else if (em == 2)
            hipLaunchKernelGGL(k_ragged_plan<2>, dim3((unsigned)nb), dim3(kScanBlock), 0, s, a);
        else if (em == 6)
            hipLaunchKernelGGL(k_ragged_plan<6>, dim3((unsigned)nb), dim3(kScanBlock), 0, s, a);
        else
#endif
            hipLaunchKernelGGL(k_ragged_plan<kShipEM>, dim3((unsigned)nb), dim3(kScanBlock), 0, s, a);
    }
    units_timer_begin(s);
#ifdef KARMA_AB  // tools build (ab.h): 2 = static wave-steps, 4 / 8 = chunks in flight, 1 / 6 = pipelined (PF 4 / 6)
    const long v = KARMA_AB_KNOB("KARMA_RAGGED_VARIANT", 0);
    if (em == 3 && v == 1)
        hipLaunchKernelGGL(k_units_ragged_pipe<4>, dim3(grid_blocks), dim3(kBlockThreads), 0, s, a);
    else if (em == 3 && v == 6)
        hipLaunchKernelGGL(k_units_ragged_pipe<6>, dim3(grid_blocks), dim3(kBlockThreads), 0, s, a);
    else if (em == 3 && v == 11)
        hipLaunchKernelGGL((k_units_ragged_pipe<4, 1>), dim3(grid_blocks), dim3(kBlockThreads), 0, s, a);
    else if (em == 3 && v == 16)
        hipLaunchKernelGGL((k_units_ragged_pipe<6, 1>), dim3(grid_blocks), dim3(kBlockThreads), 0, s, a);
    else if (em == 3 && v == 21)
        hipLaunchKernelGGL((k_units_ragged_pipe<4, 2>), dim3(grid_blocks), dim3(kBlockThreads), 0, s, a);
    else if (em == 3 && v == 26)
        hipLaunchKernelGGL((k_units_ragged_pipe<6, 2>), dim3(grid_blocks), dim3(kBlockThreads), 0, s, a);
    else if (em == 0)
        hipLaunchKernelGGL((k_units_ragged<true, kRaggedUnitsPF, 0>), dim3(grid_blocks), dim3(kBlockThreads), 0, s, a);
    else if (em == 1)
        hipLaunchKernelGGL((k_units_ragged<true, kRaggedUnitsPF, 1>), dim3(grid_blocks), dim3(kBlockThreads), 0, s, a);
    else if (em == 2)
        hipLaunchKernelGGL((k_units_ragged<true, kRaggedUnitsPF, 2>), dim3(grid_blocks), dim3(kBlockThreads), 0, s, a);
    else if (em == 6)
        hipLaunchKernelGGL((k_units_ragged<true, kRaggedUnitsPF, 6>), dim3(grid_blocks), dim3(kBlockThreads), 0, s, a);
    else if (v == 4)
        hipLaunchKernelGGL((k_units_ragged<true, 4>), dim3(grid_blocks), dim3(kBlockThreads), 0, s, a);
    else if (v == 8)
        hipLaunchKernelGGL((k_units_ragged<true, 8>), dim3(grid_blocks), dim3(kBlockThreads), 0, s, a);
    else if (v == 2)
        hipLaunchKernelGGL(k_units_ragged<false>, dim3(grid_blocks), dim3(kBlockThreads), 0, s, a);
    else
#endif
        hipLaunchKernelGGL(k_units_ragged<true>, dim3(grid_blocks), dim3(kBlockThreads), 0, s, a);
    units_timer_end(s);
    uint64_t fblocks = (a.n_rec + 1023) / 1024;  // 16 waves x 64 records per block
    // at most 2 per CU (each loads the 73 KiB combine image; the tools build's
    // KARMA_FINALIZE_PER_CU tries other counts)
    const uint64_t cap = (uint64_t)KARMA_AB_KNOB("KARMA_FINALIZE_PER_CU", 2) * (uint64_t)grid_blocks;
    if (fblocks > cap) fblocks = cap;
#ifdef KARMA_AB
    if (em == 6)
        hipLaunchKernelGGL(k_ragged_finalize<6>, dim3((unsigned)fblocks), dim3(1024), 0, s, a);
    else
#endif
    if (em & 2)
        hipLaunchKernelGGL(k_ragged_finalize<2>, dim3((unsigned)fblocks), dim3(1024), 0, s, a);
#ifdef KARMA_AB
    else
        hipLaunchKernelGGL(k_ragged_finalize<0>, dim3((unsigned)fblocks), dim3(1024), 0, s, a);
#endif
    return hipGetLastError();
}

KB_DEFINE_COLLECT(ragged)
#ifdef KARMA_AB
WLOG_SETTER(ragged)
#endif

}  // namespace engine
}  // namespace karma
