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
#include "karma_crc32c.h"
#include "wavelog.h"

namespace karma {
namespace engine {
namespace {

using namespace dev;

constexpr int kRaggedPF = 4;       // chunk loads in flight per lane: the small-record kernel
constexpr int kRaggedUnitsPF = 6;  // ... and the units kernel (k_units_ragged)
constexpr bool kRaggedNT = true;
// A ragged record's unaligned head bytes are stepped by the plan (the entering register goes
// into the first unit's descriptor), its tail bytes by finalize.  Stepping both edges in the
// units kernel from the lines it loads anyway saved the plan and finalize 15 us of scattered
// reads on configs[2] but cost the units kernel as much (round 2).

static_assert(kScanBlock % 64 == 0 && kScanBlock <= 1024 && kScanBlock >= kBuckets, "scan block shape");
constexpr uint64_t kU = kDefaultUnit;  // ragged units: absolute kU-byte boundaries
constexpr int kUShift = __builtin_ctzll(kDefaultUnit);
static_assert((kU & (kU - 1)) == 0, "unit size is a power of two");

// Unit layout of one record [p, e): its whole 16-byte blocks [a, b) = [floor16(p), ceil16(e))
// (g.a, g.b; the h = p - a bytes before the record and the t = b - e after it are masked to zero
// where the units kernel loads them), cut at absolute multiples of U = unit_bytes.  Unit j =
// [max(a, (A0+j)U), min(b, (A0+j+1)U)), A0 = a/U, k = ceil(b/U) - A0.  Only the first and the
// last unit can be partial.  Records with no aligned 16-byte block inside (g.is_short) have no
// units: finalize steps them alone.
struct RecUnits {
    Geom g;
    uint32_t h, t;   // masked head / tail bytes (< 16)
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

__device__ __forceinline__ RecUnits rec_units_at(const uint8_t* p, uint32_t n) {
    RecUnits u;
    u.g = geom(p, n);
    u.k = u.full = 0;
    u.part0 = u.part1 = u.c0 = u.c1 = u.last = 0;
    u.h = u.t = 0;
    if (!u.g.is_short) {
        u.g.a = floor16(p);  // the whole blocks
        u.g.b = ceil16(u.g.e);
        u.h = (uint32_t)(p - u.g.a);
        u.t = (uint32_t)(u.g.b - u.g.e);
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
__device__ __forceinline__ RecUnits rec_units(const RaggedArgs& A, uint64_t r) {
    return rec_units_at(A.arena + A.off[r], A.len[r]);
}

// Inclusive wave scan of 64-bit values, through DPP as wave_incl_scan32 (each step moves both
// halves).  Every lane of the wave must be active.
__device__ __forceinline__ uint64_t wave_incl_scan(uint64_t x) {
    x += dpp64<0x111, 0xf>(0ull, x);  // row_shr:1
    x += dpp64<0x112, 0xf>(0ull, x);  // row_shr:2
    x += dpp64<0x114, 0xf>(0ull, x);  // row_shr:4
    x += dpp64<0x118, 0xf>(0ull, x);  // row_shr:8
    x += dpp64<0x142, 0xa>(0ull, x);  // row_bcast:15 -> rows 1, 3
    x += dpp64<0x143, 0xc>(0ull, x);  // row_bcast:31 -> rows 2, 3
    return x;
}
// The sum over the wave (uniform).
__device__ __forceinline__ uint64_t wave_sum64(uint64_t x) {
    x = wave_incl_scan(x);
    return ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(x >> 32), 63) << 32) |
           (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)x, 63);
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

// An LDS counter per key, bumped by the lanes that want it: when every such lane of the wave has
// the same key (a batch of equal records: every lane of a plan block on one bucket, whose
// same-word atomics serialise, ~6 us of the aligned 4 KiB plan) one lane adds their number and
// the others take consecutive slots after it; otherwise one atomic per lane.  Returns the lane's
// slot (the counter's value for it).  Every lane calls this.
template <typename T>
__device__ __forceinline__ T lds_bump(T* cnt, uint32_t key, bool want) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint64_t m = __ballot(want);
    if (!m) return 0;
    const int l0 = __ffsll((long long)m) - 1;
    const uint32_t k0 = (uint32_t)__builtin_amdgcn_readlane((int)key, l0);
    if (__ballot(want && key == k0) == m) {  // (uniform)
        T base = 0;
        if ((int)lane == l0) base = atomicAdd(&cnt[k0], (T)__popcll(m));
        base = (T)__shfl((long long)base, l0);
        return base + (T)__popcll(m & (lane ? (~0ull >> (64u - lane)) : 0ull));
    }
    return want ? atomicAdd(&cnt[key], (T)1) : (T)0;
}

// The unit descriptors of the block's records (one thread per record, every lane of the wave
// calls this).  fb: the slot of the record's first full unit; cnt: the block's partial-run
// cursors by chunk count (LDS); full slots at or past full_cap and any slot at or past
// unit_cap are dropped (only when a caller's total_len is below the true payload sum: capi.cc
// sizes full_cap for each record's widened block span; k_ragged_finalize steps such records
// alone).  The first unit carries the masked head bytes u.h and inj (~init moved back over the
// h % 4 masked bytes of its word by the plan), the last unit the masked tail bytes u.t.
__device__ void write_unit_descs(const RaggedArgs& A, const RecUnits& u, bool valid, uint64_t r, uint64_t fb,
                                 unsigned long long* cnt, uint64_t full_cap, uint32_t inj) {
    const uint32_t lane = threadIdx.x & 63u;
    const uintptr_t a = reinterpret_cast<uintptr_t>(u.g.a), b = reinterpret_cast<uintptr_t>(u.g.b);
    const uint64_t A0 = a >> kUShift;
    const uint32_t hw = u.h << kDescHeadShift, tw = u.t << kDescTailShift;
    const uint64_t slot0 = lds_bump(cnt, u.c0, valid && u.part0);
    const uint64_t slot1 = lds_bump(cnt, u.c1, valid && u.part1);
    if (valid) {
        A.fbase[r] = fb;
        if (u.part0) {  // (with k == 1 also the last unit)
            A.pslot[2 * r] = slot0;
            const uintptr_t e0 = ((A0 + 1) << kUShift) < b ? ((A0 + 1) << kUShift) : b;
            if (slot0 < A.unit_cap)
                A.desc[slot0] = UnitDesc{(uint64_t)a, (uint32_t)(e0 - a) | hw | (u.k == 1 ? tw : 0u), inj};
        }
        if (u.part1) {
            A.pslot[2 * r + 1] = slot1;
            const uintptr_t s1 = (A0 + u.k - 1) << kUShift;
            if (slot1 < A.unit_cap) A.desc[slot1] = UnitDesc{(uint64_t)s1, (uint32_t)(b - s1) | tw, 0u};
        }
    }
    // Full units of the wave's 64 records are consecutive slots: the wave writes them together,
    // lane i taking slot F0 + i and finding its record by a search over the lanes' inclusive
    // unit counts, so the stores are coalesced and balanced however skewed the record sizes are.
    const uint64_t nfull = valid ? u.full : 0;
    const uint64_t incl = wave_incl_scan32((uint32_t)nfull);  // (a record's full units < 2^19: a wave's < 2^25)
    const uint64_t T = __shfl(incl, 63);
    const uint64_t F0 = __shfl(fb, 0);
    for (uint64_t base = 0; base < T; base += 64) {  // uniform trip count: shuffles see every lane
        const uint64_t i = base + lane;
        int o = 0;  // owner: the first lane whose inclusive count exceeds i
#pragma unroll
        for (int s = 32; s > 0; s >>= 1)
            if (__shfl(incl, o + s - 1) <= i) o += s;
        o = o < 63 ? o : 63;
        const uint64_t incl_o = __shfl(incl, o), full_o = __shfl(nfull, o), A0_o = __shfl(A0, o);
        const uint64_t k_o = __shfl(u.k, o);
        const uint32_t part0_o = __shfl(u.part0, o), inj_o = __shfl(inj, o), hw_o = __shfl(hw, o), tw_o = __shfl(tw, o);
        const uint64_t j = i - (incl_o - full_o) + part0_o;  // unit index within the owner's record
        const uint64_t slot = F0 + i;
        if (i < T && slot < full_cap)
            A.desc[slot] = UnitDesc{(A0_o + j) << kUShift, (uint32_t)kU | (j == 0 ? hw_o : 0u) | (j + 1 == k_o ? tw_o : 0u),
                                    j == 0 ? inj_o : 0u};
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

#ifdef KARMA_AB  // tools build: per-workgroup phase stamps of the plan and finalize (karma_ab_plan_log)
__device__ uint64_t* g_plan_log;
constexpr uint64_t kPlanLogBlocks = 4096;  // plan blocks logged; finalize's from 8 * kPlanLogBlocks on
#define PLAN_STAMP(base, i)                                                                    \
    do {                                                                                       \
        if (g_plan_log && threadIdx.x == 0 && blockIdx.x < kPlanLogBlocks)                     \
            g_plan_log[(base) + blockIdx.x * 8 + (i)] = wall_clock64();                        \
    } while (0)
// ... after this wave's loads and stores have completed (the stamp of a phase whose memory
// round trip is the point: wave 0 waits, the others run on)
#define PLAN_STAMP_DONE(base, i)                                                               \
    do {                                                                                       \
        if (g_plan_log && threadIdx.x < 64) __builtin_amdgcn_s_waitcnt(0);                     \
        PLAN_STAMP(base, i);                                                                   \
    } while (0)
#else
#define PLAN_STAMP(base, i) ((void)0)
#define PLAN_STAMP_DONE(base, i) ((void)0)
#endif

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
    excl += wave_sum64(lane <= k ? (w & kLbValueMask) : 0);  // (DPP)
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

// Wave 0 of plan block b, its counts published (lb_publish): sum the counts
// of the blocks before it (256 per step, newest first, each array until the first block that
// has published its inclusive total there), publish the inclusive totals and return the
// exclusive ones (uniform).  Every block it waits for has started (ids are taken in start
// order) and publishes its own counts before waiting on anything, so the wait ends.
// (lb_publish: the block's own counts, stored by the caller before it does other work)
__device__ __forceinline__ void lb_publish(const RaggedArgs& A, uint32_t seq, uint64_t b, uint64_t full_b, uint64_t part_b) {
    const uint64_t tag = (uint64_t)seq << 42;
    if (b > 0 && (threadIdx.x & 63u) == 0) {
        lb_store(A.lb + 1 + b, tag | kLbAgg | full_b);
        lb_store(A.lbp + b, tag | kLbAgg | part_b);
    }
}
__device__ void lookback(const RaggedArgs& A, uint32_t seq, uint64_t b, uint64_t full_b, uint64_t part_b,
                         uint64_t& exF, uint64_t& exP) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint64_t tag = (uint64_t)seq << 42;
    unsigned long long* lf = A.lb + 1;
    unsigned long long* lp = A.lbp;
    exF = exP = 0;
    if (b > 0) {
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
        lb_store(A.lb_ctl + 2, 0ull);  // k_units_ragged's dynamic wave-step counter
    }
}

// One pass over the records (plan block b = R x kScanBlock records, thread t the records
// (b R + i) kScanBlock + t, i < R): unit counts, the slots of the block's units from the
// look-back, the entering register over each record's unaligned head, and one 16-byte
// descriptor per unit.  Full units take slots [0, F) in record order; partial units
// [part_base, part_base + P), each block's run sorted by chunk count, longest first (the
// two-pass plan's order, which the units kernel streams 3 % faster on configs[2] than
// block-interleaved runs).  Replaces round 1's k_ragged_scan + k_ragged_desc: one launch, and
// no block reads every other block's totals.
// R (launch_ragged_main): enough records per thread that the plan blocks fit on the GPU at once
// (one per CU: 70 VGPRs).  A plan block is a chain of dependent memory round trips (its ticket,
// offsets and lengths, the look-back, the head blocks, the descriptor stores, ~16 us), so a
// second round of blocks doubles the plan: configs[2]'s 444 one-record blocks took 31 us, the
// last ones starting 17 us late (profiles/r05_plan_phases.json).  The head blocks are loaded
// with the offsets, before the scan and the look-back, not after them.
template <int R>
__global__ __launch_bounds__(kScanBlock) void k_ragged_plan(RaggedArgs A) {
    KB_SET_ARENA(A.kb_lo, A.kb_hi);
    PLAN_STAMP(0, 0);
    constexpr int NW = kScanBlock / 64;
    static_assert(R * NW <= 64, "one wave scans the block's wave totals");
    static_assert(2 * R * kScanBlock < 65536, "partial units of a block fit the packed scan's low 16 bits");
    __shared__ __attribute__((aligned(16))) uint32_t lds[2 * 1024];  // Z_1^-1, Z_2^-1
    // per round i (records (b R + i) kScanBlock + t): the partial runs are cut per kScanBlock
    // records, so the descriptor table is laid out as with one record per thread.  (The event window
    // around the units kernel still measures 0.2-2.3 % longer after an R > 1 plan on aligned
    // layouts, with this layout or one bucket run per block; the calls are shorter:
    // profiles/r05_plan_r1.txt, r05h_ragged.txt.)
    __shared__ unsigned long long cnt[R * kBuckets];
    __shared__ uint32_t hist[R * kBuckets];
    __shared__ uint64_t sm[R * NW];
    __shared__ uint64_t s_id, s_fbase;
    __shared__ uint32_t s_seq;
    if (threadIdx.x == 0) {
        s_id = atomicAdd(A.lb, 1ull);  // ids in start order (k_ragged_finalize resets the counter)
        s_seq = (uint32_t)lb_load(A.lb_ctl) + 1u;  // this call's tag (RaggedArgs::lb_ctl)
        if (s_id == 0) lb_store(A.lb_ctl + 1, s_seq);
    }
    copy_to_lds<2 * 1024, kScanBlock>(lds, A.comb_blob + kCombInv);
    for (uint32_t i = threadIdx.x; i < R * kBuckets; i += kScanBlock) hist[i] = 0;  // (R kBuckets may pass kScanBlock)
    __syncthreads();
    PLAN_STAMP(0, 1);  // id, tag and tables
    const uint64_t b = s_id;
    const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
    // per record only its pointer, length and init cross the barriers; the unit geometry is
    // recomputed from them.  The plan reads no record bytes: the units kernel masks the bytes
    // around a record in the blocks it loads anyway (group_unit's EDGES form).
    uint64_t packed[R];
    auto rec = [&](int i) { return (b * R + i) * kScanBlock + threadIdx.x; };
    // Every load is issued unconditionally (past the batch: the last record): a load under a
    // branch is waited for where the branches join, which would put the R records' round trips
    // one after another.
    const uint8_t* rp[R];
    uint32_t rn[R], ini[R];
#pragma unroll
    for (int i = 0; i < R; ++i) {
        const uint64_t ri = rec(i) < A.n_rec ? rec(i) : A.n_rec - 1;
        rp[i] = A.arena + A.off[ri];
        const uint32_t n = A.len[ri];
        rn[i] = rec(i) < A.n_rec ? n : 0u;
        ini[i] = A.init ? A.init[ri] : A.init_scalar;
    }
    PLAN_STAMP_DONE(0, 6);  // offsets and lengths landed
#pragma unroll
    for (int i = 0; i < R; ++i) {
        const RecUnits u = rec_units_at(rp[i], rn[i]);
        const bool valid = rec(i) < A.n_rec;
        (void)lds_bump(hist + i * kBuckets, u.c0, valid && u.part0);
        (void)lds_bump(hist + i * kBuckets, u.c1, valid && u.part1);
        // full units (high bits) and partial units (low 16 bits: at most 2 per record)
        packed[i] = valid ? (u.full << 16) | (u.part0 + u.part1) : 0;
    }
    uint64_t incl[R];
#pragma unroll
    for (int i = 0; i < R; ++i) {
        // full units (< 2^19 per record, < 2^25 per wave) and partial ones (<= 2 per record) scanned
        // apart in 32 bits, then packed as packed[i] is
        incl[i] = ((uint64_t)wave_incl_scan32((uint32_t)(packed[i] >> 16)) << 16) |
                  wave_incl_scan32((uint32_t)(packed[i] & 0xffffu));
        if (lane == 63) sm[i * NW + wave] = incl[i];
    }
    PLAN_STAMP(0, 7);  // counted, wave scans
    __syncthreads();
    if (wave == 0) {
        uint64_t t = lane < R * NW ? sm[lane] : 0;
        t = wave_incl_scan(t);
        if (lane < R * NW) sm[lane] = t;
    }
    __syncthreads();  // (hist complete)
    const uint64_t tot = sm[R * NW - 1];
    const uint64_t full_b = tot >> 16, part_b = tot & 0xffffu;
    PLAN_STAMP(0, 2);  // offsets and lengths read, block scan
    if (threadIdx.x < 64) lb_publish(A, s_seq, b, full_b, part_b);
    // each record's injection: ~init moved back over the h % 4 masked bytes before the record
    // within its first word (Z_1^-1, Z_2^-1; the record starts h bytes into its first block)
    uint32_t inj[R];
#pragma unroll
    for (int i = 0; i < R; ++i) {
        const uint32_t hb = (uint32_t)(reinterpret_cast<uintptr_t>(rp[i]) & 3u);
        uint32_t x = ~ini[i];
        if (hb & 1u) x = zmap(lds, 0, x);
        if (hb & 2u) x = zmap(lds, 1024, x);
        inj[i] = x;
    }
    PLAN_STAMP(0, 3);  // injections
    if (threadIdx.x < 64) {
        uint64_t exF, exP;
        lookback(A, s_seq, b, full_b, part_b, exF, exP);
        // the block's partial runs (round by round, longest bucket first): a wave scan of the
        // R x kBuckets counts, PER consecutive ones per lane
        {
            constexpr int NB = R * kBuckets, PER = (NB + 63) / 64;
            uint64_t loc[PER], sum = 0;
#pragma unroll
            for (int q = 0; q < PER; ++q) {
                const int o = (int)lane * PER + q, i = o / kBuckets, c = kBuckets - 1 - o % kBuckets;
                loc[q] = o < NB ? hist[i * kBuckets + c] : 0u;
                sum += loc[q];
            }
            unsigned long long run = A.part_base + exP + wave_incl_scan32((uint32_t)sum) - sum;  // (<= 2 R kScanBlock)
#pragma unroll
            for (int q = 0; q < PER; ++q) {
                const int o = (int)lane * PER + q, i = o / kBuckets, c = kBuckets - 1 - o % kBuckets;
                if (o < NB) cnt[i * kBuckets + c] = run;
                run += loc[q];
            }
        }
        if (threadIdx.x == 0) {
            s_fbase = exF;
            if (b + 1 == gridDim.x) {
                A.fbase[A.n_rec] = exF + full_b + exP + part_b;  // total units
                A.fbase[A.n_rec + 1] = exF + full_b;             // full units
            }
        }
    }
    __syncthreads();
    PLAN_STAMP(0, 4);  // look-back
#pragma unroll
    for (int i = 0; i < R; ++i) {
        const uint64_t run = (uint64_t)i * NW + wave;
        const uint64_t ex = ((run ? sm[run - 1] : 0) + incl[i] - packed[i]) >> 16;
        write_unit_descs(A, rec_units_at(rp[i], rn[i]), rec(i) < A.n_rec, rec(i), s_fbase + ex, cnt + i * kBuckets,
                         A.part_base, inj[i]);
    }
#ifdef KARMA_AB
    __syncthreads();
    PLAN_STAMP_DONE(0, 4 + 1);  // descriptors stored
#endif
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
    // wave-uniform: scalar registers, so no later use waits on the loads of fbase (vmcnt)
    m.U = uniform64(m.U);
    m.Fc = uniform64(m.Fc);
    m.shift = uniform64(m.shift);
    return m;
}

// Descriptor load through address space 1 (global_load_dwordx4, vmcnt only): a
// flat load would also count on lgkmcnt and stall the LDS lookups behind it.
__device__ __forceinline__ UnitDesc load_desc(const UnitDesc* d) {
    const u32x4 v = ldmeta16(d);
    return UnitDesc{v.x | ((uint64_t)v.y << 32), v.z, v.w};
}


// The units kernel: each unit's loads are issued when the unit starts (group_unit), the
// next descriptor is in flight meanwhile.  (A software-pipelined form, stream_unit's, measured
// 0.3-0.8 % slower on config 3 in round 2, unlike the fixed layout, where it wins 2.7 %; rebuilt
// in round 5 with ping-pong load sets and unbranched descriptor loads, so no wait drains a unit's
// loads, it still ran 0.1-0.8 % slower on every layout: profiles/r05_ragged_group_unit_pipe_ab.txt,
// DESIGN.md §4.)
// PF = 6 chunk loads in flight per lane (4: config 3 units 0.6736 vs 0.6680 ms, aligned 4 KiB
// records 0.6656 vs 0.6525; 8: no better than 4 -- profiles/r02_ragged_pf_ab.txt).  With one
// 1024-thread workgroup per CU (the 145 KiB LDS image) the chunks in flight per CU are what
// keeps HBM busy across the unit boundaries this kernel does not pipeline.
// The next wave-step of this wave (k_units_ragged): the block's static share from its LDS
// counter, then (dyn_shift) the dynamic tail, 16 steps per workgroup grab from lb_ctl[2], the
// chunk's base published in LDS by the wave that grabbed it.  Uniform over the wave.
__device__ __forceinline__ uint64_t ragged_next_step(const RaggedArgs& A, uint32_t* blk_next, uint32_t* blk_dyn,
                                                     uint32_t nidx, uint64_t S, uint64_t nws, uint64_t bw0,
                                                     uint64_t nwaves, uint32_t lane) {
    uint32_t i = 0;
    if (lane == 0) i = atomicAdd(blk_next, 1u);
    i = __builtin_amdgcn_readfirstlane(__shfl(i, 0));
    uint64_t wb_next = i < nidx ? bw0 + (i % kWavesPerBlock) + (uint64_t)(i / kWavesPerBlock) * nwaves : nws;
    if (i >= nidx && S < nws) {  // the static share is done: the dynamic tail
        const uint32_t k = i - nidx, c = k / kWavesPerBlock, j = k % kWavesPerBlock;
        uint32_t base = ~0u;
        if (c < kDynChunks) {
            if (j == 0) {  // this wave grabs the chunk (one round trip) and publishes its base
                if (lane == 0) {
                    base = (uint32_t)atomicAdd(A.lb_ctl + 2, (unsigned long long)kWavesPerBlock);
                    __hip_atomic_store(&blk_dyn[c], base, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                }
            } else if (lane == 0) {  // the chunk's grabber holds an earlier index: it is running
                while ((base = __hip_atomic_load(&blk_dyn[c], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) == ~0u)
                    __builtin_amdgcn_s_sleep(2);
            }
            base = __builtin_amdgcn_readfirstlane(__shfl((int)base, 0));
        }
        wb_next = base != ~0u && S + base + j < nws ? S + base + j : nws;
    }
    return wb_next;
}

#ifndef KARMA_UNITS_STEP_MODE  // (a build's default window step: 64 = the phased step4, whole-build A/B)
#define KARMA_UNITS_STEP_MODE 0
#endif
template <int PF = kRaggedUnitsPF, int MODE = KARMA_UNITS_STEP_MODE>
__global__ __launch_bounds__(kBlockThreads) void k_units_ragged(RaggedArgs A) {
    KB_SET_ARENA(A.kb_lo, A.kb_hi);
    __shared__ __attribute__((aligned(16))) uint32_t lds[kLdsWords];
    __shared__ uint32_t blk_next;  // the block's next wave-step (an LDS counter)
    __shared__ uint32_t blk_dyn[kDynChunks];  // dynamic tail: base of the block's c-th chunk of 16 steps
    if (threadIdx.x == 0) blk_next = kWavesPerBlock;
    for (uint32_t c = threadIdx.x; c < kDynChunks; c += blockDim.x) blk_dyn[c] = ~0u;
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
    // As k_units_fixed, the block's wave-steps b*16 + j + r*nwaves are taken in order from an
    // LDS counter, one step ahead (the next descriptor is loaded while a unit streams).  With
    // dyn_shift, the static shares end at S (whole rounds) and the last steps [S, nws) go to
    // whichever workgroup asks first: a unit here streams for tens of us, so static shares of the
    // last steps leave CUs idle while others finish.  A workgroup takes 16 steps
    // per global atomic (one wave grabs, its 15 siblings read the chunk's base from LDS): one
    // atomic per step on one address serialised at the memory side (~18 ns each, measured).
    const uint64_t nws = (U + kGroupsPerWave - 1) / kGroupsPerWave;
    uint64_t S = nws;
    if (A.dyn_shift) {
        const uint64_t d = min(nws >> A.dyn_shift, (uint64_t)kDynMaxSteps);
        const uint64_t s = (nws - d) / nwaves * nwaves;
        S = s >= nwaves ? s : nws;
    }
    const uint32_t nidx = (uint32_t)((S + nwaves - 1) / nwaves) * kWavesPerBlock;
    const uint64_t bw0 = (uint64_t)blockIdx.x * kWavesPerBlock;
    uint64_t wb = bw0 + (threadIdx.x >> 6);
    uint64_t u = wb * kGroupsPerWave + grp;
    UnitDesc d = u < U ? load_desc(A.desc + M.slot(u)) : UnitDesc{0, 0, 0};
    while (wb < nws) {
        const UnitDesc cur = d;
        const bool valid = u < U;
        const uint64_t wb_next = ragged_next_step(A, &blk_next, blk_dyn, nidx, S, nws, bw0, nwaves, lane);
        const uint64_t un = wb_next * kGroupsPerWave + grp;
        d = un < U ? load_desc(&KB_READ(A.desc, M.slot(un), A.unit_cap, kKbUnit)) : UnitDesc{0, 0, 0};
        const uint8_t* us = reinterpret_cast<const uint8_t*>(cur.us);
        const uint32_t span = cur.span & kDescSpanMask;
        const uint32_t R = group_unit<PF, kRaggedNT, true, MODE>(lds, X, l, us, us + span, us, cur.inj,
                                                           (cur.span >> kDescHeadShift) & 15u,
                                                           (cur.span >> kDescTailShift) & 15u);
        if (valid && l == 0) KB_WRITE(A.partial, M.slot(u), A.unit_cap, kKbUnit, R);
        WLOG_STEP();
        WLOG_UNIT(valid && l == 0, span);
        wb = wb_next;
        u = un;
    }
    WLOG_END(bw0 + (threadIdx.x >> 6));
}


#ifdef KARMA_AB
#include "ragged_ab.inc"  // the round-5 experiment forms of the units kernel (tools build only)
#endif

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
// ends, Z_last before the last unit), back over the t masked bytes after the record (Z_t^-1),
// ~R.  Records of more than 64 units: the whole wave folds all but the last unit with the
// 64-lane tree.  A wave takes FR x 64 consecutive records per pass (launch_ragged_main: enough
// that the grid fits the GPU at once, as the plan), and a record's loads go out in two dependent
// rounds for all FR of them: offsets, lengths, first-unit slot and partial slots (before the
// table fill), then the first ten unit contributions.  No record bytes are read.  (Round 4's
// one-record lanes took four dependent rounds -- geometry, slots, contributions, tail -- and 444
// blocks of them two rounds of blocks on configs[2]: 22 us, profiles/r05_plan_phases.json.)
// LITE (tools build A/B, round 6): the LDS fill skips the maps Z_{2U} .. Z_{64U} (24 of its 88 KiB),
// which only records of more than 64 units use; those fold with the maps read from the blob in
// global memory instead.
template <int FR, bool LITE = false>
__global__ __launch_bounds__(1024) void k_ragged_finalize(RaggedArgs A) {
    KB_SET_ARENA(A.kb_lo, A.kb_hi);
    __shared__ __attribute__((aligned(16))) uint32_t lds[kCombWords];
    PLAN_STAMP(8 * kPlanLogBlocks, 0);
    constexpr int MID = FR >= 4 ? 2 : 8;  // middle-unit contributions loaded with the first and the last
    const uint32_t lane = threadIdx.x & 63u;
    constexpr uint64_t U = kU;
    const uint64_t nwaves = (uint64_t)gridDim.x * (blockDim.x >> 6);
    const uint64_t full_cap = A.part_base ? A.part_base : A.unit_cap;
    uint64_t r0 = ((uint64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6)) * 64 * FR;
    // per record its pointer, length and slots; the unit geometry is recomputed from them
    bool valid[FR];
    uint32_t rn[FR];
    uint64_t fb[FR], ps0[FR], ps1[FR];
    const uint8_t* p[FR];
    // (every load unconditional -- past the batch: the last record; no unit: slot 0 -- so the
    // FR records' loads go out together: loads under branches are waited for at the join)
    auto stage1 = [&](uint64_t base) {
#pragma unroll
        for (int j = 0; j < FR; ++j) {
            const uint64_t r = base + (uint64_t)j * 64 + lane;
            valid[j] = r < A.n_rec;
            const uint64_t rc = valid[j] ? r : A.n_rec - 1;
            p[j] = A.arena + A.off[rc];
            const uint32_t n = A.len[rc];
            rn[j] = valid[j] ? n : 0u;
            fb[j] = A.fbase[rc];
            ps0[j] = A.pslot[2 * rc];  // (read whether or not the unit is partial: no wait on the geometry)
            ps1[j] = A.pslot[2 * rc + 1];
        }
    };
    // (Round 5 measured the first pass's unit-state loads issued before the table stores, so the
    // table fill and those loads share a round trip: finalize 13.1 against 12.6 us, calls equal,
    // profiles/r05_finalize_overlap_ab.txt -- its first loads are bandwidth, not latency.)
    if (r0 < A.n_rec) stage1(r0);
    if constexpr (LITE) {
        load_comb_tables<1024, 1024>(lds, A.comb_blob);
        load_comb_tables<kCombWords - kCombZ4, 1024>(lds + kCombZ4, A.comb_blob + kCombZ4);
    } else {
        load_comb_tables<kCombWords, 1024>(lds, A.comb_blob);
    }
    const uint32_t* big = LITE ? A.comb_blob : lds;  // the maps Z_{2^k U} of the huge records' fold
    __syncthreads();
    PLAN_STAMP(8 * kPlanLogBlocks, 1);  // tables
    // the plan's look-back words are retired after the first contributions are issued: its
    // control-word load waits for every load issued before it (vmcnt counts in order)
    bool retired = !A.lb;
    while (r0 < A.n_rec) {  // (wave-uniform)
        bool ok[FR];
        uint32_t first[FR], lastc[FR], mid[FR][MID];
#pragma unroll
        for (int j = 0; j < FR; ++j) {
            const RecUnits u = rec_units_at(p[j], rn[j]);
            ok[j] = valid[j] && fb[j] + u.full <= full_cap && (!u.part0 || ps0[j] < A.unit_cap) &&
                    (!u.part1 || ps1[j] < A.unit_cap);
            const uint64_t k = u.k;
            const bool any = ok[j] && k > 0;
            const uint64_t s0 = unit_slot(0, k, fb[j], ps0[j], ps1[j], u.part0, u.part1);
            const uint64_t s1 = unit_slot(k - 1, k, fb[j], ps0[j], ps1[j], u.part0, u.part1);
            first[j] = A.partial[any && k <= 64 ? s0 : 0];
            lastc[j] = A.partial[any && k >= 2 ? s1 : 0];
#pragma unroll
            for (int q = 0; q < MID; ++q)
                mid[j][q] = A.partial[ok[j] && k <= 64 && (uint64_t)q + 2 < k ? fb[j] + 1 + q - u.part0 : 0];
        }
        if (!retired) {
            lookback_retire(A);
            retired = true;
        }
        PLAN_STAMP_DONE(8 * kPlanLogBlocks, 2);  // (first pass) contributions loaded
        // the FR records' Horner chains (serial LDS lookups) side by side, then the rare records
        // of more than 64 units, then the last units, tails and stores
        uint32_t acc[FR];
        bool huge[FR];
#pragma unroll
        for (int j = 0; j < FR; ++j) {
            const RecUnits u = rec_units_at(p[j], rn[j]);
            const uint64_t k = u.k;
            acc[j] = 0;
            huge[j] = ok[j] && k > 64;
            if (ok[j] && k > 0 && k <= 64) {
                acc[j] = first[j];
#pragma unroll
                for (int q = 0; q < MID; ++q)
                    if ((uint64_t)q + 2 < k) acc[j] = zmap(lds, 0, acc[j]) ^ mid[j][q];
                for (uint64_t m = 1 + MID; m + 1 < k; m += 8) {  // more middle units: 8 loads in flight
                    uint32_t s[8];
#pragma unroll
                    for (int q = 0; q < 8; ++q) s[q] = m + q + 1 < k ? A.partial[fb[j] + m + q - u.part0] : 0u;
#pragma unroll
                    for (int q = 0; q < 8; ++q)
                        if (m + q + 1 < k) acc[j] = zmap(lds, 0, acc[j]) ^ s[q];
                }
            }
        }
#pragma unroll
        for (int j = 0; j < FR; ++j) {
            uint64_t hm = __ballot(huge[j]);
            while (hm) {
                const int h = __ffsll((long long)hm) - 1;
                hm &= hm - 1;
                const RecUnits u = rec_units_at(p[j], rn[j]);
                const uint64_t hk = __shfl(u.k, h) - 1;  // all units but the last
                const uint64_t hfb = __shfl(fb[j], h), hps0 = __shfl(ps0[j], h);
                const uint32_t hp0 = __shfl(u.part0, h);
                const uint64_t nb = (hk + 63) / 64;
                const int64_t pad = (int64_t)(nb * 64 - hk);
                uint32_t w = 0;
                for (uint64_t blk = 0; blk < nb; ++blk) {
                    const int64_t idx = (int64_t)(blk * 64 + lane) - pad;
                    uint32_t v = 0;
                    if (idx >= 0) v = A.partial[idx == 0 && hp0 ? hps0 : hfb + idx - hp0];
                    v = wave_tree(big, v);
                    w = zmap(big, 6 * 1024, w) ^ v;
                }
                w = __shfl(w, 0);
                if ((int)lane == h) acc[j] = w;
            }
        }
#pragma unroll
        for (int j = 0; j < FR; ++j) {
            const RecUnits u = rec_units_at(p[j], rn[j]);
            const uint64_t r = r0 + (uint64_t)j * 64 + lane;
            const uint64_t k = u.k;
            uint32_t c = acc[j];
            if (ok[j] && k >= 2) c = shift_last(lds, c, u.last, U) ^ lastc[j];  // the last unit: its own length
            if (ok[j] && k > 0) {  // back over the t masked bytes after the record: Z_t^-1 (t < 16)
#pragma unroll
                for (int i = 0; i < 4; ++i)
                    if ((u.t >> i) & 1u) c = zmap(lds, kCombInv + i * 1024, c);
            }
            if (valid[j]) {
                uint32_t res;
                if (ok[j] && k > 0)
                    res = ~c;
                else  // a short record, or (the caller's total_len was low) one whose units did not
                      // fit the table: this lane steps it alone -- slow, but never a wrong CRC
                    res = short_record(lds, kCombZ4, kCombT8, p[j], rn[j], A.init ? A.init[r] : A.init_scalar);
                A.out[r] = res;
            }
        }
        r0 += nwaves * 64 * FR;
        if (r0 < A.n_rec) stage1(r0);
    }
    if (!retired) lookback_retire(A);  // (a wave with no records)
#ifdef KARMA_AB
    __syncthreads();
    PLAN_STAMP_DONE(8 * kPlanLogBlocks, 3);  // records folded and stored
#endif
}

// The uniform-stride pass's slots (engine.h WalSpec): segment 0's start at f (replay's start), m0
// slots there, m in every later segment, sigma = n + 8 bytes apart; slot g in WAL order, its
// header at rel(g) bytes from the image start; B0 / B batches of 64 slots per segment.
struct SpecGeom {
    uint64_t S, f;
    uint32_t n, sig, m, m0, B, B0;
    bool type0;  // the first header's type is 0
    __device__ __forceinline__ uint64_t rel(uint64_t g) const {
        if (g < m0) return f + g * sig;
        const uint64_t h = g - m0;
        return (1 + h / m) * S + (h % m) * sig;
    }
};

// The summary (engine.h WalSummary::spec), by wave 0 of the SPEC kernel's last workgroup: from the
// keys, written word by word to the page-locked A.spec_out (system scope, as k_wal_publish); then
// the keys, the flag and the ticket counter are reset for the next call.  scratch: 16 dwords of
// this wave's LDS stage.
__device__ void spec_finish(const RaggedArgs& A, bool ok, const SpecGeom& G, uint32_t lane, uint32_t* scratch) {
    WalSpec* P = A.spec;
    if (lane == 0) {
        const unsigned long long ks = __hip_atomic_load(&P->stop_key, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const unsigned long long kd = __hip_atomic_load(&P->dev_key, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const uint32_t skew = __hip_atomic_load(&P->skew, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        WalSummary r{};
        r.stage_skew = skew;
        r.first_bad = ~0ull;
        if (!ok) {  // no stride for this kernel: 3 = a record of another size class (the host
                    // takes the other kernel next call), 2 = none at all
            r.spec = G.n >= 1 && G.n <= kSpecDirectMax && G.f + G.sig <= G.S && G.type0 ? 3 : 2;
            r.max_len = G.n;
        } else if (kd < ks) {
            r.spec = 2;  // declined: the walk decides
        } else {
            r.spec = 1;
            r.w1 = G.m;
            r.max_len = G.n;
            if (ks == ~0ull) {  // every segment ended cleanly
                r.n_all = G.m0 + (A.spec_nseg - 1) * (uint64_t)G.m;
                r.status = KARMA_WAL_END;
                r.end = A.spec_wal_end;
            } else {
                // slot g's header (key 2 g), or the header after a segment's last slot g (2 g + 1)
                const uint64_t g = ks / 2, rel = G.rel(g) + ((ks & 1) ? G.sig : 0u);
                r.n_all = (ks + 1) / 2;
                r.status = KARMA_WAL_CORRUPT;
                r.end = A.spec_base0 + rel;
                r.bad_off = rel;
            }
        }
        const uint32_t* w = reinterpret_cast<const uint32_t*>(&r);
        for (uint32_t i = 0; i < sizeof(WalSummary) / 4; ++i) scratch[i] = w[i];
        __hip_atomic_store(&P->stop_key, ~0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(&P->dev_key, ~0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(&P->skew, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(&P->done, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    wave_lds_sync();
    // every word but `spec`, then (their stores complete) `spec`: a host that sees spec != 0 sees the rest
    constexpr uint32_t kWords = sizeof(WalSummary) / 4, kSpecWord = offsetof(WalSummary, spec) / 4;
    static_assert(sizeof(WalSummary) % 4 == 0 && kWords <= 64, "one word per lane");
    uint32_t* out = reinterpret_cast<uint32_t*>(A.spec_out);
    if (lane < kWords && lane != kSpecWord)
        __hip_atomic_store(out + lane, scratch[lane], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __builtin_amdgcn_s_waitcnt(0);
    if (lane == 0) __hip_atomic_store(out + kSpecWord, scratch[kSpecWord], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}


// The geometry from replay's first len/type word st (uniform): a stride for payloads in [lo, hi].
__device__ __forceinline__ bool spec_geom(const RaggedArgs& A, uint32_t st, uint32_t lo, uint32_t hi, SpecGeom& G) {
    G = SpecGeom{A.spec_seg, A.spec_first, st >> 8, (st >> 8) + 8, 1u, 1u, 1u, 1u, (st & 0xffu) == 0};
    const bool ok = G.type0 && G.n >= lo && G.n <= hi && G.f + G.sig <= G.S;
    if (ok) {
        G.m = (uint32_t)(G.S / G.sig);
        G.m0 = (uint32_t)((G.S - G.f) / G.sig);
        G.B = (G.m + 63) / 64;
        G.B0 = (G.m0 + 63) / 64;
    }
    return ok;
}
__device__ __forceinline__ uint64_t spec_batches(const RaggedArgs& A, const SpecGeom& G) {
    return G.B0 + (A.spec_nseg - 1) * (uint64_t)G.B;
}

// Batch bi (uniform): segment 0's B0 batches, then B per segment.  This lane's slot: its header
// offset o (from the image start = arena - 8), payload n (0: no slot), the batch's first slot g0
// and whether the slot is its segment's last with a header after it in the segment.
__device__ __forceinline__ void spec_slot(const RaggedArgs& A, const SpecGeom& G, uint32_t bi, uint32_t lane, uint64_t& o,
                                          uint32_t& n, uint64_t& g0, bool& lastf) {
    uint32_t sg = 0, j = bi, mm = G.m0;
    uint64_t pos0 = G.f, gb = 0;
    if (bi >= G.B0) {
        const uint32_t t = bi - G.B0;
        sg = 1 + t / G.B;
        j = t - (sg - 1) * G.B;
        mm = G.m;
        pos0 = (uint64_t)sg * G.S;
        gb = G.m0 + (uint64_t)(sg - 1) * G.m;
    }
    const uint32_t i = 64u * j + lane;
    const bool v = sg < A.spec_nseg && i < mm;
    o = pos0 + (uint64_t)i * G.sig;
    n = v ? G.n : 0u;
    g0 = gb + 64u * j;
    lastf = v && i == mm - 1 && (uint64_t)sg * G.S + G.S - (pos0 + (uint64_t)mm * G.sig) >= 8;
}

__device__ __forceinline__ void read_hdr(const uint8_t* hp, uint32_t& hc, uint32_t& hs) {
    hc = (uint32_t)hp[0] | (uint32_t)hp[1] << 8 | (uint32_t)hp[2] << 16 | (uint32_t)hp[3] << 24;
    hs = (uint32_t)hp[4] | (uint32_t)hp[5] << 8 | (uint32_t)hp[6] << 16 | (uint32_t)hp[7] << 24;
}

// Slot g against its header (hc, hs) and payload CRC res; when lastf, also the header after the
// segment's last slot, at tp (key 2 g + 1).
__device__ __forceinline__ void spec_keys(const SpecGeom& G, uint32_t hc, uint32_t hs, uint32_t res, uint64_t g,
                                          bool lastf, const uint8_t* tp, unsigned long long& kstop,
                                          unsigned long long& kdev) {
    if (hs == (G.n << 8)) {  // the record the stride says: scan_record checks its CRC
        if (res != hc) kstop = 2 * g;
    } else if (hs == 0 && hc == 0) {  // an all-zero header: "Corrupt record" (size-0 quirk)
        kstop = 2 * g;
    } else {  // anything else: the stride's assumption ends here
        kdev = 2 * g;
    }
    if (lastf) {  // scan_record at the header after the segment's last slot
        uint32_t tc, ts;
        read_hdr(tp, tc, ts);
        const unsigned long long key = 2 * g + 1;
        if ((ts & 0xffu) == 1u) {
            // padding: the next segment
        } else if (tc == 0 && ts == 0) {
            kstop = key < kstop ? key : kstop;
        } else {
            kdev = key < kdev ? key : kdev;
        }
    }
}

// The wave's smallest keys to spec->stop_key / dev_key (returning atomics: the epilogue's wait
// covers them); true when it had any (uniform): the wave is then done -- its later slots have
// larger keys, which change neither the first stop nor whether a break comes before it.
__device__ __forceinline__ bool spec_report(const RaggedArgs& A, unsigned long long kstop, unsigned long long kdev,
                                            uint32_t lane) {
    if (!__ballot(kstop != ~0ull || kdev != ~0ull)) return false;
    kstop = wave_min64(kstop);
    kdev = wave_min64(kdev);
    if (lane == 0) {
        unsigned long long r0 = 0, r1 = 0;
        if (kstop != ~0ull) r0 = __hip_atomic_fetch_min(&A.spec->stop_key, kstop, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (kdev != ~0ull) r1 = __hip_atomic_fetch_min(&A.spec->dev_key, kdev, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        asm volatile("" ::"v"(r0), "v"(r1));
    }
    return true;
}

// Every thread of the workgroup: the stage flag, then a ticket; the last workgroup to finish writes
// the summary (spec_finish, wave 0, scratch: 16 dwords of LDS).  Every wave's key atomics have
// returned before its workgroup takes a ticket, so the last ticket's loads see the final keys.
__device__ void spec_epilogue(const RaggedArgs& A, bool ok, const SpecGeom& G, bool poor_seen, uint32_t* scratch) {
    const uint32_t lane = threadIdx.x & 63u;
    if (poor_seen && lane == 0) {
        const uint32_t r = __hip_atomic_fetch_or(&A.spec->skew, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        asm volatile("" ::"v"(r));
    }
    __builtin_amdgcn_s_waitcnt(0);
    __syncthreads();
    __shared__ uint32_t s_last;
    if (threadIdx.x == 0)
        s_last = __hip_atomic_fetch_add(&A.spec->done, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1u == gridDim.x;
    __syncthreads();
    if (s_last && threadIdx.x < 64) spec_finish(A, ok, G, lane, scratch);
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
// lines per instruction; one record per lane: 0.327).
// SPEC (the uniform-stride WAL replay, payloads up to kSpecDirectMax): the slots of spec_slot, 64 per
// wave as k_ragged_staged_pipe's SPEC form takes them, each slot's header read from global memory
// beside its CRC; the same keys, wave exit and last-workgroup summary.
template <bool SPEC = false>
__global__ __launch_bounds__(kBlockThreads) void k_ragged_direct4(RaggedArgs A) {
    constexpr int G = 4;
    uint64_t n_rec = A.n_rec;
    if (A.n_dev) {  // a device-sized batch: the count is known on the device only
        if (*A.gate_len > A.gate_max || *A.gate_len < A.gate_min) return;
        n_rec = *A.n_dev;
    }
    KB_SET_ARENA_SAFE(A.kb_lo, A.kb_hi, A.blob, A.blob + kBlobWords);  // the blob: empty units' address
    uint32_t sp_st = 0;  // (SPEC: replay's first len/type word, loaded beside the table fill)
    if constexpr (SPEC) {
        uint32_t crc0;
        read_hdr(KB_BYTES(A.arena - 8 + A.spec_first, 8), crc0, sp_st);
    }
    __shared__ __attribute__((aligned(16))) uint32_t lds[kLdsWords];
    load_stream_tables(lds, A.blob);
    __syncthreads();
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t X = lane_const();
    const uint8_t* safe = reinterpret_cast<const uint8_t*>(A.blob);  // 16-aligned, always mapped
    const uint64_t nwaves = (uint64_t)gridDim.x * kWavesPerBlock;
    SpecGeom SG{};
    bool sp_ok = false;
    if constexpr (SPEC) {
        sp_ok = spec_geom(A, sp_st, 1u, kSpecDirectMax, SG);
        n_rec = sp_ok ? spec_batches(A, SG) * 64 : 0;
    }
    for (uint64_t base = ((uint64_t)blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6)) * 64; base < n_rec;
         base += nwaves * 64) {
        const uint64_t ri = base + lane;
        bool vi = ri < n_rec;
        const uint8_t* pi;
        uint32_t ni, initi;
        uint64_t g0 = 0;
        bool lastf = false;
        if constexpr (SPEC) {
            uint64_t o;
            spec_slot(A, SG, (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(base >> 6)), lane, o, ni, g0, lastf);
            vi = ni != 0;
            pi = A.arena + o;
            initi = 0u;
        } else {
            pi = vi ? A.arena + A.off[ri] : A.arena;
            ni = vi ? A.len[ri] : 0u;
            initi = vi ? (A.init ? A.init[ri] : A.init_scalar) : 0u;
        }
        const uint32_t res = direct_batch<G, kRaggedPF, kRaggedNT, 0>(lds, X, safe, pi, ni, initi, vi);
        if constexpr (SPEC) {
            unsigned long long kstop = ~0ull, kdev = ~0ull;
            if (vi) {
                uint32_t hc, hs;
                read_hdr(KB_BYTES(pi - 8, 8), hc, hs);
                spec_keys(SG, hc, hs, res, g0 + lane, lastf, KB_BYTES(pi + ni, lastf ? 8u : 0u), kstop, kdev);
            }
            if (spec_report(A, kstop, kdev, lane)) break;
        } else if (vi) {
            A.out[ri] = res;
            if (A.cmp_stored && ni && res != A.cmp_stored[ri]) atomicMin(A.cmp_bad, (unsigned long long)ri);
        }
    }
    if constexpr (SPEC) {
        __shared__ uint32_t scratch[16];
        spec_epilogue(A, sp_ok, SG, false, scratch);
    }
}

// The staged kernel software-pipelined across batches: batch k + 1's extent and batch k + 2's
// offsets / lengths are in flight while batch k is stepped (a wave's batches are otherwise one
// chain of three memory latencies and the steps: DESIGN.md §8a), plain scalars across the loop.
// The records' windows are aligned to their ends (lane_record_end: no head or tail steps); the
// stage holds the extent 16 bytes in, after a slack the first window may read.  When a batch's
// records start on few LDS banks the stage is bank-skewed, one pad dword after every 128 bytes
// (dword q at q + q / 32), so records whose stride is a multiple of 32 bytes (120-B payloads +
// 8-B headers put every lane on one bank) read their windows without conflicts; stores then go
// out as dwords.  The 16-copy stride image is read with lanes 16-31 taking the tables in swapped
// order (stride_step16s: no bank conflicts; the plain order measured 2-way conflicts).
// SK: the kernel carries the skewed stage beside the plain one (a second code path: 172 VGPRs,
// 3-5 us on 188-B strides); without it a bank-poor batch is staged plainly (correct, with bank
// conflicts).  Either form reports bank-poor batches in *stage_skew_seen, so the WAL replay picks
// the next call's form from this one's records.
// R8 (plain stage only): the 8-copy stride image (32 KiB, stride_step8) instead of the 16-copy
// one, so kStgWaves8 waves' stages fit the LDS (the plain form's 146 VGPRs allow 3 waves per SIMD).
// TM (timing attribution, tools build only, wrong CRCs): 1 = no CRC steps (each lane xors one
// stage word into its result), 2 = no record loads or stage stores (the steps run over whatever
// the stage holds), 3 = neither.
// WIDE (not with R8): lane_record_end's phased window loop (SMODE bit 6): every LDS read of a
// window in flight together, one round trip per window (tools build A/B KARMA_SPEC_WIDE=0 /
// KARMA_STAGE_WIDE=0: the loop the compiler schedules, two; 1M x 180 B uniform pass 52.8 -> 51.1
// us, profiles/r06_staged_phased_window_ab.txt).
// AL (with WIDE): the phased loop's fast path for windows that are whole stage dwords (every active
// lane's sh == 0: no funnel shifts; 52.7 -> 51.9 us on 180 B, profiles/r06_staged_aligned_path_ab.txt;
// tools build KARMA_SPEC_AL=0: without it).
// NWO (tools build A/B, with R8): that many waves instead of kStgWaves8, leaving LDS for another
// kernel's workgroups on the same CU (the sliced WAL replay's walkers, wal.cc).
// SPEC (the uniform-stride WAL replay, engine.h WalSpec): every workgroup reads segment 0's first
// header (the stride; a header that gives none ends the kernel, workgroup 0 records it), the
// records are then the slots of a_spec_nseg segments, a batch the 64 slots of one segment from
// 64 j (batch b: segment b / B, j = b % B), each with its 8-byte header in front (arena = image
// + 8; the extent starts at the first header); no lists are read and no CRCs stored.  Per slot:
// its header against (n, type 0) and its payload CRC against the header's field; a segment's last
// batch also classifies the header after its last slot.  The wave's smallest keys go to
// spec->stop_key / dev_key by one atomicMin, and the wave then ends: its later slots have larger
// keys, which can change neither the first stop nor whether a break comes before it.
template <bool SK, bool R8 = false, int TM = 0, int NWO = 0, bool SPEC = false, bool P2 = false, bool WIDE = !R8,
          bool AL = WIDE>
__global__ __launch_bounds__((NWO ? NWO : R8 ? kStgWaves8 : kStgWaves) * 64) void k_ragged_staged_pipe(RaggedArgs A) {
    static_assert(!P2 || SPEC, "two batches in flight: the uniform-stride form only");
    static_assert(!(SK && R8), "the 8-copy form has the plain stage only");
    static_assert(!(SPEC && NWO), "the uniform-stride form has no wave-count override");
    static_assert(!(WIDE && R8), "the phased window loop reads the 16-copy image");
    constexpr bool END = true;
    constexpr int NW = NWO ? NWO : R8 ? kStgWaves8 : kStgWaves, SMODE = R8 ? 32 : WIDE ? (AL ? 216 : 88) : 24;
    constexpr int TW = R8 ? kRep8Words : kRep16Words, Z4 = TW, T8 = TW + 1024, BUF = TW + 1280;
    constexpr uint32_t kLead = 16u, kFit = kStgBytes - 32u;
    constexpr uint32_t kStride = SK ? kStgBytes + kStgBytes / 32 : kStgBytes;  // bytes per wave's stage
    uint64_t n_rec = A.n_rec;
    if (A.n_dev) {
        if (*A.gate_len > A.gate_max || *A.gate_len < A.gate_min) return;
        n_rec = *A.n_dev;
    }
    if (n_rec == 0) return;  // (uniform: a device-sized batch with nothing in it skips the table fill)
    KB_SET_ARENA(A.kb_lo, A.kb_hi);
    // SPEC: segment 0's first len/type word, loaded beside the table fill
    uint32_t sp_st = 0;
    if constexpr (SPEC) {
        const uint8_t* h0 = KB_BYTES(A.arena - 8 + A.spec_first, 8);
        sp_st = (uint32_t)h0[4] | (uint32_t)h0[5] << 8 | (uint32_t)h0[6] << 16 | (uint32_t)h0[7] << 24;
    }
    __shared__ __attribute__((aligned(16))) uint32_t lds[BUF + NW * (int)(kStride / 4)];
    static_assert((BUF + NW * (int)(kStride / 4)) * 4 <= 160 * 1024, "LDS of one workgroup");
    if constexpr (R8) {
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
    // SPEC: the slots (uniform); every wave reaches the epilogue
    SpecGeom G{};
    bool sp_ok = false;
    if constexpr (SPEC) {
        sp_ok = spec_geom(A, sp_st, 1u, kStgGateLen, G);
        n_rec = sp_ok ? spec_batches(A, G) * 64 : 0;
    } else if (base >= n_rec) {
        return;
    }
    // (SPEC: g0 the batch's first slot, lastf this lane's slot is its segment's last and a header
    // follows it in the segment)
    auto ld_meta = [&](uint64_t b, uint64_t& o, uint32_t& n, uint32_t& ini, uint64_t& g0, bool& lastf) {
        if constexpr (SPEC) {  // arithmetic, no loads
            spec_slot(A, G, (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(b >> 6)), lane, o, n, g0, lastf);
            ini = 0u;
            return;
        }
        (void)g0;
        (void)lastf;
        const uint64_t ri = b + lane;
        const bool v = ri < n_rec;
        o = v ? A.off[ri] : 0;
        n = v ? A.len[ri] : 0u;
        ini = v ? (A.init ? A.init[ri] : A.init_scalar) : 0u;
    };
    auto extent = [&](uint64_t o, uint32_t n, uintptr_t& lo, uintptr_t& hi) {
        if constexpr (SPEC) {  // consecutive slots from lane 0: arithmetic (no wave reduction)
            const uint64_t live = __ballot(n != 0);
            if (!live) {
                lo = hi = 0;
                return;
            }
            const uintptr_t p0 = reinterpret_cast<uintptr_t>(A.arena) + uniform64(o);  // (lane 0's slot)
            lo = (p0 - 8) & ~uintptr_t(15);
            hi = (p0 + (uint64_t)(__popcll(live) - 1) * G.sig + G.n + 15) & ~uintptr_t(15);
            return;
        }
        const uintptr_t p = reinterpret_cast<uintptr_t>(A.arena) + o;
        const uintptr_t p0 = SPEC ? p - 8 : p;  // (SPEC: from the record's header)
        uint64_t l = n ? (p0 & ~uintptr_t(15)) : ~0ull, h = n ? ((p + n + 15) & ~uintptr_t(15)) : 0ull;
        wave_prefix_minmax(l, h);  // (DPP; lane 63 holds the wave's)
        lo = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(l >> 32), 63) << 32) |
             (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)l, 63);
        hi = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(h >> 32), 63) << 32) |
             (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)h, 63);
    };
    u32x4 v[kStgVecs];
    auto issue_into = [&](u32x4 (&dst)[kStgVecs], uintptr_t lo, uintptr_t hi) {
        if constexpr ((TM & 2) != 0) return;
        const uint32_t nv = (uint32_t)((hi - lo) / 16);
#pragma unroll
        for (int q = 0; q < kStgVecs; ++q) {
            const uint32_t j = lane + 64u * q;  // past the extent: its first block again (no branch)
            dst[q] = ldg<true>(reinterpret_cast<const uint8_t*>(lo + 16ull * (j < nv ? j : 0u)));
        }
    };
    auto issue = [&](uintptr_t lo, uintptr_t hi) { issue_into(v, lo, hi); };
    auto store_stage = [&](const u32x4 (&src)[kStgVecs], bool sk) {
#pragma unroll
        for (int q = 0; q < kStgVecs; ++q) {
            uint32_t at = kLead + 16u * (lane + 64u * q);
            at = at >= kStgBytes ? 0u : at;  // (END) the last slot, past any extent, into the slack
            if (sk) {  // 4 dwords in one 128-byte line: contiguous after the skew
                const uint32_t d = at / 4 + at / 128;
                stage32[d] = src[q].x;
                stage32[d + 1] = src[q].y;
                stage32[d + 2] = src[q].z;
                stage32[d + 3] = src[q].w;
            } else {
                *reinterpret_cast<u32x4*>(stage + at) = src[q];
            }
        }
        wave_lds_sync();
    };
    // batch `base`: meta (o, n, ini), extent; batch base + step: meta (o2, n2, ini2)
    uint64_t o, o2, gq = 0, gq2 = 0;
    uint32_t n, ini, n2, ini2;
    bool lf = false, lf2 = false;
    uintptr_t lo, hi;
    ld_meta(base, o, n, ini, gq, lf);
    ld_meta(base + step, o2, n2, ini2, gq2, lf2);
    extent(o, n, lo, hi);
    bool fits = hi != 0 && hi - lo <= kFit;
    // does the batch at (o, n, lo) need the skewed stage?  (banks of the records' first dwords)
    bool poor_seen = false, poor_checked = false;
    auto skewed = [&](uint64_t o, uint32_t n, uintptr_t lo) {
        if constexpr (SPEC && !SK) {  // (one stride: the wave's first batch reports for the hint)
            if (poor_checked) return false;
            poor_checked = true;
        } else if (!SK && !A.stage_skew_seen) {
            return false;
        }
        const uintptr_t p = reinterpret_cast<uintptr_t>(A.arena) + o;
        uint32_t bits = n ? 1u << (((uint32_t)(p - lo) >> 2) & 31u) : 0u;
        bits = wave_or32(bits);
        // (a batch of fewer than 12 records -- a segment's last slots, the batch's end -- is poor
        // only when its records share banks)
        const uint32_t live = (uint32_t)__popcll(__ballot(n != 0));
        const bool poor = (uint32_t)__builtin_popcount(bits) < (live < 12u ? live : 12u);
        poor_seen |= poor;
        return SK && poor;
    };
    [[maybe_unused]] uint32_t tm_sink = 0;
    // One batch: each lane's record from the stage (or global memory), its CRC stored (lists) or
    // checked against its header (SPEC: true when the wave reported a key and is done).
    auto proc = [&](uint64_t base, uint64_t o, uint32_t n, uint32_t ini, uintptr_t lo, bool fits, bool sk, uint64_t gq,
                    bool lf) -> bool {
        const uint64_t ri = base + lane;
        [[maybe_unused]] uint32_t spec_res = 0;
        if (ri < n_rec) {
            uint32_t res = ini;
            const uintptr_t p = reinterpret_cast<uintptr_t>(A.arena) + o;
            if (n && (TM & 1) != 0) {
                res = ini ^ stage32[(kLead + (uint32_t)(p - lo)) / 4];
            } else if (n) {
                if (fits && END && n >= 4 && sk)
                    res = lane_record_end<SMODE>(lds, X, Z4, kLead + (uint32_t)(p - lo), n, ini,
                                                 [&](uint32_t q) { return stage32[q + (q >> 5)]; });
                else if (fits && END && n >= 4)
                    res = lane_record_end<SMODE>(lds, X, Z4, kLead + (uint32_t)(p - lo), n, ini, [&](uint32_t q) {
                        return *reinterpret_cast<const uint32_t*>(stage + 4u * q);
                    });
                else if (fits)
                    res = lane_record<R8 ? 32 : 8>(lds, X, Z4, T8, p, n, ini, [&](uintptr_t a) {
                        const uint32_t at = kLead + (uint32_t)(a - lo);
                        if (sk) {
                            const uint32_t d = at / 4 + at / 128;
                            return u32x4{stage32[d], stage32[d + 1], stage32[d + 2], stage32[d + 3]};
                        }
                        return *reinterpret_cast<const u32x4*>(stage + at);
                    });
                else
                    res = lane_record<R8 ? 32 : 8>(lds, X, Z4, T8, p, n, ini,
                                      [&](uintptr_t a) { return ld16(reinterpret_cast<const uint8_t*>(a)); });
            }
            if constexpr (SPEC) {
                spec_res = res;  // (checked below, with every lane of the wave)
            } else {
                A.out[ri] = res;
                if (A.cmp_stored && n && res != A.cmp_stored[ri]) atomicMin(A.cmp_bad, (unsigned long long)ri);
            }
        }
        if constexpr (SPEC) {
            // the slot's header: its CRC field and len/type word, from the stage (or global memory)
            // (read after the CRC steps: read before them, the kernel measured 4 us slower)
            unsigned long long kstop = ~0ull, kdev = ~0ull;
            if (ri < n_rec && n) {
                const uintptr_t p = reinterpret_cast<uintptr_t>(A.arena) + o;
                uint32_t hc, hs;
                if (fits) {
                    const uint32_t at = kLead + (uint32_t)(p - 8 - lo), q = at >> 2, sh = at & 3u;
                    uint32_t d0, d1, d2;
                    if (sk) {
                        d0 = stage32[q + (q >> 5)];
                        d1 = stage32[(q + 1) + ((q + 1) >> 5)];
                        d2 = stage32[(q + 2) + ((q + 2) >> 5)];
                    } else {
                        d0 = stage32[q];
                        d1 = stage32[q + 1];
                        d2 = stage32[q + 2];
                    }
                    hc = __builtin_amdgcn_alignbyte(d1, d0, sh);
                    hs = __builtin_amdgcn_alignbyte(d2, d1, sh);
                } else {
                    read_hdr(KB_BYTES(reinterpret_cast<const uint8_t*>(p - 8), 8), hc, hs);
                }
                spec_keys(G, hc, hs, spec_res, gq + lane, lf, KB_BYTES(reinterpret_cast<const uint8_t*>(p + n), lf ? 8u : 0u),
                          kstop, kdev);
            }
            if constexpr (TM != 0) {  // (timing forms: every batch; the keys kept alive through a sink)
                tm_sink ^= (uint32_t)kstop ^ (uint32_t)(kstop >> 32) ^ (uint32_t)kdev;
            } else if (spec_report(A, kstop, kdev, lane)) {
                return true;
            }
        }
        return false;
    };
    bool sk = fits && skewed(o, n, lo);
    if constexpr (SPEC && P2) {
        // Two batches in flight (the slots' meta is arithmetic): batch k's bytes in one register
        // set while batch k + 1's land in the other; batch k + 2 is issued into the set batch k
        // leaves once it is in the stage.  (The unrolled pair keeps the sets in registers.)
        u32x4 v2[kStgVecs];
        uintptr_t lo2 = 0, hi2 = 0;
        bool fits2 = false, sk2 = false;
        if (fits) issue_into(v, lo, hi);
        if (base + step < n_rec) {
            extent(o2, n2, lo2, hi2);
            fits2 = hi2 != 0 && hi2 - lo2 <= kFit;
            sk2 = fits2 && skewed(o2, n2, lo2);
            if (fits2) issue_into(v2, lo2, hi2);
        }
        // one batch out of `cur` (its set), batch + 2 steps issued into it; false: the wave is done
        auto step_one = [&](u32x4 (&cur)[kStgVecs]) -> bool {
            if (fits && (TM & 2) == 0) store_stage(cur, sk);
            const uint64_t nn = base + 2 * step;
            uint64_t o3 = 0, gq3 = 0;
            uint32_t n3 = 0, ini3 = 0;
            bool lf3 = false, fits3 = false, sk3 = false;
            uintptr_t lo3 = 0, hi3 = 0;
            if (nn < n_rec) {
                ld_meta(nn, o3, n3, ini3, gq3, lf3);
                extent(o3, n3, lo3, hi3);
                fits3 = hi3 != 0 && hi3 - lo3 <= kFit;
                sk3 = fits3 && skewed(o3, n3, lo3);
                if (fits3) issue_into(cur, lo3, hi3);
            }
            const bool done = proc(base, o, n, ini, lo, fits, sk, gq, lf);
            wave_lds_sync();
            if (done || base + step >= n_rec) return false;
            base += step;
            o = o2; n = n2; ini = ini2; gq = gq2; lf = lf2; lo = lo2; hi = hi2; fits = fits2; sk = sk2;
            o2 = o3; n2 = n3; ini2 = ini3; gq2 = gq3; lf2 = lf3; lo2 = lo3; hi2 = hi3; fits2 = fits3; sk2 = sk3;
            return true;
        };
        if (base < n_rec)
            while (step_one(v) && step_one(v2)) {
            }
    } else {
    if (fits) issue(lo, hi);
    for (bool run = !SPEC || base < n_rec; run;) {
        if (fits && (TM & 2) == 0) store_stage(v, sk);
        const uint64_t nb = base + step;
        const bool more = nb < n_rec;
        uintptr_t lo2 = 0, hi2 = 0;
        bool fits2 = false, sk2 = false;
        uint64_t o3 = 0, gq3 = 0;
        uint32_t n3 = 0, ini3 = 0;
        bool lf3 = false;
        if (more) {
            extent(o2, n2, lo2, hi2);
            fits2 = hi2 != 0 && hi2 - lo2 <= kFit;
            sk2 = fits2 && skewed(o2, n2, lo2);
            if (fits2) issue(lo2, hi2);
            ld_meta(nb + step, o3, n3, ini3, gq3, lf3);
        }
        if (proc(base, o, n, ini, lo, fits, sk, gq, lf)) break;
        wave_lds_sync();
        if (!more) break;
        base = nb;
        o = o2; n = n2; ini = ini2; gq = gq2; lf = lf2;
        o2 = o3; n2 = n3; ini2 = ini3; gq2 = gq3; lf2 = lf3;
        lo = lo2; hi = hi2; fits = fits2; sk = sk2;
    }
    }  // (one batch in flight)
    if constexpr (SPEC) {
        if (TM != 0 && tm_sink == 0x9e3779b9u) poor_seen = true;  // (never in practice: keeps the sink)
        spec_epilogue(A, sp_ok, G, poor_seen, stage32);
        return;
    }
    if (poor_seen && A.stage_skew_seen && lane == 0) *A.stage_skew_seen = 1u;  // (benign races: all store 1)
}


}  // namespace

hipError_t launch_ragged_direct(const RaggedArgs& a, int grid_blocks, hipStream_t s) {
    if (a.n_rec == 0) return hipSuccess;
    units_timer_begin(s);
    // (the tools build's KARMA_DIRECT_VARIANT=20: the LDS-staged kernel over the bounded ABI, so
    // the tests hold it to parity on batches of every shape; the caller passes the lane blob)
    if (KARMA_AB_KNOB("KARMA_DIRECT_VARIANT", 0) == 20)
        hipLaunchKernelGGL((k_ragged_staged_pipe<true>), dim3(grid_blocks), dim3(kStgWaves * 64), 0, s, a);
    else if (KARMA_AB_KNOB("KARMA_DIRECT_VARIANT", 0) == 21) {  // (the plain stage only)
#ifdef KARMA_AB
        // (KARMA_STAGE_TIMING: the timing forms, k_ragged_staged_pipe's TM)
        const long tm = KARMA_AB_KNOB("KARMA_STAGE_TIMING", 0);
        if (tm == 1)
            hipLaunchKernelGGL((k_ragged_staged_pipe<false, false, 1>), dim3(grid_blocks), dim3(kStgWaves * 64), 0, s, a);
        else if (tm == 2)
            hipLaunchKernelGGL((k_ragged_staged_pipe<false, false, 2>), dim3(grid_blocks), dim3(kStgWaves * 64), 0, s, a);
        else if (tm == 3)
            hipLaunchKernelGGL((k_ragged_staged_pipe<false, false, 3>), dim3(grid_blocks), dim3(kStgWaves * 64), 0, s, a);
        else
#endif
            hipLaunchKernelGGL((k_ragged_staged_pipe<false>), dim3(grid_blocks), dim3(kStgWaves * 64), 0, s, a);
    }
#ifdef KARMA_AB
    else if (KARMA_AB_KNOB("KARMA_DIRECT_VARIANT", 0) == 22)  // (the 8-copy image, kStgWaves8 waves)
        hipLaunchKernelGGL((k_ragged_staged_pipe<false, true>), dim3(grid_blocks), dim3(kStgWaves8 * 64), 0, s, a);
#endif
    else
        hipLaunchKernelGGL(k_ragged_direct4<>, dim3(grid_blocks), dim3(kBlockThreads), 0, s, a);
    units_timer_end(s);
    return hipGetLastError();
}

hipError_t launch_ragged_staged_dev(const RaggedArgs& a, int grid_blocks, hipStream_t s, bool skew) {
    if (a.n_rec == 0 || !a.n_dev || !a.gate_len) return hipErrorInvalidValue;
    // (round 5 measured two batches' loads in flight per wave, a depth-2 variant of this kernel,
    // slower: 0.1229 vs 0.1201 ms per 1M x 180 B replay call, profiles/r05_replay_depth2.txt)
    // (Round 5 measured two lanes per record -- a wave staging 32 records in 6 KiB, each lane
    // stepping half a record's windows, 12 waves per CU: 49.2 against 51.2 us on 1M x 180 B, and
    // no faster per replay call, 0.1179 vs 0.1183 ms: profiles/r05_staged_probe_pair.json,
    // r05_replay_pair.txt.  The staged kernel is bound by its staging round trips as much as by its
    // steps.)
    if (skew) {
        hipLaunchKernelGGL((k_ragged_staged_pipe<true>), dim3(grid_blocks), dim3(kStgWaves * 64), 0, s, a);
#ifdef KARMA_AB
    } else if (const long r8 = KARMA_AB_KNOB("KARMA_STAGE_R8", 0); r8 == 6 || r8 == 4) {
        // (A/B, round 6: the 8-copy image with 6 or 4 waves, 109 / 85 KiB of LDS: room beside it
        // for 12 / 18 of the sliced replay's 4 KiB walkers per CU)
        if (r8 == 6)
            hipLaunchKernelGGL((k_ragged_staged_pipe<false, true, 0, 6>), dim3(grid_blocks), dim3(6 * 64), 0, s, a);
        else
            hipLaunchKernelGGL((k_ragged_staged_pipe<false, true, 0, 4>), dim3(grid_blocks), dim3(4 * 64), 0, s, a);
    } else if (r8) {  // (A/B: the 8-copy image, kStgWaves8 waves; not
        // shipped: 1M x 180 B 0.1219 vs 0.1215 ms per replay call, 100-B payloads 0.0978 vs 0.1007)
        const uint64_t g = std::min<uint64_t>((uint64_t)grid_blocks, (a.n_rec + 64 * kStgWaves8 - 1) / (64 * kStgWaves8));
        hipLaunchKernelGGL((k_ragged_staged_pipe<false, true>), dim3((unsigned)g), dim3(kStgWaves8 * 64), 0, s, a);
    } else if (!KARMA_AB_KNOB("KARMA_STAGE_WIDE", 1)) {  // (A/B: the window loop before the phased one)
        hipLaunchKernelGGL((k_ragged_staged_pipe<false, false, 0, 0, false, false, false>), dim3(grid_blocks), dim3(kStgWaves * 64), 0, s, a);
#endif
    } else {
        hipLaunchKernelGGL((k_ragged_staged_pipe<false>), dim3(grid_blocks), dim3(kStgWaves * 64), 0, s, a);
    }
    return hipGetLastError();
}

hipError_t launch_ragged_staged_spec(const RaggedArgs& a, int grid_blocks, hipStream_t s, bool skew) {
    if (!a.spec || !a.spec_out || !a.spec_nseg || a.spec_seg < 9 || a.spec_seg >= (1ull << 31) || grid_blocks <= 0 ||
        a.n_dev || a.spec_first + 9 > a.spec_seg)
        return hipErrorInvalidValue;
#ifdef KARMA_AB
    if (KARMA_AB_KNOB("KARMA_SPEC_P2", 0)) {  // (A/B: two batches in flight per wave)
        if (const long tm = KARMA_AB_KNOB("KARMA_SPEC_TIMING", 0); tm == 1)
            hipLaunchKernelGGL((k_ragged_staged_pipe<false, false, 1, 0, true, true>), dim3(grid_blocks), dim3(kStgWaves * 64), 0, s, a);
        else if (tm == 2)
            hipLaunchKernelGGL((k_ragged_staged_pipe<false, false, 2, 0, true, true>), dim3(grid_blocks), dim3(kStgWaves * 64), 0, s, a);
        else
            hipLaunchKernelGGL((k_ragged_staged_pipe<false, false, 0, 0, true, true>), dim3(grid_blocks), dim3(kStgWaves * 64), 0, s, a);
        return hipGetLastError();
    }
    // (timing forms, wrong results: 1 = no CRC steps, 2 = no record loads or stage stores, 3 = neither)
    if (const long tm = KARMA_AB_KNOB("KARMA_SPEC_TIMING", 0); tm == 1) {
        hipLaunchKernelGGL((k_ragged_staged_pipe<false, false, 1, 0, true>), dim3(grid_blocks), dim3(kStgWaves * 64), 0, s, a);
        return hipGetLastError();
    } else if (tm == 2) {
        hipLaunchKernelGGL((k_ragged_staged_pipe<false, false, 2, 0, true>), dim3(grid_blocks), dim3(kStgWaves * 64), 0, s, a);
        return hipGetLastError();
    } else if (tm == 3) {
        hipLaunchKernelGGL((k_ragged_staged_pipe<false, false, 3, 0, true>), dim3(grid_blocks), dim3(kStgWaves * 64), 0, s, a);
        return hipGetLastError();
    }
    if (!KARMA_AB_KNOB("KARMA_SPEC_WIDE", 1)) {  // (A/B: round 6's window loop, before the phased one)
        if (skew)
            hipLaunchKernelGGL((k_ragged_staged_pipe<true, false, 0, 0, true, false, false>), dim3(grid_blocks), dim3(kStgWaves * 64), 0, s, a);
        else
            hipLaunchKernelGGL((k_ragged_staged_pipe<false, false, 0, 0, true, false, false>), dim3(grid_blocks), dim3(kStgWaves * 64), 0, s, a);
        return hipGetLastError();
    }
    if (!KARMA_AB_KNOB("KARMA_SPEC_AL", 1)) {  // (A/B: the phased loop without its dword-aligned fast path)
        if (skew)
            hipLaunchKernelGGL((k_ragged_staged_pipe<true, false, 0, 0, true, false, true, false>), dim3(grid_blocks), dim3(kStgWaves * 64), 0, s, a);
        else
            hipLaunchKernelGGL((k_ragged_staged_pipe<false, false, 0, 0, true, false, true, false>), dim3(grid_blocks), dim3(kStgWaves * 64), 0, s, a);
        return hipGetLastError();
    }
    if (KARMA_AB_KNOB("KARMA_SPEC_R8", 0)) {  // (A/B: the 8-copy image, kStgWaves8 waves, plain stage)
        hipLaunchKernelGGL((k_ragged_staged_pipe<false, true, 0, 0, true>), dim3(grid_blocks), dim3(kStgWaves8 * 64), 0, s, a);
        return hipGetLastError();
    }
#endif
    if (skew)
        hipLaunchKernelGGL((k_ragged_staged_pipe<true, false, 0, 0, true>), dim3(grid_blocks), dim3(kStgWaves * 64), 0, s, a);
    else
        hipLaunchKernelGGL((k_ragged_staged_pipe<false, false, 0, 0, true>), dim3(grid_blocks), dim3(kStgWaves * 64), 0, s, a);
    return hipGetLastError();
}

hipError_t launch_ragged_direct_spec(const RaggedArgs& a, int grid_blocks, hipStream_t s) {
    if (!a.spec || !a.spec_out || !a.spec_nseg || a.spec_seg < 9 || a.spec_seg >= (1ull << 31) || grid_blocks <= 0 ||
        a.n_dev || a.spec_first + 9 > a.spec_seg)
        return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_ragged_direct4<true>, dim3(grid_blocks), dim3(kBlockThreads), 0, s, a);
    return hipGetLastError();
}

hipError_t launch_ragged_direct_dev(const RaggedArgs& a, int grid_blocks, hipStream_t s) {
    if (a.n_rec == 0 || !a.n_dev || !a.gate_len) return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_ragged_direct4<>, dim3(grid_blocks), dim3(kBlockThreads), 0, s, a);
    return hipGetLastError();
}

hipError_t launch_ragged_scan(const RaggedArgs& a, hipStream_t s) {
    if (a.n_rec == 0) return hipSuccess;
    if (a.unit_bytes != kU) return hipErrorInvalidValue;
    const uint64_t nb = ragged_scan_blocks(a.n_rec);
    hipLaunchKernelGGL(k_ragged_scan, dim3((unsigned)nb), dim3(kScanBlock), 0, s, a);
    return hipGetLastError();
}

#ifndef KARMA_PLAN_RMAX
#define KARMA_PLAN_RMAX 4  // most records per plan thread (a build-time A/B knob: 1 = round 4's one-record blocks)
#endif
hipError_t launch_ragged_main(const RaggedArgs& a, int grid_blocks, hipStream_t s) {
    if (a.n_rec == 0) return hipSuccess;
    if (!a.lb || !a.lb_ctl || a.lb_seq_max < 2 || a.lb_seq_max > (1u << 22)) return hipErrorInvalidValue;
    // records per plan thread / finalize lane: the fewest (1, 2, 4) that fit each grid on the GPU
    // at once, one workgroup per CU (grid_blocks = the CU count); larger batches take rounds of 4
    const uint64_t cu = grid_blocks > 0 ? (uint64_t)grid_blocks : 1;
    const uint64_t nb1 = ragged_scan_blocks(a.n_rec);
    int R = KARMA_PLAN_RMAX == 1 || nb1 <= cu ? 1 : KARMA_PLAN_RMAX == 2 || nb1 <= 2 * cu ? 2 : 4;
    if (const long rf = KARMA_AB_KNOB("KARMA_PLAN_R", 0); rf == 1 || rf == 2 || rf == 4) R = (int)rf;  // (A/B)
    const unsigned pb = (unsigned)((nb1 + R - 1) / R);
    if (R == 1)
        hipLaunchKernelGGL(k_ragged_plan<1>, dim3(pb), dim3(kScanBlock), 0, s, a);
    else if (R == 2)
        hipLaunchKernelGGL(k_ragged_plan<2>, dim3(pb), dim3(kScanBlock), 0, s, a);
    else
        hipLaunchKernelGGL(k_ragged_plan<4>, dim3(pb), dim3(kScanBlock), 0, s, a);
#ifdef KARMA_AB
    // (timing: the timed units kernel follows an untimed one instead of the plan; only with
    // KARMA_RAGGED_DYN=0 -- the first kernel takes the dynamic tail's counter to its end)
    if (KARMA_AB_KNOB("KARMA_RAGGED_UNITS_TWICE", 0) && !a.dyn_shift)
        hipLaunchKernelGGL(k_units_ragged<>, dim3(grid_blocks), dim3(kBlockThreads), 0, s, a);
#endif
    units_timer_begin(s);
#ifdef KARMA_AB
    // timing forms (wrong results): 1 = steps without the LDS lookups, 2 = no lane fold / tree, 3 = both
    if (const int fx = KARMA_AB_KNOB("KARMA_RAGGED_UNITS_FIXEDLOOP", 0); fx == 1)
        hipLaunchKernelGGL(k_units_ragged_fixedloop<false>, dim3(grid_blocks), dim3(kBlockThreads), 0, s, a);
    else if (fx == 2)
        hipLaunchKernelGGL(k_units_ragged_fixedloop<true>, dim3(grid_blocks), dim3(kBlockThreads), 0, s, a);
    else if (fx == 3)
        hipLaunchKernelGGL((k_units_ragged_fixedloop<true, true>), dim3(grid_blocks), dim3(kBlockThreads), 0, s, a);
    else if (fx == 4)
        hipLaunchKernelGGL((k_units_ragged_fixedloop<true, false, true>), dim3(grid_blocks), dim3(kBlockThreads), 0, s, a);
    else if (fx == 5)
        hipLaunchKernelGGL((k_units_ragged_fixedloop<false, true>), dim3(grid_blocks), dim3(kBlockThreads), 0, s, a);
    else if (const int st = KARMA_AB_KNOB("KARMA_RAGGED_UNITS_STREAM", 0); st == 40)  // PF, dynamic tail
        hipLaunchKernelGGL((k_units_ragged_stream<4, false>), dim3(grid_blocks), dim3(kBlockThreads), 0, s, a);
    else if (st == 41)
        hipLaunchKernelGGL((k_units_ragged_stream<4, true>), dim3(grid_blocks), dim3(kBlockThreads), 0, s, a);
    else if (st == 60)
        hipLaunchKernelGGL((k_units_ragged_stream<6, false>), dim3(grid_blocks), dim3(kBlockThreads), 0, s, a);
    else if (st == 61)
        hipLaunchKernelGGL((k_units_ragged_stream<6, true>), dim3(grid_blocks), dim3(kBlockThreads), 0, s, a);
    else if (const int fl = KARMA_AB_KNOB("KARMA_RAGGED_UNITS_FLAT", 0); fl == 8)
        hipLaunchKernelGGL((k_units_ragged_flat<8>), dim3(grid_blocks), dim3(kBlockThreads), 0, s, a);
    else if (fl == 4)
        hipLaunchKernelGGL((k_units_ragged_flat<4>), dim3(grid_blocks), dim3(kBlockThreads), 0, s, a);
    else if (fl == 83)
        hipLaunchKernelGGL((k_units_ragged_flat<8, 3>), dim3(grid_blocks), dim3(kBlockThreads), 0, s, a);
    else if (fl == 864)  // arithmetic unit addresses (aligned unit-sized records only), no descriptor loads
        hipLaunchKernelGGL((k_units_ragged_flat<8, 64>), dim3(grid_blocks), dim3(kBlockThreads), 0, s, a);
    else if (fl == 8128)  // no unit-state stores
        hipLaunchKernelGGL((k_units_ragged_flat<8, 128>), dim3(grid_blocks), dim3(kBlockThreads), 0, s, a);
    else if (fl == 8192)  // both
        hipLaunchKernelGGL((k_units_ragged_flat<8, 192>), dim3(grid_blocks), dim3(kBlockThreads), 0, s, a);
    else if (const int um = KARMA_AB_KNOB("KARMA_RAGGED_UNITS_MODE", 0); um == 1)
        hipLaunchKernelGGL((k_units_ragged<kRaggedUnitsPF, 1>), dim3(grid_blocks), dim3(kBlockThreads), 0, s, a);
    else if (um == 2)
        hipLaunchKernelGGL((k_units_ragged<kRaggedUnitsPF, 2>), dim3(grid_blocks), dim3(kBlockThreads), 0, s, a);
    else if (um == 3)
        hipLaunchKernelGGL((k_units_ragged<kRaggedUnitsPF, 3>), dim3(grid_blocks), dim3(kBlockThreads), 0, s, a);
    else if (um == 64)  // (A/B: the phased window step, step4 MODE 64)
        hipLaunchKernelGGL((k_units_ragged<kRaggedUnitsPF, 64>), dim3(grid_blocks), dim3(kBlockThreads), 0, s, a);
    else
#endif
        hipLaunchKernelGGL(k_units_ragged<>, dim3(grid_blocks), dim3(kBlockThreads), 0, s, a);
    units_timer_end(s);
    const uint64_t fb1 = (a.n_rec + 1023) / 1024;  // 16 waves x 64 records per block
    int FR = fb1 <= cu ? 1 : fb1 <= 2 * cu ? 2 : 4;
    if (const long ff = KARMA_AB_KNOB("KARMA_FINALIZE_FR", 0); ff == 1 || ff == 2 || ff == 4) FR = (int)ff;  // (A/B)
    const unsigned fblocks = (unsigned)std::min<uint64_t>((fb1 + FR - 1) / FR, cu);
#ifdef KARMA_AB
    if (KARMA_AB_KNOB("KARMA_FINALIZE_LITE", 0)) {  // (A/B: the LDS fill without the huge records' maps)
        if (FR == 1)
            hipLaunchKernelGGL((k_ragged_finalize<1, true>), dim3(fblocks), dim3(1024), 0, s, a);
        else if (FR == 2)
            hipLaunchKernelGGL((k_ragged_finalize<2, true>), dim3(fblocks), dim3(1024), 0, s, a);
        else
            hipLaunchKernelGGL((k_ragged_finalize<4, true>), dim3(fblocks), dim3(1024), 0, s, a);
        return hipGetLastError();
    }
#endif
    if (FR == 1)
        hipLaunchKernelGGL(k_ragged_finalize<1>, dim3(fblocks), dim3(1024), 0, s, a);
    else if (FR == 2)
        hipLaunchKernelGGL(k_ragged_finalize<2>, dim3(fblocks), dim3(1024), 0, s, a);
    else
        hipLaunchKernelGGL(k_ragged_finalize<4>, dim3(fblocks), dim3(1024), 0, s, a);
    return hipGetLastError();
}

KB_DEFINE_COLLECT(ragged)
#ifdef KARMA_AB
WLOG_SETTER(ragged)
hipError_t set_plan_log(void* p) {
    uint64_t* q = static_cast<uint64_t*>(p);
    return hipMemcpyToSymbol(HIP_SYMBOL(g_plan_log), &q, sizeof(q));
}
#endif

}  // namespace engine
}  // namespace karma
