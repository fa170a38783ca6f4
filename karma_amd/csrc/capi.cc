// karma_amd/csrc/capi.cc -- the C ABI (include/karma_crc32c.h): argument
// checks, unit planning, per-device table blobs, per-stream workspaces and
// the RCCL communicator.  Every device entry point is stream-ordered and
// returns a KARMA_E_* status; nothing throws across the ABI and nothing falls
// back to the CPU.
#include <hip/hip_runtime_api.h>

#include <algorithm>
#include <atomic>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <new>
#include <string>
#include <utility>
#include <vector>

#include "ab.h"
#include "bounds.h"
#include "engine.h"
#include "karma_crc32c.h"
#include "stream_state.h"

using namespace karma::engine;

namespace {

thread_local std::string g_last;

int fail(int code, const std::string& what) {
    g_last = what;
    return code;
}

int hip_fail(hipError_t e, const char* what) {
    g_last = std::string(what) + ": " + hipGetErrorString(e);
    return e == hipErrorOutOfMemory ? KARMA_E_NOMEM : KARMA_E_HIP;
}

#define KARMA_HIP(expr)                                 \
    do {                                                \
        hipError_t _e = (expr);                         \
        if (_e != hipSuccess) return hip_fail(_e, #expr); \
    } while (0)

#define KARMA_RC(expr)          \
    do {                        \
        int _rc = (expr);       \
        if (_rc) return _rc;    \
    } while (0)

constexpr uint64_t kMinSplitUnit = 2048;  // smallest unit when records are split
constexpr uint32_t kDirectMaxLen = 1024;  // ragged records up to this: one record per group
constexpr uint64_t kOverdecompose = 4;    // units per group before splitting records
constexpr uint64_t kSegOnceUnits = 128;      // units per workgroup of k_segment_once (8 x 16 waves)
constexpr uint64_t kSegOnceMin = 256 << 10;  // single records from this size take it
constexpr long kSegOnceDefault = 1;          // 1: the grid's last workgroup folds; 2: the last-arriving one
constexpr uint64_t kSplitOverdecompose = 64;  // units per group once split (2 KiB units up to 4 GiB
                                              // batches; 4: config 4 0.653 ms, 64: 0.609)

uint64_t ceil_div(uint64_t a, uint64_t b) { return (a + b - 1) / b; }
uint64_t round_up(uint64_t a, uint64_t m) { return ceil_div(a, m) * m; }
size_t align256(size_t x) { return (x + 255) & ~size_t(255); }

struct DevState {
    bool ready = false;
    int cu = 0;
    uint32_t* blob = nullptr;       // the streaming kernels' tables (stride 128)
    uint32_t* lane_blob = nullptr;  // the LDS-staged kernel's tables (stride 16: one record per lane)
    uint32_t* quad_blob = nullptr;  // k_ragged_direct4's tables (stride 64)
    std::map<uint64_t, uint32_t*> comb;  // unit bytes -> combine blob
    std::map<std::pair<uint64_t, uint64_t>, uint32_t*> bcomb;  // (unit bytes, states per thread) -> block blob
};

// HIP operations of the per-stream state (stream_state.h).
struct HipStateOps {
    int alloc(void** p, size_t bytes) {
        const hipError_t e = hipMalloc(p, bytes);
        return e == hipSuccess ? 0 : hip_fail(e, "hipMalloc (stream state)");
    }
    void free(void* p) { (void)hipFree(p); }
    int zero(void* p, size_t bytes, void* s) {
        const hipError_t e = hipMemsetAsync(p, 0, bytes, (hipStream_t)s);
        return e == hipSuccess ? 0 : hip_fail(e, "hipMemsetAsync (stream state)");
    }
    int sync_stream(void* s) {
        const hipError_t e = hipStreamSynchronize((hipStream_t)s);
        return e == hipSuccess ? 0 : hip_fail(e, "hipStreamSynchronize (stream state)");
    }
    int sync_device(int dev) {
        int cur = 0;
        (void)hipGetDevice(&cur);
        hipError_t e = hipSetDevice(dev);
        if (e == hipSuccess) e = hipDeviceSynchronize();
        (void)hipSetDevice(cur);
        return e == hipSuccess ? 0 : hip_fail(e, "hipDeviceSynchronize (trim)");
    }
    bool capturing(void* s) {
        hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
        if (hipStreamIsCapturing((hipStream_t)s, &st) != hipSuccess) {
            (void)hipGetLastError();
            return false;
        }
        return st != hipStreamCaptureStatusNone;
    }
};

// One lock for the library state; held across planning and enqueueing so a
// workspace is never reallocated between another call's lookup and launch.
std::mutex g_mu;
std::vector<DevState> g_dev;
// Per (device, stream): the workspace, the ragged plan's look-back words and the fused record
// combine's words (stream_state.h: what is freed when, and what a captured graph keeps).
//   look-back words (RaggedArgs::lb, crc_ragged.hip): [0] counts started plan blocks, [1 + b]
//     block b's full-unit status and [1 + half + b] its partial-unit status, tagged with the
//     call's seq; then the control words lb_ctl.  Calls on one stream run in order, so a call
//     sees only its own tag or older ones.  The counter and the tag live on the device
//     (k_ragged_plan / k_ragged_finalize), so a captured ragged call replays any number of
//     times.  Zeroed when allocated; the device clears them when the 22-bit tag wraps.
//   fused words (FixedArgs::fctl, k_units_fixed FUSE, k_segment_once): [0] arrival tickets (zero
//     between calls), [1] the last finished call's
//     tag, then kBlockCombMaxPerThread * 1024 tagged wave states.  Zeroed once and never moved:
//     the tags only grow, so no state a later call reads carries its tag before that call wrote it.
StreamStates<HipStateOps> g_states;
using State = StreamStates<HipStateOps>::State;

// hipStreamPerThread is one handle for many streams: its state is keyed per calling thread, by a
// generation number (odd, so never a stream handle), not by an address a later thread may reuse.
// A thread's exit hands its per-thread state to the next trim (its stream is gone).
std::atomic<uint64_t> g_thread_gen{0};
struct ThreadKey {
    uintptr_t key = 0;
    ~ThreadKey() {
        if (!key) return;
        std::lock_guard<std::mutex> lk(g_mu);
        g_states.orphan(key);
    }
};
thread_local ThreadKey t_key;
uintptr_t stream_key(hipStream_t s) {
    if (s != hipStreamPerThread) return reinterpret_cast<uintptr_t>(s);
    if (!t_key.key) t_key.key = (uintptr_t)((++g_thread_gen << 1) | 1u);
    return t_key.key;
}

int current_device(int* dev) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return fail(KARMA_E_NO_DEVICE, "no HIP device visible");
    KARMA_HIP(hipGetDevice(dev));
    return 0;
}

// Caller holds g_mu.
int dev_state(int dev, DevState** out) {
    if ((int)g_dev.size() <= dev) g_dev.resize(dev + 1);
    DevState& d = g_dev[dev];
    if (!d.ready) {
        hipDeviceProp_t prop;
        KARMA_HIP(hipGetDeviceProperties(&prop, dev));
        d.cu = prop.multiProcessorCount > 0 ? prop.multiProcessorCount : 1;
        std::vector<uint32_t> host(kBlobWords);
        build_stream_blob(host.data());
        KARMA_HIP(hipMalloc(&d.blob, kBlobWords * sizeof(uint32_t)));
        KARMA_HIP(hipMemcpy(d.blob, host.data(), kBlobWords * sizeof(uint32_t), hipMemcpyHostToDevice));
        build_quad_blob(host.data());
        KARMA_HIP(hipMalloc(&d.quad_blob, kBlobWords * sizeof(uint32_t)));
        KARMA_HIP(hipMemcpy(d.quad_blob, host.data(), kBlobWords * sizeof(uint32_t), hipMemcpyHostToDevice));
        build_lane_blob(host.data());
        KARMA_HIP(hipMalloc(&d.lane_blob, kBlobWords * sizeof(uint32_t)));
        KARMA_HIP(hipMemcpy(d.lane_blob, host.data(), kBlobWords * sizeof(uint32_t), hipMemcpyHostToDevice));
        d.ready = true;
    }
    *out = &d;
    return 0;
}

int comb_blob(DevState& d, uint64_t unit_bytes, const uint32_t** out) {
    auto it = d.comb.find(unit_bytes);
    if (it == d.comb.end()) {
        std::vector<uint32_t> host(kCombWords);
        build_combine_blob(unit_bytes, host.data());
        uint32_t* p = nullptr;
        KARMA_HIP(hipMalloc(&p, kCombWords * sizeof(uint32_t)));
        KARMA_HIP(hipMemcpy(p, host.data(), kCombWords * sizeof(uint32_t), hipMemcpyHostToDevice));
        it = d.comb.emplace(unit_bytes, p).first;
    }
    *out = it->second;
    return 0;
}

int block_comb_blob(DevState& d, uint64_t unit_bytes, uint64_t per_thread, const uint32_t** out) {
    const auto key = std::make_pair(unit_bytes, per_thread);
    auto it = d.bcomb.find(key);
    if (it == d.bcomb.end()) {
        std::vector<uint32_t> host(kBlockCombWords);
        build_block_combine_blob(unit_bytes, per_thread, host.data());
        uint32_t* p = nullptr;
        KARMA_HIP(hipMalloc(&p, kBlockCombWords * sizeof(uint32_t)));
        KARMA_HIP(hipMemcpy(p, host.data(), kBlockCombWords * sizeof(uint32_t), hipMemcpyHostToDevice));
        it = d.bcomb.emplace(key, p).first;
    }
    *out = it->second;
    return 0;
}

// Caller holds g_mu.  The stream's scratch buffer, grown on demand (by a quarter more than asked).
int workspace(int dev, hipStream_t s, size_t bytes, void** out) {
    State& st = g_states.get(dev, stream_key(s), s);
    KARMA_RC(g_states.grow(st, st.ws, bytes, align256(bytes + bytes / 4), false));
    *out = st.ws.p;
    return 0;
}

// Caller holds g_mu.
int fused_words(int dev, hipStream_t s, unsigned long long** out) {
    State& st = g_states.get(dev, stream_key(s), s);
    const size_t bytes = (2 + kBlockCombMaxPerThread * 1024) * sizeof(unsigned long long);
    KARMA_RC(g_states.grow(st, st.fused, bytes, bytes, true));
    *out = static_cast<unsigned long long*>(st.fused.p);
    return 0;
}

// Caller holds g_mu.  Binds the stream's look-back words for nb plan blocks.
int bind_lookback(int dev, hipStream_t s, uint64_t nb, RaggedArgs& a) {
    State& st = g_states.get(dev, stream_key(s), s);
    const uint64_t want_half = std::max<uint64_t>(2 * nb, 2048);
    const uint64_t have_half = st.lb.p ? (st.lb.bytes / sizeof(unsigned long long) - 4) / 2 : 0;
    if (have_half < nb) {
        const size_t bytes = (1 + 2 * want_half + 3) * sizeof(unsigned long long);
        KARMA_RC(g_states.grow(st, st.lb, bytes, bytes, true));
    }
    unsigned long long* w = static_cast<unsigned long long*>(st.lb.p);
    const uint64_t half = (st.lb.bytes / sizeof(unsigned long long) - 4) / 2;
    a.lb = w;
    a.lbp = w + 1 + half;
    a.lb_ctl = w + 1 + 2 * half;
    a.lb_words = 2 * half;
    // (the tools build can lower the wrap point to test it: KARMA_LB_SEQ_MAX, ab.h)
    a.lb_seq_max = (uint32_t)std::min<long>(KARMA_AB_KNOB("KARMA_LB_SEQ_MAX", 1l << 22), 1l << 22);
    a.dyn_shift = (uint32_t)std::min<long>(std::max<long>(KARMA_AB_KNOB("KARMA_RAGGED_DYN", KARMA_RAGGED_DYN_SHIFT), 0), 16);
    return 0;
}

// ---- fixed-size records ---------------------------------------------------
// Units per group when records are split (the tools build's KARMA_SPLIT_OVERDECOMPOSE, ab.h).
uint64_t split_overdecompose() {
    const long v = KARMA_AB_KNOB("KARMA_SPLIT_OVERDECOMPOSE", (long)kSplitOverdecompose);
    return v < 1 ? 1 : v > 256 ? 256 : (uint64_t)v;
}

// Largest in-wave split of a big batch's records (2; the tools build's KARMA_FOLD_MAX_K
// also tries 4, 8 and 1 = off, ab.h).
uint64_t fold_max_k() {
    const long v = KARMA_AB_KNOB("KARMA_FOLD_MAX_K", 2);
    return v >= 8 ? 8 : v >= 4 ? 4 : v >= 2 ? 2 : 1;
}

int fixed_locked(int dev, DevState& ds, const void* d_data, size_t rec_bytes, size_t n_rec, const uint32_t* d_init,
                 uint32_t init, uint32_t* d_out, hipStream_t s) {
    const uint64_t groups = (uint64_t)ds.cu * kWavesPerBlock * kGroupsPerWave;
    const uint64_t target = kOverdecompose * groups;
    uint64_t unit, k;
    uint32_t fold_k = 0;
    if (rec_bytes <= (size_t)kChunk || n_rec >= target) {
        unit = round_up(std::max<uint64_t>(rec_bytes, 1), kChunk);
        k = 1;
        // Batches that fill the GPU: records of >= 2 split units are cut into 2, 4 or 8 units
        // whose groups sit in one wave (folded there, no combine launch).  Finer wave-steps
        // balance the CU's waves better: 1M x 4 KiB as 2M x 2 KiB units, DESIGN.md §4.
        const uint64_t max_k = fold_max_k();
        for (uint64_t kw = max_k; kw >= 2 && n_rec >= target; kw /= 2) {
            const uint64_t u = round_up(ceil_div(rec_bytes, kw), kChunk);
            if (u >= kMinSplitUnit) {
                unit = u;
                k = kw;
                fold_k = (uint32_t)kw;
                break;
            }
        }
    } else {
        const uint64_t k_ideal = ceil_div(split_overdecompose() * groups, n_rec);
        unit = std::max<uint64_t>(kMinSplitUnit, round_up(ceil_div(rec_bytes, k_ideal), kChunk));
        k = ceil_div(rec_bytes, unit);
        if (k == 1) {
            unit = round_up(rec_bytes, kChunk);
        } else if (k <= kGroupsPerWave && fold_max_k() > 1) {
            // 2-8 units: a power of two, folded inside the wave like the big batches' split
            uint64_t kw = 2;
            while (kw < k) kw *= 2;
            unit = std::max<uint64_t>(kMinSplitUnit, round_up(ceil_div(rec_bytes, kw), kChunk));
            k = kw;
            fold_k = (uint32_t)kw;
        } else {
            // a whole number of waves per record (the leading units are then empty: the
            // units are end-aligned), so each wave folds its 8 units (k_units_fixed WAVE_COMB)
            k = round_up(k, kGroupsPerWave);
        }
    }
    FixedArgs a;
    a.arena = static_cast<const uint8_t*>(d_data);
    a.rec_bytes = rec_bytes;
    a.n_rec = n_rec;
    a.init = d_init;
    a.init_scalar = init;
    a.unit_bytes = unit;
    a.units_per_rec = k;
    a.out = d_out;
    a.partial = nullptr;
    a.blob = ds.blob;
    a.comb_maps = nullptr;
    a.fold_k = fold_k;
    a.fctl = nullptr;
    a.block_blob = nullptr;
    a.comb_m = 0;
    if (fold_k) {
        KARMA_RC(comb_blob(ds, unit, &a.comb_maps));
        // (the tools build's KARMA_FIXED_GRID_MULT: that many workgroups per CU, dispatched in
        // rounds, so the hardware hands the later ones to the CUs that finish first)
        const long gm = KARMA_AB_KNOB("KARMA_FIXED_GRID_MULT", 1);
        KARMA_HIP(launch_fixed(a, ds.cu * (int)(gm < 1 ? 1 : gm > 16 ? 16 : gm), s));
        return 0;
    }
    if (k == 1) {
        KARMA_HIP(launch_fixed(a, ds.cu, s));
        return 0;
    }
    KARMA_RC(comb_blob(ds, unit, &a.comb_maps));  // Z_U, Z_2U, Z_4U lead the unit's combine blob
    // (the tools build's KARMA_SEGMENT_ONCE: 0 = the looping fused kernel, 2 = the last-arriving
    // workgroup folds)
    const long seg_once = KARMA_AB_KNOB("KARMA_SEGMENT_ONCE", kSegOnceDefault);
    if (n_rec == 1 && rec_bytes >= kSegOnceMin &&
        rec_bytes <= (uint64_t)ds.cu * kSegOnceUnits * segment_once_max_unit(a.arena, rec_bytes) && seg_once) {
        // one segment (up to 64 MiB on 256 CUs): every wave streams one wave-step of 8 units with all
        // of its loads in flight at once, workgroups fold their waves (k_segment_once)
        const uint64_t G = std::min<uint64_t>(ds.cu, std::max<uint64_t>(1, ceil_div(rec_bytes, kSegOnceUnits * 512)));
        a.unit_bytes = round_up(ceil_div(rec_bytes, kSegOnceUnits * G), kChunk);
        a.units_per_rec = kSegOnceUnits * G;
        a.fold_k = 0;
        KARMA_RC(comb_blob(ds, a.unit_bytes, &a.comb_maps));
        KARMA_RC(comb_blob(ds, a.unit_bytes * kSegOnceUnits, &a.block_blob));
        unsigned long long* w = nullptr;
        KARMA_RC(fused_words(dev, s, &w));
        a.fctl = w;
        a.partial = reinterpret_cast<uint32_t*>(w + 2);
        KARMA_HIP(launch_segment_once(a, (int)G, s, seg_once == 2));
        return 0;
    }
    if (n_rec == 1 && k / kGroupsPerWave <= kBlockCombMaxPerThread * 1024) {
        // one record (a segment scan): the units kernel's last workgroup folds the wave states
        // itself (k_units_fixed FUSE), one launch instead of two
        const uint64_t k_in = k / kGroupsPerWave;
        a.comb_m = ceil_div(k_in, 1024);
        KARMA_RC(block_comb_blob(ds, unit * kGroupsPerWave, a.comb_m, &a.block_blob));
        unsigned long long* w = nullptr;
        KARMA_RC(fused_words(dev, s, &w));
        a.fctl = w;
        a.partial = reinterpret_cast<uint32_t*>(w + 2);
        KARMA_HIP(launch_fixed(a, ds.cu, s));
        return 0;
    }
    const size_t part_bytes = align256(n_rec * k * sizeof(uint32_t));
    const size_t lvl_bytes = align256(n_rec * ceil_div(k, 64) * sizeof(uint32_t));
    void* ws = nullptr;
    KARMA_RC(workspace(dev, s, part_bytes + 2 * lvl_bytes, &ws));
    a.partial = static_cast<uint32_t*>(ws);
    uint32_t* bufs[2] = {reinterpret_cast<uint32_t*>(static_cast<char*>(ws) + part_bytes),
                         reinterpret_cast<uint32_t*>(static_cast<char*>(ws) + part_bytes + lvl_bytes)};
    KARMA_HIP(launch_fixed(a, ds.cu, s));
    const uint32_t* in = a.partial;  // one state per wave of 8 units
    uint64_t k_in = k / kGroupsPerWave, d = unit * kGroupsPerWave;
    // few records: every state of a record in one launch, one block per record
    if (n_rec <= 4 * (uint64_t)ds.cu && k_in <= kBlockCombMaxPerThread * 1024) {
        const uint64_t m = ceil_div(k_in, 1024);
        const uint32_t* bb = nullptr;
        KARMA_RC(block_comb_blob(ds, d, m, &bb));
        KARMA_HIP(launch_combine_block(a, in, k_in, m, bb, s));
        return 0;
    }
    for (int which = 0;; which ^= 1) {
        const uint64_t k_out = ceil_div(k_in, 64);
        const uint32_t* cb = nullptr;
        KARMA_RC(comb_blob(ds, d, &cb));
        uint32_t* outs = k_out == 1 ? nullptr : bufs[which];
        KARMA_HIP(launch_combine_fixed(a, in, k_in, outs, k_out, cb, s));
        if (k_out == 1) break;
        in = outs;
        k_in = k_out;
        d *= 64;
    }
    return 0;
}

// ---- ragged records -------------------------------------------------------
struct RaggedLayout {
    size_t fbase_off, pslot_off, sums_off, psums_off, desc_off, part_off, total;
};

RaggedLayout ragged_layout(uint64_t n_rec, uint64_t cap) {
    RaggedLayout L;
    const uint64_t nb = ragged_scan_blocks(n_rec);
    L.fbase_off = 0;
    L.pslot_off = L.fbase_off + align256((n_rec + 2) * sizeof(uint64_t));
    L.sums_off = L.pslot_off + align256(2 * n_rec * sizeof(uint64_t));
    L.psums_off = L.sums_off + align256(nb * sizeof(uint64_t));
    L.desc_off = L.psums_off + align256(nb * sizeof(uint64_t));
    L.part_off = L.desc_off + align256(cap * sizeof(UnitDesc));
    L.total = L.part_off + align256(cap * sizeof(uint32_t));
    return L;
}

void bind_ragged(RaggedArgs& a, void* ws, const RaggedLayout& L, uint64_t cap) {
    char* b = static_cast<char*>(ws);
    a.fbase = reinterpret_cast<uint64_t*>(b + L.fbase_off);
    a.pslot = reinterpret_cast<uint64_t*>(b + L.pslot_off);
    a.block_sums = reinterpret_cast<uint64_t*>(b + L.sums_off);
    a.block_psums = reinterpret_cast<uint64_t*>(b + L.psums_off);
    a.desc = reinterpret_cast<UnitDesc*>(b + L.desc_off);
    a.partial = reinterpret_cast<uint32_t*>(b + L.part_off);
    a.unit_cap = cap;
}

// The bounds build (bounds.h) checks record-byte loads against the arena's allocation.
void bind_arena_bounds(RaggedArgs& a) {
#ifdef KARMA_BOUNDS
    hipDeviceptr_t base = nullptr;
    size_t size = 0;
    if (a.arena && hipMemGetAddressRange(&base, &size, (hipDeviceptr_t)a.arena) == hipSuccess) {
        a.kb_lo = reinterpret_cast<uintptr_t>(base);
        a.kb_hi = a.kb_lo + size;
    } else {
        (void)hipGetLastError();
        a.kb_lo = 0;
        a.kb_hi = ~uintptr_t(0);
    }
#else
    (void)a;
#endif
}

int ragged_locked(int dev, DevState& ds, const void* d_arena, const uint64_t* d_off, const uint32_t* d_len,
                  size_t n_rec, size_t total_len, const uint32_t* d_init, uint32_t init, uint32_t* d_out,
                  hipStream_t s) {
    RaggedArgs a{};
    a.arena = static_cast<const uint8_t*>(d_arena);
    a.off = d_off;
    a.len = d_len;
    a.n_rec = n_rec;
    a.init = d_init;
    a.init_scalar = init;
    a.unit_bytes = kDefaultUnit;
    a.out = d_out;
    a.blob = ds.blob;
    bind_arena_bounds(a);
    KARMA_RC(comb_blob(ds, kDefaultUnit, &a.comb_blob));
    // Unit table: full units in [0, cap_full), partial units (at most 2 per record) after them.
    uint64_t cap_full, cap;
    void* ws = nullptr;
    if (total_len > 0) {
        // A record's units cover its whole 16-byte blocks [floor16(p), ceil16(p + n)): at most
        // n + 30 bytes, so its full (aligned, whole) units number at most (n + 30) / U, and the
        // batch's at most (total_len + 30 n_rec) / U.  (A record of U - 8 bytes at offset 8 mod U,
        // the WAL framing at stride U, fills a whole unit: ceil(total_len / U) alone undercounts.)
        cap_full = std::max<uint64_t>(1, ceil_div(total_len + 30 * (uint64_t)n_rec, kDefaultUnit));
        cap = cap_full + 2 * n_rec;
        const RaggedLayout L = ragged_layout(n_rec, cap);
        KARMA_RC(workspace(dev, s, L.total, &ws));
        bind_ragged(a, ws, L, cap);
    } else {
        // Unknown total: count the units (k_ragged_scan), read the block totals back and size
        // the unit table.
        cap = n_rec;
        RaggedLayout L = ragged_layout(n_rec, cap);
        KARMA_RC(workspace(dev, s, L.total, &ws));
        bind_ragged(a, ws, L, cap);
        KARMA_HIP(launch_ragged_scan(a, s));
        const uint64_t nb = ragged_scan_blocks(n_rec);
        std::vector<uint64_t> sums(2 * nb);
        KARMA_HIP(hipMemcpyAsync(sums.data(), a.block_sums, nb * sizeof(uint64_t), hipMemcpyDeviceToHost, s));
        KARMA_HIP(hipMemcpyAsync(sums.data() + nb, a.block_psums, nb * sizeof(uint64_t), hipMemcpyDeviceToHost, s));
        KARMA_HIP(hipStreamSynchronize(s));
        uint64_t full = 0, parts = 0;
        for (uint64_t i = 0; i < nb; ++i) {
            full += sums[i];
            parts += sums[nb + i];
        }
        cap_full = std::max<uint64_t>(full, 1);
        cap = cap_full + parts;
        L = ragged_layout(n_rec, cap);
        KARMA_RC(workspace(dev, s, L.total, &ws));
        bind_ragged(a, ws, L, cap);
    }
    a.part_base = cap_full;
    KARMA_RC(bind_lookback(dev, s, ragged_scan_blocks(n_rec), a));
    KARMA_HIP(launch_ragged_main(a, ds.cu, s));
    return 0;
}

struct Locked {
    std::lock_guard<std::mutex> lk{g_mu};
    int dev = 0;
    DevState* ds = nullptr;
    int rc = 0;
    Locked() {
        rc = current_device(&dev);
        if (!rc) rc = dev_state(dev, &ds);
    }
};

}  // namespace

namespace karma::engine {
int device_quad_blob(int dev, const uint32_t** out) {
    (void)dev;  // the current device (the caller set it)
    Locked L;
    if (L.rc) return L.rc;
    *out = L.ds->quad_blob;
    return 0;
}
int device_lane_blob(int dev, const uint32_t** out) {
    (void)dev;
    Locked L;
    if (L.rc) return L.rc;
    *out = L.ds->lane_blob;
    return 0;
}
int ragged_small_batch(const void* d_arena, const uint64_t* d_off, const uint32_t* d_len, size_t n_rec,
                       uint32_t* d_out, hipStream_t s) {
    return karma_crc32c_batch_ragged_bounded(d_arena, d_off, d_len, n_rec, 0, 1, nullptr, 0, d_out, s);
}
int ragged_small_batch_dev(const void* d_arena, const uint64_t* d_off, const uint32_t* d_len, const uint64_t* d_n,
                           uint64_t n_cap, const uint32_t* d_gate_len, uint32_t gate_max, uint32_t* d_out,
                           const uint32_t* d_stored, uint64_t* d_first_bad, hipStream_t s, int which,
                           bool stage_skew, uint32_t* d_skew_seen) {
    if (!n_cap) return 0;
    Locked L;
    if (L.rc) return L.rc;
    RaggedArgs a{};
    a.arena = static_cast<const uint8_t*>(d_arena);
    a.off = d_off;
    a.len = d_len;
    a.n_rec = n_cap;
    a.out = d_out;
    a.blob = L.ds->quad_blob;
    a.n_dev = d_n;
    a.gate_len = d_gate_len;
    a.gate_max = gate_max;
    a.cmp_stored = d_stored;
    a.cmp_bad = reinterpret_cast<unsigned long long*>(d_first_bad);
    bind_arena_bounds(a);
    // Two gated launches split the range of the batch's largest payload (known on the device
    // only): up to kStgGateLen the LDS-staged kernel (64 consecutive WAL payloads per wave's
    // stage, windows aligned to the record ends: k_ragged_staged_pipe), above it the 4-lane
    // groups (k_ragged_direct4); the other one returns at once (~5 us for the 4-lane kernel's
    // 4,096 waves to read the gate).  kSmallStaged / kSmallDirect launch one of them only.
    const uint32_t stg_max = std::min<uint32_t>(gate_max, kStgGateLen);
    if (which == kSmallDirect) a.gate_min = stg_max + 1;
    // (tools build, KARMA_SMALL_STAGED=0: the 4-lane launch below then takes the whole range,
    // gate_min 0, whatever `which` says, so the caller's small_batch_covers never overstates)
    if (which != kSmallDirect && KARMA_AB_KNOB("KARMA_SMALL_STAGED", 1)) {
        RaggedArgs b = a;
        b.blob = L.ds->lane_blob;
        b.gate_max = stg_max;
        b.stage_skew_seen = d_skew_seen;
        uint64_t sblocks = std::min<uint64_t>((uint64_t)L.ds->cu, ceil_div(n_cap, 64 * kStgWaves));
        if (const long g = KARMA_AB_KNOB("KARMA_STAGE_BLOCKS", 0); g > 0)  // (A/B: fewer CUs for the batch)
            sblocks = std::min<uint64_t>(sblocks, (uint64_t)g);
        units_timer_begin(s);  // (karma_crc32c_time_next_units: the replay's CRC kernel)
        KARMA_HIP(launch_ragged_staged_dev(b, (int)sblocks, s, stage_skew));
        units_timer_end(s);
        if (gate_max <= stg_max || which == kSmallStaged) return 0;
        a.gate_min = stg_max + 1;
    }
    const uint64_t blocks = std::min<uint64_t>((uint64_t)L.ds->cu, ceil_div(n_cap, 64 * kWavesPerBlock));
    KARMA_HIP(launch_ragged_direct_dev(a, (int)blocks, s));
    return 0;
}
int ragged_spec_batch_dev(const void* d_wal, uint64_t nseg, uint64_t seg_bytes, uint64_t first_pos, uint64_t base0,
                          uint64_t wal_end, WalSpec* d_spec, WalSummary* h_out, hipStream_t s, bool stage_skew,
                          bool direct) {
    Locked L;
    if (L.rc) return L.rc;
    RaggedArgs a{};
    a.arena = static_cast<const uint8_t*>(d_wal) + 8;  // payloads: the image shifted by the header
    a.n_rec = 1;  // (the slot count comes from segment 0's header, in the kernel)
    a.blob = direct ? L.ds->quad_blob : L.ds->lane_blob;
    a.spec = d_spec;
    a.spec_nseg = nseg;
    a.spec_seg = seg_bytes;
    a.spec_first = first_pos;
    a.spec_base0 = base0;
    a.spec_wal_end = wal_end;
    a.spec_out = h_out;
    bind_arena_bounds(a);
    units_timer_begin(s);  // (karma_crc32c_time_next_units: the replay's CRC kernel)
    if (direct)
        KARMA_HIP(launch_ragged_direct_spec(a, L.ds->cu, s));
    else
        KARMA_HIP(launch_ragged_staged_spec(a, L.ds->cu, s, stage_skew));
    units_timer_end(s);
    return 0;
}
namespace {
thread_local hipEvent_t t_units_start = nullptr, t_units_stop = nullptr;
}
#ifdef KARMA_AB
}  // namespace karma::engine
// Tools build only (wavelog.h): the units kernels log one WaveLogRec per wave into d_buf
// (cap records); d_buf = NULL stops the log.
// Tools build only: k_segment_once writes 8 wall-clock stamps per workgroup into d_buf (NULL: off):
// entry, tables and loads landed, waves folded, state published; the last workgroup also after
// its wait and at its end.
extern "C" int karma_ab_seg_log(void* d_buf) {
    return karma::engine::set_seg_log(d_buf) == hipSuccess ? 0 : KARMA_E_HIP;
}
// Tools build only: k_ragged_plan writes 6 wall-clock stamps per workgroup into d_buf[8 b ..] (entry,
// tables, block scan, look-back, entering registers, descriptors), k_ragged_finalize 3 into
// d_buf[32768 + 8 b ..] (entry, tables, records); NULL: off.
extern "C" int karma_ab_plan_log(void* d_buf) {
    return karma::engine::set_plan_log(d_buf) == hipSuccess ? 0 : KARMA_E_HIP;
}
extern "C" int karma_ab_wave_log(void* d_buf, uint64_t cap) {
    using namespace karma::engine;
    if (set_wave_log_ragged(d_buf, d_buf ? cap : 0) != hipSuccess || set_wave_log_fixed(d_buf, d_buf ? cap : 0) != hipSuccess)
        return KARMA_E_HIP;
    return 0;
}
namespace karma::engine {
#endif
void units_timer_begin(hipStream_t s) {
    if (t_units_start) (void)hipEventRecord(t_units_start, s);
}
void units_timer_end(hipStream_t s) {
    if (!t_units_start) return;
    if (t_units_stop) (void)hipEventRecord(t_units_stop, s);
    t_units_start = t_units_stop = nullptr;
}
// shared with rccl_comm.cc so RCCL failures land in karma_crc32c_last_error()
int set_last_error(int code, const std::string& what) { return fail(code, what); }
// The library's own streams (host, WAL, KFP contexts): their per-stream state freed before the
// context destroys the stream, so no state outlives its handle (which hipStreamCreate may hand
// out again).
int release_internal_stream(int dev, hipStream_t s) {
    if (!s) return 0;
    std::lock_guard<std::mutex> lk(g_mu);
    return g_states.release(dev, stream_key(s));
}
size_t stream_state_count() {
    std::lock_guard<std::mutex> lk(g_mu);
    return g_states.states();
}
}  // namespace karma::engine

extern "C" {

int karma_crc32c_abi_version(void) { return KARMA_CRC32C_ABI_VERSION; }

#ifdef KARMA_BOUNDS
// Bounds build only (bounds.h): out[0] = violations since the last reset, out[1..3] = the
// first one's site, index and capacity.  reset != 0 clears the reports afterwards.
int karma_debug_bounds_report(uint64_t* out, int reset) {
    if (!out) return fail(KARMA_E_INVALID, "debug_bounds_report: null");
    KARMA_HIP(hipDeviceSynchronize());
    KbReport all{0, 0, 0, 0};
    for (auto collect : {kb_collect_fixed, kb_collect_ragged, kb_collect_util, kb_collect_wal}) {
        KbReport r{};
        KARMA_HIP(collect(&r, reset != 0));
        if (r.count && !all.count) all = r;
        else all.count += r.count;
    }
    out[0] = all.count;
    out[1] = all.site;
    out[2] = all.index;
    out[3] = all.cap;
    return 0;
}
#endif

const char* karma_crc32c_strerror(int status) {
    switch (status) {
        case KARMA_OK: return "ok";
        case KARMA_E_INVALID: return "invalid argument";
        case KARMA_E_NO_DEVICE: return "no usable HIP device";
        case KARMA_E_HIP: return "HIP runtime error";
        case KARMA_E_NOMEM: return "out of memory";
        case KARMA_E_RCCL: return "RCCL error";
        case KARMA_E_IO: return "file I/O error";
        default: return "unknown status";
    }
}

const char* karma_crc32c_last_error(void) { return g_last.c_str(); }

int karma_crc32c_time_next_units(void* start_event, void* stop_event) {
    if (!start_event != !stop_event) return fail(KARMA_E_INVALID, "time_next_units: give both events or neither");
    karma::engine::t_units_start = static_cast<hipEvent_t>(start_event);
    karma::engine::t_units_stop = static_cast<hipEvent_t>(stop_event);
    return 0;
}

int karma_device_cu_count(void) {
    Locked L;
    if (L.rc) return L.rc;
    return L.ds->cu;
}

int karma_crc32c_batch_fixed(const void* d_data, size_t rec_bytes, size_t n_rec, const uint32_t* d_init,
                             uint32_t init, uint32_t* d_out, karma_stream_t stream) {
    if (n_rec == 0) return KARMA_OK;
    if (!d_out || (!d_data && rec_bytes)) return fail(KARMA_E_INVALID, "batch_fixed: null pointer");
    Locked L;
    if (L.rc) return L.rc;
    return fixed_locked(L.dev, *L.ds, d_data, rec_bytes, n_rec, d_init, init, d_out, (hipStream_t)stream);
}

int karma_crc32c_batch_ragged(const void* d_arena, const uint64_t* d_off, const uint32_t* d_len, size_t n_rec,
                              size_t total_len, const uint32_t* d_init, uint32_t init, uint32_t* d_out,
                              karma_stream_t stream) {
    return karma_crc32c_batch_ragged_bounded(d_arena, d_off, d_len, n_rec, total_len, 0, d_init, init, d_out, stream);
}

int karma_crc32c_batch_ragged_bounded(const void* d_arena, const uint64_t* d_off, const uint32_t* d_len, size_t n_rec,
                                      size_t total_len, uint32_t max_len, const uint32_t* d_init, uint32_t init,
                                      uint32_t* d_out, karma_stream_t stream) {
    if (n_rec == 0) return KARMA_OK;
    if (!d_out || !d_off || !d_len) return fail(KARMA_E_INVALID, "batch_ragged: null pointer");
    Locked L;
    if (L.rc) return L.rc;
    if (max_len && max_len <= kDirectMaxLen) {
        // every record small: one record per 4-lane group, no plan kernels (k_ragged_direct4); exact for
        // any length, so a wrong bound costs balance, never correctness
        RaggedArgs a{};
        a.arena = static_cast<const uint8_t*>(d_arena);
        a.off = d_off;
        a.len = d_len;
        a.n_rec = n_rec;
        a.init = d_init;
        a.init_scalar = init;
        a.out = d_out;
        const long dv = KARMA_AB_KNOB("KARMA_DIRECT_VARIANT", 0);
        const bool staged = dv >= 20 && dv <= 22;  // tools build: the LDS-staged kernel (its three forms)
        a.blob = staged ? L.ds->lane_blob : L.ds->quad_blob;
        bind_arena_bounds(a);
        // a wave takes 64 records: no more workgroups than the batch fills (each one loads its
        // table image into LDS first)
        const uint64_t per_block = 64 * (staged ? kStgWaves : kWavesPerBlock);
        const uint64_t blocks = std::min<uint64_t>((uint64_t)L.ds->cu, ceil_div(n_rec, per_block));
        KARMA_HIP(launch_ragged_direct(a, (int)blocks, (hipStream_t)stream));
        return KARMA_OK;
    }
    return ragged_locked(L.dev, *L.ds, d_arena, d_off, d_len, n_rec, total_len, d_init, init, d_out,
                         (hipStream_t)stream);
}

int karma_crc32c_stream(uint32_t init, const void* d_data, size_t n, uint32_t* d_out, karma_stream_t stream) {
    return karma_crc32c_batch_fixed(d_data, n, 1, nullptr, init, d_out, stream);
}

// ---- resource lifetime (include/karma_crc32c.h, stream_state.h) -----------------------------
namespace {
int select_device(int device, int* dev) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return fail(KARMA_E_NO_DEVICE, "no HIP device visible");
    if (device >= n) return fail(KARMA_E_INVALID, "device index out of range");
    if (device >= 0) KARMA_HIP(hipSetDevice(device));
    KARMA_HIP(hipGetDevice(dev));
    return 0;
}
}  // namespace

int karma_crc32c_release_stream(int device, karma_stream_t stream) {
    int dev = 0;
    KARMA_RC(select_device(device, &dev));
    std::lock_guard<std::mutex> lk(g_mu);
    if (HipStateOps().capturing(stream)) return fail(KARMA_E_INVALID, "release_stream: the stream is capturing");
    return g_states.release(dev, stream_key((hipStream_t)stream));
}

int karma_crc32c_trim(int device) {
    int dev = 0;
    KARMA_RC(select_device(device, &dev));
    {
        std::lock_guard<std::mutex> lk(g_mu);
        KARMA_RC(g_states.trim(dev));
    }
    return karma::engine::trim_host_contexts(dev);
}

int karma_crc32c_graph_hold(int device, int delta) {
    int dev = 0;
    KARMA_RC(select_device(device, &dev));
    std::lock_guard<std::mutex> lk(g_mu);
    return g_states.hold(dev, delta);
}

int karma_crc32c_stream_states(void) { return (int)karma::engine::stream_state_count(); }

}  // extern "C"

extern "C" {

int karma_crc32c_batch_fixed_sharded(karma_comm_t comm, const void* d_local, size_t rec_bytes, size_t n_local,
                                     uint32_t init, uint32_t* d_local_out, uint32_t* d_all_out, int root,
                                     karma_stream_t stream) {
    if (!comm) return fail(KARMA_E_INVALID, "batch_fixed_sharded: null comm");
    KARMA_RC(karma_crc32c_batch_fixed(d_local, rec_bytes, n_local, nullptr, init, d_local_out, stream));
    return karma_crc32c_gather_u32(comm, d_local_out, n_local, d_all_out, root, stream);
}

// ---- synthetic data / probes -----------------------------------------------------
int karma_fill_splitmix64(void* d_dst, size_t n_bytes, uint64_t seed, uint64_t first_byte, karma_stream_t stream) {
    if (!n_bytes) return 0;
    if (!d_dst || (first_byte & 7u) || (reinterpret_cast<uintptr_t>(d_dst) & 15u))
        return fail(KARMA_E_INVALID, "fill_splitmix64: null, first_byte % 8 or destination not 16-byte aligned");
    int dev;
    KARMA_RC(current_device(&dev));
    KARMA_HIP(launch_fill_splitmix(static_cast<uint8_t*>(d_dst), n_bytes, seed, first_byte, (hipStream_t)stream));
    return 0;
}

int karma_stream_probe(const void* d_src, size_t n_bytes, uint32_t* d_out, karma_stream_t stream) {
    if (!d_out || (!d_src && n_bytes) || (reinterpret_cast<uintptr_t>(d_src) & 15u))
        return fail(KARMA_E_INVALID, "stream_probe: null or source not 16-byte aligned");
    Locked L;
    if (L.rc) return L.rc;
    KARMA_HIP(launch_stream_probe(static_cast<const uint8_t*>(d_src), n_bytes, d_out, L.ds->cu,
                                  (hipStream_t)stream));
    return 0;
}

}  // extern "C"
