// karma_amd/csrc/wal.cc -- batched WAL framing and replay on top of the GPU
// CRC batches.
//
// Record format (karma-store/segment_file.cc:21-31, common.h:11):
//   [crc u32 LE = Value(payload)][len << 8 | type u32 LE][payload]
// type 1 = padding to the segment end with '0' bytes and crc field 0
// (segment_file.cc:33-49); a segment tail shorter than a header is padded
// with '0' bytes only (:34-39).
//
// (karma_wal_append_batch, sivir::build_sqe's loop, is in wal_append.cc.)
// karma_wal_replay        = sivir::open's loop over wal::scan_record
//   (sivir.cc:31-41, wal.cc:34-87), entirely on the device over an image in
//   HBM (wal_device.hip): segment-parallel header walk, one ragged CRC batch
//   over every payload, first mismatch; replay stops where scan_record would
//   return false.  A host image is first streamed into HBM through pinned
//   staging buffers filled by several threads.  The reference's quirk for a type-0
//   record of size 0 is kept: read_exact_at returns early for size 0
//   (segment_file.cc:8) so the CRC is taken over the stale 4-byte len/type
//   word just read (wal.cc:50-60).  It is load-bearing: it is what ends replay
//   at the zero-filled, never-written part of the last segment.
#include <hip/hip_runtime_api.h>
#include <unistd.h>
#include <sys/stat.h>
#include <fcntl.h>
#include <dirent.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "ab.h"
#include "engine.h"
#include "host_stage.h"
#include "host_trace.h"
#include "karma_crc32c.h"

namespace karma::engine {
int set_last_error(int code, const std::string& what);  // capi.cc

// How the walk splits the segments.  The header chain is serial inside a
// segment, so few segments leave most of the GPU idle: each segment is then cut
// into sub-ranges (at least 16 KiB) so that about 20 walkers per CU run, and
// k_wal_resolve stitches their lists.  Many segments: one walker per segment.
// sub_bytes != 0 forces the sub-range size (karma_wal_tuning: tests, tuning);
// the tools build's KARMA_WALK_VARIANT=1 (ab.h) selects k_wal_walk instead.
WalWalkPlan wal_walk_plan(uint64_t seg_bytes, uint64_t nseg, int cu, uint64_t sub_bytes, bool inline_crc,
                          bool list_crc) {
    WalWalkPlan p{1, 0, 0, 0, list_crc ? 3 : inline_crc ? 2 : 0, cu};
    if (list_crc) inline_crc = false;  // the walkers are k_wal_walk_sub's
    const uint64_t tiles = (seg_bytes + kWalkTile - 1) / kWalkTile;
    uint64_t sub_tiles = tiles;
    if (!inline_crc && KARMA_AB_KNOB("KARMA_WALK_VARIANT", 0) == 1) {
        p.kernel = 1;
    } else if (sub_bytes) {
        sub_tiles = std::max<uint64_t>(1, sub_bytes / kWalkTile);
    } else {
        // walkers: 20 per CU (1M x 180 B in 188 segments of 1 MiB: 40 KiB sub-ranges; 24-40 KiB
        // measured 11 us faster per replay call than 48 KiB); with the CRCs
        // inline, one workgroup of kWalFuseWaves walkers per CU
        const uint64_t per_cu = inline_crc ? (uint64_t)kWalFuseWaves : 20;
        const uint64_t want = per_cu * (uint64_t)(cu > 0 ? cu : 1);
        if (nseg > 0 && nseg < want) {
            const uint64_t per = (want + nseg - 1) / nseg;  // sub-ranges per segment
            sub_tiles = std::max<uint64_t>(4, (tiles + per - 1) / per);
        }
    }
    sub_tiles = std::min(sub_tiles, tiles);
    sub_tiles = std::max(sub_tiles, (tiles + kMaxSub - 1) / kMaxSub);
    p.sub_bytes = sub_tiles * kWalkTile;
    p.nsub = p.kernel == 1 ? 1 : (seg_bytes + p.sub_bytes - 1) / p.sub_bytes;
    if (p.nsub == 1) p.sub_bytes = seg_bytes;
    p.sub_cap = p.sub_bytes / 8 + 1;
    p.cand_cap = p.nsub * p.sub_cap;
    return p;
}

}  // namespace karma::engine

namespace {

// body(i) for i in [lo, hi) on up to 16 std::threads, at least `grain` items each.
template <typename F>
void parallel_for(uint64_t lo, uint64_t hi, uint64_t grain, F&& body) {
    const uint64_t n = hi > lo ? hi - lo : 0;
    const uint64_t nthr = std::min<uint64_t>(16, std::max<uint64_t>(1, n / std::max<uint64_t>(grain, 1)));
    if (nthr <= 1) {
        for (uint64_t i = lo; i < hi; ++i) body(i);
        return;
    }
    std::vector<std::thread> th;
    for (uint64_t t = 0; t < nthr; ++t)
        th.emplace_back([&, t] {
            for (uint64_t i = lo + n * t / nthr; i < lo + n * (t + 1) / nthr; ++i) body(i);
        });
    for (auto& x : th) x.join();
}

int fail(int code, const char* what) { return karma::engine::set_last_error(code, what); }
int fail(int code, const std::string& what) { return karma::engine::set_last_error(code, what); }

// Per-device replay context: a stream, the device image buffer (host images
// are streamed into it), the walk's candidate tables, the contiguous lists and
// the pinned staging ring of the upload.  Grow-only; one replay at a time per
// device (the context's lock).
struct DevBuf {
    void* p = nullptr;
    size_t bytes = 0;
    bool host = false;
    int ensure(size_t want, bool pinned_host = false) {
        if (p && bytes >= want) return 0;
        if (p) (void)(host ? hipHostFree(p) : hipFree(p));
        p = nullptr;
        bytes = 0;
        want = std::max<size_t>(want + want / 8, 256);
        const hipError_t e = pinned_host ? hipHostMalloc(&p, want, hipHostMallocDefault) : hipMalloc(&p, want);
        if (e != hipSuccess) {
            p = nullptr;
            return fail(e == hipErrorOutOfMemory ? KARMA_E_NOMEM : KARMA_E_HIP, "wal_replay: allocation");
        }
        bytes = want;
        host = pinned_host;
        return 0;
    }
    void release() {
        if (p) (void)(host ? hipHostFree(p) : hipFree(p));
        p = nullptr;
        bytes = 0;
    }
    template <typename T>
    T* as() const {
        return static_cast<T*>(p);
    }
};

// Walkers switch to direct header rounds after a fast round of this many headers.
constexpr uint32_t kDirectStreak = 8;
// Passes that skip the uniform-stride pass after it declined (a WAL of mixed sizes declines in
// its probe: ~10 us of a call that then walks).
constexpr uint32_t kSpecSkip = 16;
#ifdef KARMA_AB
std::atomic<int> g_spec_last{0};  // the last pass's uniform-stride outcome (karma_ab_wal_spec_last)
#endif
constexpr uint32_t kSmallRecordMax = 1024;      // payloads up to this take the one-record-per-group batch
struct ReplayCtx {
    std::mutex mu;
    bool ready = false;
    int cu = 1;
    hipStream_t st = nullptr;
    // the sliced pass (tools build, KARMA_WAL_SLICES=2): the CRC batches' stream and the events
    // ordering them after their slice's gather
    hipStream_t st2 = nullptr;
    hipEvent_t ev[3] = {nullptr, nullptr, nullptr};
    DevBuf img, crec, clen, ccrc, meta, sub, span, cbase, off, len, stored, crc, sum;
    // the fused resolve + gather's tagged words (WalArgs::rg_words), zeroed when (re)allocated and
    // when the 16-bit call tag wraps
    DevBuf rgw;
    void* rgw_zeroed = nullptr;
    uint32_t rg_seq = 0;
    DevBuf h_small;                             // pinned readback of the summary
    uint64_t img_gen = 0;                       // uploads of a host image into img so far
    // the largest payload of the last device-planned pass on this context: the next pass
    // launches only the small-record kernel that covered it (karma::engine::SmallWhich)
    bool have_len_hint = false;
    uint32_t len_hint = 0;
    // whether the last pass's staged batch met records on few LDS banks: this pass then launches
    // the staged kernel with the skewed stage (else the plain-stage form, 3-5 us faster)
    bool skew_hint = true;
    // the uniform-stride pass (WalSpec): its probe result on the device; after it declines, the
    // next kSpecSkip passes go straight to the walk
    DevBuf spec;
    void* spec_init = nullptr;  // spec holds the between-calls state (keys ~0, counters 0) for this allocation
    uint32_t spec_skip = 0;
    int init(int dev) {
        if (ready) return 0;
        hipDeviceProp_t prop;
        if (hipGetDeviceProperties(&prop, dev) != hipSuccess) return fail(KARMA_E_HIP, "hipGetDeviceProperties");
        cu = std::max(1, prop.multiProcessorCount);
        if (hipStreamCreateWithFlags(&st, hipStreamNonBlocking) != hipSuccess) return fail(KARMA_E_HIP, "stream");
        ready = true;
        return 0;
    }
    // karma_crc32c_trim (the caller holds mu): everything freed, recreated by the next replay.
    void reset(int dev) {
        if (!ready) return;
        (void)hipStreamSynchronize(st);
        (void)karma::engine::release_internal_stream(dev, st);
        for (DevBuf* b : {&img, &crec, &clen, &ccrc, &meta, &sub, &span, &cbase, &off, &len, &stored, &crc, &sum, &h_small,
                          &rgw, &spec})
            b->release();
        rgw_zeroed = nullptr;
        rg_seq = 0;
        spec_init = nullptr;
        (void)hipStreamDestroy(st);
        st = nullptr;
        if (st2) {
            (void)hipStreamSynchronize(st2);
            (void)karma::engine::release_internal_stream(dev, st2);
            (void)hipStreamDestroy(st2);
            st2 = nullptr;
        }
        for (hipEvent_t& e : ev) {
            if (e) (void)hipEventDestroy(e);
            e = nullptr;
        }
        ++img_gen;  // a replay between passes must not take the freed image for its own
        ready = false;
    }
};
std::mutex g_rctx_mu;
std::vector<std::unique_ptr<ReplayCtx>> g_rctx;

ReplayCtx& replay_ctx(int dev) {
    std::lock_guard<std::mutex> g(g_rctx_mu);
    if ((int)g_rctx.size() <= dev) g_rctx.resize(dev + 1);
    if (!g_rctx[dev]) g_rctx[dev] = std::make_unique<ReplayCtx>();
    return *g_rctx[dev];
}

}  // namespace

int karma::engine::trim_replay_ctx(int dev) {
    ReplayCtx& c = replay_ctx(dev);
    std::lock_guard<std::mutex> lk(c.mu);
    c.reset(dev);
    return 0;
}

namespace {

// Fills dst with image bytes [off, off + n) (offsets relative to the image start); the
// image is streamed into HBM through the library's pinned staging (host_stage.h).
using ImageFill = karma::engine::HostFill;

// A host image already in the replay context's device buffer (replay_core's later passes reuse it):
// its first segment and the context's upload count when it was uploaded (gen 0: none).
struct Uploaded {
    uint64_t seg = 0, gen = 0;
};
int replay_pass(const uint8_t* d_wal, const ImageFill* fill, size_t wal_bytes, size_t seg_bytes, uint64_t start,
                uint64_t* h_n_records, uint64_t* h_stop, int* h_status, uint64_t* h_rec_off, size_t rec_cap,
                int device, const karma_wal_tuning* tuning, const uint8_t* h_pinned, Uploaded* up);

// sivir::open's loop (sivir.cc:31-41) as device passes.  One pass replays from `start` until
// scan_record would return false, or until an accepted size-0 record carries the chain past a
// segment's end (kWalSpill, engine.h): the reference then enters the next segment 1-4 bytes in
// (it advances record.size() = 12, wal.cc:66 / sivir.cc:38), so the next pass starts there.
// The records of all passes are concatenated.  A chain carried past the image's last segment
// ends replay (scan_record finds no segment, wal.cc:86) with the stop offset past wal_bytes,
// where sivir::open's start_wal_offset is left.  A host image is streamed into HBM once: the later
// passes start at or past the first one's segment and walk the copy already there.
int replay_core(const uint8_t* d_wal, const ImageFill* fill, size_t wal_bytes, size_t seg_bytes, uint64_t start,
                uint64_t* h_n_records, uint64_t* h_stop, int* h_status, uint64_t* h_rec_off, size_t rec_cap,
                int device, const karma_wal_tuning* tuning, const uint8_t* h_pinned = nullptr) {
    uint64_t total = 0;
    Uploaded up;
    while (true) {
        uint64_t n = 0, stop = 0;
        int status = 0;
        const uint64_t got = std::min<uint64_t>(total, rec_cap);
        if (const int rc = replay_pass(d_wal, fill, wal_bytes, seg_bytes, start, &n, &stop, &status,
                                       h_rec_off ? h_rec_off + got : nullptr, rec_cap - got, device, tuning, h_pinned,
                                       &up))
            return rc;
        total += n;
        if (status != (int)karma::engine::kWalSpill) {
            *h_n_records = total;
            *h_stop = stop;
            *h_status = status;
            return 0;
        }
        start = stop;  // > the previous start: every pass makes progress
        if (start >= wal_bytes) {  // carried past the last segment: scan_record finds none
            *h_n_records = total;
            *h_stop = start;
            *h_status = KARMA_WAL_END;
            return 0;
        }
    }
}

}  // namespace

extern "C" {

#ifdef KARMA_AB
// Tools build only: the last replay pass's uniform-stride outcome on any device (0 not tried,
// 1 its result taken, 2 declined: the walk decided).
int karma_ab_wal_spec_last(void) { return g_spec_last.load(); }
#endif

int karma_wal_replay(const void* h_wal, const void* d_wal, size_t wal_bytes, size_t seg_bytes, uint64_t start,
                     uint64_t* h_n_records, uint64_t* h_stop, int* h_status, uint64_t* h_rec_off, size_t rec_cap,
                     int device) {
    return karma_wal_replay_tuned(h_wal, d_wal, wal_bytes, seg_bytes, start, h_n_records, h_stop, h_status, h_rec_off,
                                  rec_cap, device, nullptr);
}

int karma_wal_replay_tuned(const void* h_wal, const void* d_wal, size_t wal_bytes, size_t seg_bytes, uint64_t start,
                           uint64_t* h_n_records, uint64_t* h_stop, int* h_status, uint64_t* h_rec_off, size_t rec_cap,
                           int device, const karma_wal_tuning* tuning) {
    // (start may lie up to 4 bytes past the image: where replay stops after an accepted size-0
    // record at the image end, wal.cc:66 / sivir.cc:38; such a stop is a valid start, replaying nothing)
    if ((!h_wal && !d_wal) || !h_n_records || !h_stop || !h_status || seg_bytes < 1 || wal_bytes % seg_bytes ||
        start > wal_bytes + 4 || seg_bytes >= (uint64_t(1) << 31) ||
        (tuning && (tuning->crc_batch < 0 || tuning->crc_batch > KARMA_WAL_CRC_INLINE)))
        return fail(KARMA_E_INVALID, "wal_replay");
    const uint8_t* src = static_cast<const uint8_t*>(h_wal);
    const ImageFill copy = [src](uint8_t* dst, uint64_t off, size_t n) {
        std::memcpy(dst, src + off, n);
        return 0;
    };
    // a page-locked image is DMA'd as it is (no staging copies)
    const uint8_t* pinned = !d_wal && karma::engine::host_range_pinned(src, wal_bytes) ? src : nullptr;
    return replay_core(static_cast<const uint8_t*>(d_wal), d_wal ? nullptr : &copy, wal_bytes, seg_bytes, start,
                       h_n_records, h_stop, h_status, h_rec_off, rec_cap, device, tuning, pinned);
}

}  // extern "C"

namespace {

#ifdef KARMA_AB
// The device-planned pass in two slices of segments (tools build A/B, KARMA_WAL_SLICES=2; round 6,
// DESIGN.md §8a): slice k's walk and gather on the replay stream, its staged CRC batch on a second
// stream ordered after that gather by an event, so slice 1's walk can run beside slice 0's CRCs.
// Each slice is replayed as an image of its own (its lists, its summary); replay enters slice 1 at
// offset 0 exactly when slice 0's walk ended cleanly at its last segment's end (status END: no
// stop, no spill), and its results then follow slice 0's.  Otherwise slice 1's work was
// speculative and slice 0's result is the pass's (a spill continues in replay_core as usual).
// Taken only when the previous pass's largest payload went to the staged kernel; returns 1 when a
// slice's payloads were not covered by it (the caller then runs the pass unsliced).
int sliced_pass(ReplayCtx& c, const karma::engine::WalArgs& A, const karma_wal_tuning* tuning, uint64_t* h_n_records,
                uint64_t* h_stop, int* h_status, uint64_t* h_rec_off, size_t rec_cap) {
    using namespace karma::engine;
    const uint64_t seg = A.seg_bytes, nwork = A.nwork;
    const uint64_t n0 = (nwork + 1) / 2, ns[2] = {n0, nwork - n0};
    // (KARMA_WAL_SLICE_PLAN=1: the sub-range split of the whole image's plan, not of a slice's)
    const uint64_t plan_nseg = KARMA_AB_KNOB("KARMA_WAL_SLICE_PLAN", 0) ? nwork : n0;
    const WalWalkPlan plan = wal_walk_plan(seg, plan_nseg, c.cu, tuning ? tuning->walk_sub_bytes : 0, false, false);
    const uint64_t cap[2] = {ns[0] * seg / 8 + ns[0], ns[1] * seg / 8 + ns[1]};
    if (!c.st2 && hipStreamCreateWithFlags(&c.st2, hipStreamNonBlocking) != hipSuccess) {
        c.st2 = nullptr;
        return fail(KARMA_E_HIP, "wal_replay: stream");
    }
    for (hipEvent_t& e : c.ev)
        if (!e && hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) {
            e = nullptr;
            return fail(KARMA_E_HIP, "wal_replay: event");
        }
    for (auto [b, bytes] : {std::pair<DevBuf*, size_t>{&c.crec, nwork * plan.cand_cap * 4}, {&c.clen, nwork * plan.cand_cap * 4},
                            {&c.ccrc, nwork * plan.cand_cap * 4}, {&c.meta, nwork * sizeof(WalSegMeta)},
                            {&c.sub, nwork * plan.nsub * sizeof(WalSubMeta)}, {&c.span, nwork * plan.nsub * 8},
                            {&c.cbase, nwork * 8}, {&c.sum, 2 * sizeof(WalSummary)}, {&c.off, (cap[0] + cap[1]) * 8},
                            {&c.len, (cap[0] + cap[1]) * 4}, {&c.stored, (cap[0] + cap[1]) * 4}, {&c.crc, (cap[0] + cap[1]) * 4}})
        if (const int rc = b->ensure(bytes)) return rc;
    if (const int rc = c.h_small.ensure(2 * sizeof(WalSummary), true)) return rc;
    WalArgs S[2];
    for (int k = 0; k < 2; ++k) {
        const uint64_t s0 = k ? n0 : 0, l0 = k ? cap[0] : 0;
        WalArgs& a = S[k];
        a = A;
        a.wal = A.wal + s0 * seg;
        a.base0 = A.base0 + s0 * seg;
        a.first_pos = k ? 0 : A.first_pos;
        a.nwork = ns[k];
        a.img_bytes = ns[k] * seg;
        a.wal_end = a.base0 + a.img_bytes;
        a.nsub = plan.nsub;
        a.sub_bytes = plan.sub_bytes;
        a.sub_cap = plan.sub_cap;
        a.cand_cap = plan.cand_cap;
        a.cand_rec = c.crec.as<uint32_t>() + s0 * plan.cand_cap;
        a.cand_len = c.clen.as<uint32_t>() + s0 * plan.cand_cap;
        a.cand_crc = c.ccrc.as<uint32_t>() + s0 * plan.cand_cap;
        a.meta = c.meta.as<WalSegMeta>() + s0;
        a.sub = c.sub.as<WalSubMeta>() + s0 * plan.nsub;
        a.span = c.span.as<uint32_t>() + s0 * plan.nsub * 2;
        a.cand_base = c.cbase.as<uint64_t>() + s0;
        a.sum = c.sum.as<WalSummary>() + k;
        a.first_bad = &a.sum->first_bad;
        a.off = c.off.as<uint64_t>() + l0;
        a.len = c.len.as<uint32_t>() + l0;
        a.stored = c.stored.as<uint32_t>() + l0;
        a.crc = c.crc.as<uint32_t>() + l0;
        a.n_all = cap[k];
    }
    const long skew_knob = KARMA_AB_KNOB("KARMA_STAGE_SKEW", -1);
    for (int k = 0; k < 2; ++k) {
        WalArgs& a = S[k];
        if (launch_wal_walk(a, ns[k], plan, c.st) != hipSuccess || launch_wal_gather(a, ns[k], true, c.cu, c.st) != hipSuccess ||
            hipEventRecord(c.ev[k], c.st) != hipSuccess || hipStreamWaitEvent(c.st2, c.ev[k], 0) != hipSuccess)
            return fail(KARMA_E_HIP, "wal_replay: sliced walk");
        if (const int rc = ragged_small_batch_dev(a.wal + 8, a.off, a.len, &a.sum->n_all, cap[k], &a.sum->max_len,
                                                  kSmallRecordMax, const_cast<uint32_t*>(a.crc), a.stored, a.first_bad,
                                                  c.st2, kSmallStaged, skew_knob >= 0 ? skew_knob != 0 : c.skew_hint,
                                                  &a.sum->stage_skew))
            return rc;
    }
    WalSummary* H = c.h_small.as<WalSummary>();
    if (hipEventRecord(c.ev[2], c.st2) != hipSuccess || hipStreamWaitEvent(c.st, c.ev[2], 0) != hipSuccess ||
        launch_wal_publish(S[0].sum, H, c.st) != hipSuccess || launch_wal_publish(S[1].sum, H + 1, c.st) != hipSuccess ||
        hipStreamSynchronize(c.st) != hipSuccess)
        return fail(KARMA_E_HIP, "wal_replay: sliced pass");
    const WalSummary a = H[0], b = H[1];
    const bool whole = a.status == KARMA_WAL_END;  // replay entered slice 1 at its first byte
    const uint32_t max_len = std::max(a.n_all ? a.max_len : 0u, whole && b.n_all ? b.max_len : 0u);
    if (max_len > kStgGateLen) return 1;  // not all payloads were checksummed by the staged batch
    if (a.n_all || (whole && b.n_all)) {
        c.have_len_hint = true;
        c.len_hint = max_len;
    }
    c.skew_hint = a.stage_skew != 0 || (whole && b.stage_skew != 0);
    const uint64_t n_all[2] = {a.n_all, whole ? b.n_all : 0};
    uint64_t accepted = n_all[0] + n_all[1];
    int status = (int)(whole ? b.status : a.status);
    uint64_t end = whole ? b.end : a.end;
    int bad_k = -1;
    uint64_t bad_i = 0;
    if (a.first_bad < n_all[0]) {
        bad_k = 0;
        bad_i = a.first_bad;
        accepted = a.first_bad;
    } else if (whole && b.first_bad < n_all[1]) {
        bad_k = 1;
        bad_i = b.first_bad;
        accepted = n_all[0] + b.first_bad;
    }
    if (bad_k >= 0) {  // the first mismatch in WAL order: "Corrupt record"
        uint64_t at = 0;
        if (hipMemcpyAsync(&at, S[bad_k].off + bad_i, 8, hipMemcpyDeviceToHost, c.st) != hipSuccess ||
            hipStreamSynchronize(c.st) != hipSuccess)
            return fail(KARMA_E_HIP, "wal_replay: D2H");
        status = KARMA_WAL_CORRUPT;
        end = S[bad_k].base0 + at;
    }
    if (h_rec_off && rec_cap && accepted) {  // slice 0's offsets, then slice 1's
        uint64_t done = 0;
        for (int k = 0; k < 2 && done < std::min<uint64_t>(accepted, rec_cap); ++k) {
            const uint64_t m = std::min<uint64_t>({n_all[k], accepted - done, rec_cap - done});
            if (!m) continue;
            if (hipMemcpyAsync(h_rec_off + done, S[k].off, m * 8, hipMemcpyDeviceToHost, c.st) != hipSuccess ||
                hipStreamSynchronize(c.st) != hipSuccess)
                return fail(KARMA_E_HIP, "wal_replay: D2H offsets");
            const uint64_t base = S[k].base0;
            uint64_t* o = h_rec_off + done;
            parallel_for(0, m, 1 << 16, [&](uint64_t i) { o[i] += base; });
            done += m;
        }
    }
    *h_n_records = accepted;
    *h_stop = end;
    *h_status = status;
    return 0;
}
#endif

// One replay pass (replay_core): the image is d_wal, or produced by fill and streamed into
// HBM (or, h_pinned: the same image in page-locked host memory, one DMA).  Offsets in and
// out are relative to the image start.
int replay_pass(const uint8_t* d_wal, const ImageFill* fill, size_t wal_bytes, size_t seg_bytes, uint64_t start,
                uint64_t* h_n_records, uint64_t* h_stop, int* h_status, uint64_t* h_rec_off, size_t rec_cap,
                int device, const karma_wal_tuning* tuning, const uint8_t* h_pinned, Uploaded* up) {
    using namespace karma::engine;
    const uint64_t nseg = wal_bytes / seg_bytes;
    const uint64_t s0 = std::min<uint64_t>(start / seg_bytes, nseg);
    const uint64_t nwork = nseg - s0;
    if (!nwork) {  // nothing past start: replay is already at the end
        *h_n_records = 0;
        *h_stop = start;
        *h_status = KARMA_WAL_END;
        return 0;
    }
    int n = 0, dev = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return fail(KARMA_E_NO_DEVICE, "no HIP device visible");
    if (device >= n) return fail(KARMA_E_INVALID, "wal_replay: device index out of range");
    if (device >= 0 && hipSetDevice(device) != hipSuccess) return fail(KARMA_E_HIP, "hipSetDevice");
    if (hipGetDevice(&dev) != hipSuccess) return fail(KARMA_E_HIP, "hipGetDevice");
    ReplayCtx& c = replay_ctx(dev);
    std::lock_guard<std::mutex> lk(c.mu);
    if (const int rc = c.init(dev)) return rc;
    PhaseTimer T("wal_replay");
    const uint64_t base0 = s0 * seg_bytes, img_bytes = nwork * seg_bytes;
    WalArgs A{};
    // 0. the image in HBM: the caller's copy, or the host image streamed in
    if (d_wal) {
        A.wal = static_cast<const uint8_t*>(d_wal) + base0;
    } else if (up && up->gen && up->gen == c.img_gen && s0 >= up->seg) {
        // a later pass of the same replay: the image is still in the context's buffer (no other
        // upload since, the context's lock held by each pass)
        A.wal = c.img.as<const uint8_t>() + (s0 - up->seg) * seg_bytes;
    } else {
        if (const int rc = c.img.ensure(img_bytes)) return rc;
        ++c.img_gen;
        if (up) *up = Uploaded{s0, c.img_gen};
        if (h_pinned) {
            if (hipMemcpyAsync(c.img.p, h_pinned + base0, img_bytes, hipMemcpyHostToDevice, c.st) != hipSuccess ||
                hipStreamSynchronize(c.st) != hipSuccess)
                return fail(KARMA_E_HIP, "wal_replay: image upload");
        } else if (const int rc = staged_upload(dev, c.img.p, *fill, base0, img_bytes)) {
            return rc;
        }
        A.wal = c.img.as<const uint8_t>();
        T.mark("image upload");
    }
    A.base0 = base0;
    A.img_bytes = img_bytes;
    A.nwork = nwork;
    A.seg_bytes = seg_bytes;
    A.first_pos = start - base0;
    A.direct_streak = (uint32_t)KARMA_AB_KNOB("KARMA_WALK_DIRECT", kDirectStreak);
    const int batch = tuning ? tuning->crc_batch : KARMA_WAL_CRC_PLAN;
    // Images up to kDevicePlanMax take a device-planned path (one host round trip): with the
    // default plan the walkers checksum the candidates inline (k_wal_walk_crc); the tools
    // build's other walk / small-record kernels, and KARMA_WAL_CRC_SEPARATE, walk first and
    // then run one small-record batch over the gathered lists (the round-2 path).
    const bool dev_plan = img_bytes <= kDevicePlanMax && batch != KARMA_WAL_CRC_UNITS;
    // (k_wal_plan packs the inline path's first mismatch as ordinal << 24 | segment: fewer than
    // 2^24 segments, else the gathered batch)
    const bool inline_crc = dev_plan && batch == KARMA_WAL_CRC_INLINE && nwork < (uint64_t(1) << 24) &&
                            KARMA_AB_KNOB("KARMA_WALK_VARIANT", 0) == 0;
    // the walkers' lists checksummed after the walk by the LDS-staged kernel (k_wal_list_crc)
    // instead of by the walkers themselves (k_wal_walk_crc)
    const bool list_crc = inline_crc && KARMA_AB_KNOB("KARMA_WAL_LIST_CRC", 0) != 0;
    if (inline_crc) {
        if (const int rc = list_crc ? device_lane_blob(dev, &A.crc_blob) : device_quad_blob(dev, &A.crc_blob))
            return rc;
#ifdef KARMA_BOUNDS
        hipDeviceptr_t lo = nullptr;
        size_t sz = 0;
        if (hipMemGetAddressRange(&lo, &sz, (hipDeviceptr_t)A.wal) == hipSuccess) {
            A.kb_lo = reinterpret_cast<uintptr_t>(lo);
            A.kb_hi = A.kb_lo + sz;
        } else {
            (void)hipGetLastError();
            A.kb_lo = 0;
            A.kb_hi = ~uintptr_t(0);
        }
#endif
    }
#ifdef KARMA_AB
    if (KARMA_AB_KNOB("KARMA_WAL_SLICES", 1) == 2 && dev_plan && !inline_crc && batch == KARMA_WAL_CRC_PLAN &&
        nwork >= 2 && (nwork + 1) / 2 <= 1024 && c.have_len_hint && c.len_hint <= kStgGateLen) {
        const int rc = sliced_pass(c, A, tuning, h_n_records, h_stop, h_status, h_rec_off, rec_cap);
        if (rc != 1) return rc;
        c.have_len_hint = false;  // the unsliced pass below launches both small-record kernels
    }
#endif
#ifdef KARMA_AB
    g_spec_last = 0;
#endif
    // 0b. the uniform-stride pass (engine.h WalSpec): when replay's first header (at
    //     `start`) is a record of n <= kStgGateLen bytes, check the rest of its segment and every later
    //     segment as records of that size and their CRCs in one staged batch, with no walk, gather or
    //     lists.  Its result is final when the first place that breaks the assumption (if any) comes
    //     after replay's stop; otherwise the walk below decides (one host round trip spent).  The
    //     tools build's KARMA_WAL_SPEC: 0 never, 2 every pass (no skipping after a decline).
    const long spec_knob = KARMA_AB_KNOB("KARMA_WAL_SPEC", 1);
    // (a caller's forced sub-range size asks for the walk: karma_wal_tuning)
    const bool spec_try = spec_knob != 0 && dev_plan && !inline_crc && batch == KARMA_WAL_CRC_PLAN &&
                          A.first_pos + 9 <= seg_bytes && !(tuning && tuning->walk_sub_bytes) && nwork <= kSpecMaxSeg &&
                          (spec_knob == 2 || c.spec_skip == 0);
    if (!spec_try && c.spec_skip) --c.spec_skip;
    if (spec_try) {
        if (const int rc = c.h_small.ensure(64, true)) return rc;
        if (const int rc = c.spec.ensure(sizeof(WalSpec))) return rc;
        WalSpec* d_spec = c.spec.as<WalSpec>();
        if (c.spec.p != c.spec_init) {  // a fresh allocation: the state each pass leaves for the next
            static const WalSpec kFresh{~0ull, ~0ull, 0u, 0u};
            if (hipMemcpyAsync(d_spec, &kFresh, sizeof(kFresh), hipMemcpyHostToDevice, c.st) != hipSuccess ||
                hipStreamSynchronize(c.st) != hipSuccess)
                return fail(KARMA_E_HIP, "wal_replay: uniform-stride state");
            c.spec_init = c.spec.p;
        }
        WalSummary* S = c.h_small.as<WalSummary>();
        S->spec = 0;  // (the kernel's last workgroup overwrites it: 0 after the sync would be no result)
        // one launch: its workgroups read the stride from segment 0's first header, check every
        // slot, and the last one writes the summary straight into page-locked memory
        // the 4-lane form when the last pass's payloads were over the staged kernel's gate
        const bool direct = c.have_len_hint && c.len_hint > kStgGateLen;
        if (const int rc = ragged_spec_batch_dev(A.wal, nwork, seg_bytes, A.first_pos, base0, wal_bytes, d_spec, S, c.st,
                                                 c.skew_hint, direct))
            return rc;
        // The host waits for the summary word itself, the kernel's last write, not for the stream
        // (0.0579 vs 0.0636 ms per rotated 1M x 180 B call, profiles/r06_replay_uniform_stride_ab.txt):
        // every read of the image is done by then, and later work on the stream is ordered after the
        // kernel anyway.  The stream sync follows only if the word never comes (a fault: its error).
        // (tools build: KARMA_WAL_SPEC_POLL=0 syncs the stream instead)
        bool seen = false;
        if (KARMA_AB_KNOB("KARMA_WAL_SPEC_POLL", 1)) {
            const auto t0 = std::chrono::steady_clock::now();
            while (!(seen = __atomic_load_n(&S->spec, __ATOMIC_ACQUIRE) != 0) &&
                   std::chrono::steady_clock::now() - t0 < std::chrono::milliseconds(50)) {
            }
        }
        if (!seen && hipStreamSynchronize(c.st) != hipSuccess) return fail(KARMA_E_HIP, "wal_replay: uniform-stride pass");
        T.mark("uniform-stride pass (device)");
#ifdef KARMA_AB
        g_spec_last = (int)S->spec;
#endif
        if (S->spec == 1) {
            const uint64_t accepted = S->n_all, m = S->w1, sig = (uint64_t)S->max_len + 8, f = A.first_pos;
            const uint64_t m0 = (seg_bytes - f) / sig;  // segment 0's slots, from replay's start
            c.have_len_hint = true;
            c.len_hint = S->max_len;
            c.skew_hint = S->stage_skew != 0;
            if (h_rec_off && rec_cap && accepted) {  // slot g: f + g sigma in segment 0, then m per segment
                const uint64_t k = std::min<uint64_t>(accepted, rec_cap);
                parallel_for(0, k, 1 << 16, [&](uint64_t g) {
                    h_rec_off[g] = base0 + (g < m0 ? f + g * sig : (1 + (g - m0) / m) * seg_bytes + (g - m0) % m * sig);
                });
                T.mark("offsets");
            }
            *h_n_records = accepted;
            *h_stop = S->end;
            *h_status = (int)S->status;
            return 0;
        }
        if (S->spec == 3) {  // the other kernel's size class: the next pass takes it (no skipping)
            c.have_len_hint = true;
            c.len_hint = S->max_len;
        } else {
            c.spec_skip = kSpecSkip;
        }
    }
    // 1. segment-parallel header walk (sub-range walkers when there are few segments)
    const WalWalkPlan plan =
        wal_walk_plan(seg_bytes, nwork, c.cu, tuning ? tuning->walk_sub_bytes : 0, inline_crc, list_crc);
    A.nsub = plan.nsub;
    A.sub_bytes = plan.sub_bytes;
    A.sub_cap = plan.sub_cap;
    A.cand_cap = plan.cand_cap;
    if (const int rc = c.crec.ensure(nwork * A.cand_cap * 4)) return rc;
    if (const int rc = c.clen.ensure(nwork * A.cand_cap * 4)) return rc;
    if (const int rc = c.ccrc.ensure(nwork * A.cand_cap * 4)) return rc;
    if (const int rc = c.meta.ensure(nwork * sizeof(WalSegMeta))) return rc;
    if (const int rc = c.sub.ensure(nwork * plan.nsub * sizeof(WalSubMeta))) return rc;
    if (const int rc = c.span.ensure(nwork * plan.nsub * 2 * sizeof(uint32_t))) return rc;
    if (const int rc = c.cbase.ensure(nwork * 8)) return rc;
    if (const int rc = c.sum.ensure(sizeof(WalSummary))) return rc;
    if (const int rc = c.h_small.ensure(64, true)) return rc;  // the summary readback
    A.cand_rec = c.crec.as<uint32_t>();
    A.cand_len = c.clen.as<uint32_t>();
    A.cand_crc = c.ccrc.as<uint32_t>();
    A.meta = c.meta.as<WalSegMeta>();
    A.sub = c.sub.as<WalSubMeta>();
    A.span = c.span.as<uint32_t>();
    A.cand_base = c.cbase.as<uint64_t>();
    A.sum = c.sum.as<WalSummary>();
    A.first_bad = &A.sum->first_bad;
    A.wal_end = wal_bytes;
    const uint32_t direct_max = batch == KARMA_WAL_CRC_DIRECT ? ~0u : kSmallRecordMax;  // the device-side gate
    int small_which = kSmallBoth;
    auto bind_lists = [&](uint64_t cap) {  // the contiguous lists for up to cap candidates
        if (const int rc = c.off.ensure(cap * 8)) return rc;
        if (const int rc = c.len.ensure(cap * 4)) return rc;
        if (const int rc = c.stored.ensure(cap * 4)) return rc;
        if (const int rc = c.crc.ensure(cap * 4)) return rc;
        A.off = c.off.as<uint64_t>();
        A.len = c.len.as<uint32_t>();
        A.stored = c.stored.as<uint32_t>();
        A.crc = c.crc.as<uint32_t>();
        A.n_all = cap;
        return 0;
    };
    // 2. the replay plan on the device (k_wal_plan: the segments replay enters, their list
    //    offsets, the summary).  Device-planned path, separate batch: the lists are sized for the
    //    most candidates the image can hold (a header every 8 bytes), and the gather, the
    //    small-record CRC batch and the compare are enqueued right behind the walk; the CRC
    //    kernel checks the summary itself and does nothing when a payload is over 1 KiB.  Inline
    //    CRCs: the plan also finds the first mismatch the walkers reported.  One host round trip
    //    then reads the summary; only WALs with larger records (or, inline, a run the walkers
    //    could not checksum) need a second one (the ragged plan is sized on the host).
    const uint64_t cap_all = img_bytes / 8 + nwork;
    // (up to 1024 segments the device-planned gather reduces the metas itself: no plan launch)
    const bool fused_plan = dev_plan && !inline_crc && nwork <= 1024;
    // the resolve and the fused-plan gather in one launch (k_wal_resolve_gather: 0.1084 vs 0.1106 ms
    // per rotated 1M x 180 B call, profiles/r06_replay_rg_ab.txt); the tools build's KARMA_WAL_RG=0
    // keeps round 5's two launches for A/B
    const bool rg = fused_plan && plan.nsub > 1 && plan.nsub <= kMaxSub && KARMA_AB_KNOB("KARMA_WAL_RG", 1) != 0;
    if (rg) {
        constexpr size_t kRgBytes = 2 * 1024 * sizeof(unsigned long long);
        if (const int rc = c.rgw.ensure(kRgBytes)) return rc;
        if (++c.rg_seq >= (1u << 16)) c.rg_seq = 1;
        if (c.rgw.p != c.rgw_zeroed || c.rg_seq == 1) {
            if (hipMemsetAsync(c.rgw.p, 0, kRgBytes, c.st) != hipSuccess)
                return fail(KARMA_E_HIP, "wal_replay: hipMemsetAsync");
            c.rgw_zeroed = c.rgw.p;
        }
        A.rg_words = c.rgw.as<unsigned long long>();
        A.rg_tag = c.rg_seq;
    }
    if (launch_wal_walk(A, nwork, plan, c.st, !rg) != hipSuccess ||
        (!fused_plan && launch_wal_plan(A, nwork, c.st) != hipSuccess))
        return fail(KARMA_E_HIP, "wal_replay: header walk");
    if (dev_plan && !inline_crc) {
        if (const int rc = bind_lists(cap_all)) return rc;
        if ((rg ? launch_wal_resolve_gather(A, nwork, c.st) : launch_wal_gather(A, nwork, fused_plan, c.cu, c.st)) !=
            hipSuccess)
            return fail(KARMA_E_HIP, "wal_replay: gather");
        // the CRC batch is also the check (first mismatch into the summary): no compare launch.
        // Which kernel covers the largest payload is known on the device only; the last pass's
        // largest payload picks one launch (the other one, gated off, cost ~5 us), and a pass
        // whose records it did not cover runs the batch again below (one more round trip).
        small_which = !c.have_len_hint ? kSmallBoth : c.len_hint <= kStgGateLen ? kSmallStaged : kSmallDirect;
        if (const long w = KARMA_AB_KNOB("KARMA_SMALL_WHICH", -1); w >= 0 && w <= 2) small_which = (int)w;  // (A/B)
        const long skew_knob = KARMA_AB_KNOB("KARMA_STAGE_SKEW", -1);  // (A/B: 0 plain, 1 skewed stage)
        if (const int rc = ragged_small_batch_dev(A.wal + 8, A.off, A.len, &A.sum->n_all, cap_all, &A.sum->max_len,
                                                  direct_max, c.crc.as<uint32_t>(), A.stored, A.first_bad, c.st,
                                                  small_which, skew_knob >= 0 ? skew_knob != 0 : c.skew_hint,
                                                  &A.sum->stage_skew))
            return rc;
    }
    WalSummary* S = c.h_small.as<WalSummary>();  // (page-locked: the device writes it, launch_wal_publish)
    if (launch_wal_publish(A.sum, S, c.st) != hipSuccess || hipStreamSynchronize(c.st) != hipSuccess)
        return fail(KARMA_E_HIP, "wal_replay: walk + plan");
    T.mark(inline_crc ? "walk + inline CRCs + plan (device)"
                      : dev_plan ? "walk + plan + gather + CRCs (device)" : "walk + plan (device)");
    // replay enters segment s+1 only if segment s ended cleanly (k_wal_plan)
    int status = (int)S->status;
    uint64_t end = S->end;
    const uint64_t w1 = S->w1, n_all = S->n_all;
    const uint32_t max_len = S->max_len;
    const bool small = batch == KARMA_WAL_CRC_DIRECT ||
                       ((batch == KARMA_WAL_CRC_PLAN || batch == KARMA_WAL_CRC_SEPARATE || batch == KARMA_WAL_CRC_INLINE) &&
                        max_len <= kSmallRecordMax);
    // inline CRCs complete: the first mismatch is known (no gathered lists exist yet)
    const bool inline_done = inline_crc && !S->crc_unknown;
    const bool lists = dev_plan && !inline_crc;  // the device-planned gather wrote them
    // the device-sized batch ran and covered every payload
    const bool batch_done = lists && small && small_batch_covers(small_which, max_len, direct_max);
    if (lists && n_all) {
        c.have_len_hint = true;
        c.len_hint = max_len;
        if (small_which != kSmallDirect && max_len <= kStgGateLen) c.skew_hint = S->stage_skew != 0;
    }
    uint64_t accepted = n_all;
    if (inline_done && S->first_bad < n_all) {
        accepted = S->first_bad;
        status = KARMA_WAL_CORRUPT;
        end = base0 + S->bad_off;
    }
    if (n_all && !inline_done && !batch_done) {
        // 3. the host-sized CRC batch: large payloads (the ragged plan), an image too large for
        //    the device-planned lists, runs the inline walk could not checksum, or payloads the
        //    one small-record kernel launched above did not cover
        if (!lists) {
            if (const int rc = bind_lists(n_all)) return rc;
            if (launch_wal_gather(A, nwork, false, c.cu, c.st) != hipSuccess)
                return fail(KARMA_E_HIP, "wal_replay: gather");
        }
        // payload = header + 8: the arena is the image shifted by the header
        if (const int rc = small ? ragged_small_batch(A.wal + 8, A.off, A.len, n_all, c.crc.as<uint32_t>(), c.st)
                                 : karma_crc32c_batch_ragged(A.wal + 8, A.off, A.len, n_all, w1 * seg_bytes, nullptr,
                                                             0, c.crc.as<uint32_t>(), c.st))
            return rc;
        if (launch_wal_compare(A, n_all, c.cu, c.st) != hipSuccess ||
            hipMemcpyAsync(&S->first_bad, A.first_bad, 8, hipMemcpyDeviceToHost, c.st) != hipSuccess ||
            hipStreamSynchronize(c.st) != hipSuccess)
            return fail(KARMA_E_HIP, "wal_replay: CRC check");
        T.mark("CRC batch + compare");
    }
    if (n_all) {
        if (!inline_done && S->first_bad < n_all) {  // the first mismatch in WAL order: "Corrupt record"
            accepted = S->first_bad;
            status = KARMA_WAL_CORRUPT;
            uint64_t at = 0;
            if (hipMemcpyAsync(&at, A.off + accepted, 8, hipMemcpyDeviceToHost, c.st) != hipSuccess ||
                hipStreamSynchronize(c.st) != hipSuccess)
                return fail(KARMA_E_HIP, "wal_replay: D2H");
            end = base0 + at;
        }
        if (h_rec_off && rec_cap && accepted && inline_done) {  // the offsets: the lists are gathered now
            if (const int rc = bind_lists(n_all)) return rc;
            if (launch_wal_gather(A, nwork, false, c.cu, c.st) != hipSuccess)
                return fail(KARMA_E_HIP, "wal_replay: gather");
        }
        if (h_rec_off && rec_cap && accepted) {
            const uint64_t k = std::min<uint64_t>(accepted, rec_cap);
            // (on the replay's stream: it is non-blocking, so a legacy-stream copy would not wait
            // for the gather just enqueued there)
            if (hipMemcpyAsync(h_rec_off, A.off, k * 8, hipMemcpyDeviceToHost, c.st) != hipSuccess ||
                hipStreamSynchronize(c.st) != hipSuccess)
                return fail(KARMA_E_HIP, "wal_replay: D2H offsets");
            parallel_for(0, k, 1 << 16, [&](uint64_t i) { h_rec_off[i] += base0; });
        }
        T.mark("offsets");
    }
    *h_n_records = accepted;
    *h_stop = end;
    *h_status = status;
    return 0;
}

}  // namespace


extern "C" {

int karma_wal_replay_dir(const char* dir, size_t seg_bytes, uint64_t start, uint64_t* h_base, uint64_t* h_n_records,
                         uint64_t* h_stop, int* h_status, uint64_t* h_rec_off, size_t rec_cap, int device) {
    if (!dir || !h_base || !h_n_records || !h_stop || !h_status) return fail(KARMA_E_INVALID, "wal_replay_dir");
    // wal::load_from_path (wal.cc:9-27): the regular files of the directory, each named by
    // the decimal WAL offset of its first byte, in offset order
    struct Seg {
        uint64_t off, size;
        std::string path;
    };
    std::vector<Seg> segs;
    DIR* d = opendir(dir);
    if (!d) return fail(KARMA_E_IO, std::string("wal_replay_dir: cannot open ") + dir);
    while (const dirent* e = readdir(d)) {
        const std::string name = e->d_name;
        if (name.empty() || name.find_first_not_of("0123456789") != std::string::npos) continue;
        const std::string path = std::string(dir) + "/" + name;
        struct stat st;
        if (stat(path.c_str(), &st) != 0 || !S_ISREG(st.st_mode)) continue;
        segs.push_back(Seg{std::strtoull(name.c_str(), nullptr, 10), (uint64_t)st.st_size, path});
    }
    closedir(d);
    std::sort(segs.begin(), segs.end(), [](const Seg& a, const Seg& b) { return a.off < b.off; });
    if (segs.empty()) {
        *h_base = 0;
        *h_n_records = 0;
        *h_stop = start;
        *h_status = KARMA_WAL_END;
        return 0;
    }
    if (!seg_bytes) seg_bytes = segs[0].size;
    const uint64_t base = segs[0].off;
    for (size_t i = 0; i < segs.size(); ++i)  // one image: equal sizes, no gaps
        if (segs[i].size != seg_bytes || segs[i].off != base + i * seg_bytes)
            return fail(KARMA_E_INVALID, "wal_replay_dir: segment files must have equal sizes and no gaps: " +
                                             segs[i].path);
    const uint64_t wal_bytes = segs.size() * seg_bytes;
    if (start < base || start > base + wal_bytes || seg_bytes >= (uint64_t(1) << 31))
        return fail(KARMA_E_INVALID, "wal_replay_dir: start outside the segments");
    std::vector<int> fds(segs.size(), -1);
    auto close_all = [&] {
        for (int fd : fds)
            if (fd >= 0) ::close(fd);
    };
    for (size_t i = 0; i < segs.size(); ++i)
        if ((fds[i] = ::open(segs[i].path.c_str(), O_RDONLY)) < 0) {
            close_all();
            return fail(KARMA_E_IO, "wal_replay_dir: cannot open " + segs[i].path);
        }
    // the staging threads read the files straight into the pinned buffers
    const ImageFill read_files = [&](uint8_t* dst, uint64_t off, size_t n) {
        while (n) {
            const uint64_t f = off / seg_bytes, in = off - f * seg_bytes;
            const size_t take = std::min<uint64_t>(n, seg_bytes - in);
            size_t got = 0;
            while (got < take) {
                const ssize_t r = ::pread(fds[f], dst + got, take - got, (off_t)(in + got));
                if (r <= 0) return fail(KARMA_E_IO, "wal_replay_dir: short read of " + segs[f].path);
                got += (size_t)r;
            }
            dst += take;
            off += take;
            n -= take;
        }
        return 0;
    };
    const int rc = replay_core(nullptr, &read_files, wal_bytes, seg_bytes, start - base, h_n_records, h_stop, h_status,
                               h_rec_off, rec_cap, device, nullptr);
    close_all();
    if (rc) return rc;
    *h_base = base;
    *h_stop += base;
    if (h_rec_off) {
        const uint64_t k = std::min<uint64_t>(*h_n_records, rec_cap);
        for (uint64_t i = 0; i < k; ++i) h_rec_off[i] += base;
    }
    return 0;
}

}  // extern "C"
