// karma_amd/csrc/wal_append.cc -- batched WAL append:
// sivir::build_sqe's loop (sivir.cc:276-317) over segment_file::append_record /
// append_footer (segment_file.cc:21-49), with the payload CRCs of the whole batch
// computed on the GPU.
//
// Record format (segment_file.cc:21-31, common.h:11):
//   [crc u32 LE = Value(payload)][len << 8 | type u32 LE][payload]
// type 1 pads to the segment end with '0' bytes and crc field 0 (:33-49); a
// segment tail shorter than a header is '0' bytes only (:34-39).
//
// The path is PCIe-bound (the payloads start in host memory), so every stage is
// overlapped with the upload, on the library's persistent host threads (run_pool):
//   1. placement (thread 0, sequential: can_hold, else footer + next segment),
//      published in blocks of records (small blocks first, so the pipeline fills fast);
//   2. framing workers take the blocks as they are published (a condition variable,
//      no spinning: the box's CPU quota is shared by every thread): each writes its
//      records' length fields and payloads into the WAL image AND packs the payloads
//      into the library's pinned staging (one copy when the block's payloads are
//      contiguous in the source), then enqueues the block's DMA, its CRC batch (one
//      record per group of 8 lanes when every payload <= 1 KiB) and the D2H of its
//      CRCs on one of 8 streams, and records the block's event;
//   3. when no block is left to frame, the threads write the CRC fields block by
//      block as each block's event completes, while later blocks are still in flight.
// Nothing is page-locked per call: the staging is pinned once and grows.
#include <hip/hip_runtime_api.h>

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <cstring>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "engine.h"
#include "host_stage.h"
#include "host_trace.h"
#include "karma_crc32c.h"
#include "wal_place.h"

namespace karma::engine {
int set_last_error(int code, const std::string& what);  // capi.cc
}

namespace {

using karma::engine::set_last_error;

constexpr uint64_t kHeader = karma::engine::kWalHeader;  // store::RECORD_HEADER_LENGTH (common.h:11)
constexpr size_t kBlockRecords = 16384;              // a published block: at most this many records
constexpr uint64_t kBlockBytesFirst = uint64_t(256) << 10;  // payload bytes of the first block,
constexpr uint64_t kBlockBytesMax = uint64_t(4) << 20;      // doubling up to this
constexpr uint64_t kCallBytes = uint64_t(1) << 30;   // payload bytes staged per pass (larger batches loop)
constexpr int kStreams = 8;                          // DMA / CRC streams the blocks rotate over

inline void put32(uint8_t* p, uint32_t v) { std::memcpy(p, &v, 4); }  // little-endian host

struct Buf {
    void* p = nullptr;
    size_t bytes = 0;
    bool host = false;
    int ensure(size_t want, bool pinned_host) {
        if (p && bytes >= want) return 0;
        if (p) (void)(host ? hipHostFree(p) : hipFree(p));
        p = nullptr;
        bytes = 0;
        want = std::max<size_t>(want + want / 8, 4096);
        const hipError_t e = pinned_host ? hipHostMalloc(&p, want, hipHostMallocDefault) : hipMalloc(&p, want);
        if (e != hipSuccess) {
            p = nullptr;
            return set_last_error(e == hipErrorOutOfMemory ? KARMA_E_NOMEM : KARMA_E_HIP, "wal_append: allocation");
        }
        bytes = want;
        host = pinned_host;
        return 0;
    }
    template <typename T>
    T* as() const {
        return static_cast<T*>(p);
    }
};

// Per-device append context: the streams, one event per block, the grow-only staging
// (pinned) and device copies of the packed payloads, their offsets, lengths and CRCs,
// and the host placement arrays (kept: a fresh 8 MiB vector costs its page faults).
struct AppendCtx {
    std::mutex mu;
    bool ready = false;
    hipStream_t st[kStreams] = {};
    std::vector<hipEvent_t> ev;
    Buf h_pay, h_off, h_len, h_crc;  // pinned
    Buf d_pay, d_off, d_len, d_crc;  // device
    std::vector<uint64_t> at;
    std::vector<size_t> bstart;
    int init() {
        if (ready) return 0;
        for (auto& s : st)
            if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess)
                return set_last_error(KARMA_E_HIP, "wal_append: stream");
        ready = true;
        return 0;
    }
    int events(size_t n) {
        while (ev.size() < n) {
            hipEvent_t e;
            if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess)
                return set_last_error(KARMA_E_HIP, "wal_append: event");
            ev.push_back(e);
        }
        return 0;
    }
};

std::mutex g_mu;
std::vector<std::unique_ptr<AppendCtx>> g_ctx;

AppendCtx& ctx_for(int dev) {
    std::lock_guard<std::mutex> g(g_mu);
    if ((int)g_ctx.size() <= dev) g_ctx.resize(dev + 1);
    if (!g_ctx[dev]) g_ctx[dev] = std::make_unique<AppendCtx>();
    return *g_ctx[dev];
}

// One pass over records [0, n) of the caller's arrays (payload total pay_total <= kCallBytes,
// or a single record): frames what fits from *cursor, returns the number framed.
int append_pass(AppendCtx& C, int dev, const uint8_t* src, const uint64_t* src_off, const uint32_t* len, size_t n,
                uint64_t pay_total, uint32_t max_len, uint8_t* wal, size_t wal_bytes, size_t seg_bytes,
                uint64_t* cursor, uint64_t* rec_off, size_t* n_framed) {
    karma::engine::PhaseTimer T("wal_append");
    // blocks: at most n / kBlockRecords + (payload / smallest block) + the doubling steps
    const size_t max_blocks = n / kBlockRecords + pay_total / kBlockBytesFirst + 32;
    if (const int rc = C.h_pay.ensure(pay_total + 16, true)) return rc;
    if (const int rc = C.d_pay.ensure(pay_total + 16, false)) return rc;
    if (const int rc = C.h_off.ensure(n * 8, true)) return rc;
    if (const int rc = C.d_off.ensure(n * 8, false)) return rc;
    if (const int rc = C.h_len.ensure(n * 4, true)) return rc;
    if (const int rc = C.d_len.ensure(n * 4, false)) return rc;
    if (const int rc = C.h_crc.ensure(n * 4, true)) return rc;
    if (const int rc = C.d_crc.ensure(n * 4, false)) return rc;
    if (const int rc = C.events(max_blocks)) return rc;
    if (C.at.size() < n) C.at.resize(n);
    if (C.bstart.size() < max_blocks + 2) C.bstart.resize(max_blocks + 2);
    T.mark("buffers");
    uint8_t* hp = C.h_pay.as<uint8_t>();
    uint64_t* ho = C.h_off.as<uint64_t>();
    uint32_t* hl = C.h_len.as<uint32_t>();
    uint32_t* hc = C.h_crc.as<uint32_t>();
    uint64_t* at = C.at.data();
    size_t* bstart = C.bstart.data();
    bstart[0] = 0;

    std::mutex mu;
    std::condition_variable cv;
    size_t published = 0;  // blocks whose end is known (bstart[k + 1] valid); under mu
    bool placing = true;   // under mu
    int framing = 0;       // threads still in stage 2; under mu
    std::atomic<size_t> next_block{0}, next_fill{0};
    std::atomic<int> crc_rc{0};
    size_t framed = 0;
    uint64_t end_cursor = *cursor;
    // Thread 0 places and then helps; every thread frames blocks while any are left, then
    // writes CRC fields of completed blocks.  Returns only when its own work is done.
    auto frame_block = [&](size_t k) {
        const size_t lo = bstart[k], hi = bstart[k + 1];
        bool contiguous = true;
        for (size_t i = lo; i < hi; ++i) {  // segment_file::append_record: length field + payload
            uint8_t* p = wal + at[i];
            const uint32_t L = len[i];
            put32(p + 4, L << 8 | 0u);
            std::memcpy(p + kHeader, src + src_off[i], L);
            hl[i] = L;
            if (i > lo && src_off[i] != src_off[i - 1] + len[i - 1]) contiguous = false;
        }
        const uint64_t plo = ho[lo], phi = ho[hi - 1] + hl[hi - 1];
        if (contiguous) {
            std::memcpy(hp + plo, src + src_off[lo], phi - plo);
        } else {
            for (size_t i = lo; i < hi; ++i) std::memcpy(hp + ho[i], wal + at[i] + kHeader, hl[i]);  // from cache
        }
        for (size_t i = lo; i < hi; ++i) ho[i] -= plo;  // the block's kernel sees its own slice
        hipStream_t s = C.st[k % kStreams];
        const size_t nr = hi - lo;
        uint8_t* dp = C.d_pay.as<uint8_t>();
        uint64_t* doff = C.d_off.as<uint64_t>() + lo;
        uint32_t* dlen = C.d_len.as<uint32_t>() + lo;
        if (hipMemcpyAsync(dp + plo, hp + plo, phi - plo, hipMemcpyHostToDevice, s) != hipSuccess ||
            hipMemcpyAsync(doff, ho + lo, nr * 8, hipMemcpyHostToDevice, s) != hipSuccess ||
            hipMemcpyAsync(dlen, hl + lo, nr * 4, hipMemcpyHostToDevice, s) != hipSuccess)
            return KARMA_E_HIP;
        if (const int rc = karma_crc32c_batch_ragged_bounded(dp + plo, doff, dlen, nr, phi - plo, max_len, nullptr, 0,
                                                             C.d_crc.as<uint32_t>() + lo, s))
            return rc;
        if (hipMemcpyAsync(hc + lo, C.d_crc.as<uint32_t>() + lo, nr * 4, hipMemcpyDeviceToHost, s) != hipSuccess ||
            hipEventRecord(C.ev[k], s) != hipSuccess)
            return KARMA_E_HIP;
        return 0;
    };
    auto worker = [&](int t) {
        if (t > 0 && hipSetDevice(dev) != hipSuccess) {  // thread 0 is the caller's (device set)
            int zero = 0;
            crc_rc.compare_exchange_strong(zero, (int)KARMA_E_HIP);
        }
        if (t == 0) {  // 1. placement (sivir::build_sqe's loop), published block by block
            karma::engine::WalPlacer place(seg_bytes, wal_bytes, *cursor);
            std::vector<std::pair<uint64_t, uint64_t>> footers;  // (wal offset, segment end)
            size_t nb = 0, f = 0;
            uint64_t packed = 0, bbytes = 0, blimit = kBlockBytesFirst;
            for (; f < n; ++f) {
                const uint64_t L = len[f];
                uint64_t f0, f1;
                const bool ok = place.place(L, &at[f], &f0, &f1);
                if (f1 > f0) footers.emplace_back(f0, f1);
                if (!ok) break;
                ho[f] = packed;
                packed += L;
                bbytes += L;
                if (f + 1 - bstart[nb] == kBlockRecords || bbytes >= blimit) {
                    std::lock_guard<std::mutex> lk(mu);
                    bstart[++nb] = f + 1;
                    published = nb;
                    bbytes = 0;
                    blimit = std::min(2 * blimit, kBlockBytesMax);
                    cv.notify_all();
                }
            }
            {
                std::lock_guard<std::mutex> lk(mu);
                if (bstart[nb] < f) bstart[++nb] = f;
                published = nb;
                placing = false;
                framed = f;
                end_cursor = place.cur;
            }
            cv.notify_all();
            for (const auto& fp : footers) {  // segment_file::append_footer
                const uint64_t room = fp.second - fp.first;
                if (room < kHeader) {
                    std::memset(wal + fp.first, '0', room);
                } else {
                    put32(wal + fp.first, 0);
                    put32(wal + fp.first + 4, uint32_t((room - kHeader) << 8 | 1u));
                    std::memset(wal + fp.first + kHeader, '0', room - kHeader);
                }
            }
        }
        // 2. framing, DMA and CRC batches, block by block
        while (!crc_rc.load(std::memory_order_relaxed)) {
            const size_t k = next_block.fetch_add(1);
            {
                std::unique_lock<std::mutex> lk(mu);
                cv.wait(lk, [&] { return published > k || !placing; });
                if (k >= published) break;  // placement ended before this block
            }
            if (const int rc = frame_block(k)) {
                int zero = 0;
                crc_rc.compare_exchange_strong(zero, rc);
                break;
            }
        }
        // 3. CRC fields of the blocks in order, each once its event has completed.  Every
        // block must have been enqueued first (an event never recorded in this call would
        // not wait), so the threads meet here; the DMAs and kernels are still in flight.
        size_t nb;
        {
            std::unique_lock<std::mutex> lk(mu);
            if (--framing == 0) cv.notify_all();
            cv.wait(lk, [&] { return framing == 0; });
            nb = published;
        }
        while (!crc_rc.load(std::memory_order_relaxed)) {
            const size_t k = next_fill.fetch_add(1);
            if (k >= nb) break;
            if (hipEventSynchronize(C.ev[k]) != hipSuccess) {
                int zero = 0;
                crc_rc.compare_exchange_strong(zero, (int)KARMA_E_HIP);
                break;
            }
            for (size_t i = bstart[k]; i < bstart[k + 1]; ++i) put32(wal + at[i], hc[i]);
        }
    };
    const int nthr = (int)std::min<size_t>(karma::engine::kPoolThreads + 1, std::max<size_t>(1, n / 1024));
    framing = nthr;
    karma::engine::run_pool(nthr, worker);
    T.mark("placement + framing + CRCs");
    for (auto& s : C.st)  // nothing of this call may be in flight when it returns
        if (hipStreamSynchronize(s) != hipSuccess && !crc_rc) crc_rc = KARMA_E_HIP;
    if (const int rc = crc_rc.load())  // payloads and length fields are written; CRC fields may not be
        return rc == KARMA_E_HIP ? set_last_error(rc, "wal_append: device pipeline") : rc;
    if (rec_off) std::memcpy(rec_off, at, framed * sizeof(uint64_t));
    *cursor = end_cursor;
    *n_framed = framed;
    return 0;
}

}  // namespace

extern "C" int karma_wal_append_batch(const void* h_src, const uint64_t* h_src_off, const uint32_t* h_len, size_t n,
                                      void* h_wal, size_t wal_bytes, size_t seg_bytes, uint64_t* h_cursor,
                                      uint64_t* h_rec_off, size_t* h_n_framed, int device) {
    if (!h_cursor || !h_n_framed || (n && (!h_src || !h_src_off || !h_len)) || !h_wal || seg_bytes < kHeader ||
        wal_bytes % seg_bytes)
        return set_last_error(KARMA_E_INVALID, "wal_append_batch");
    *h_n_framed = 0;
    if (!n) return 0;
    int nd = 0, dev = 0;
    if (hipGetDeviceCount(&nd) != hipSuccess || nd <= 0) return set_last_error(KARMA_E_NO_DEVICE, "no HIP device visible");
    if (device >= nd) return set_last_error(KARMA_E_INVALID, "wal_append: device index out of range");
    if (device >= 0 && hipSetDevice(device) != hipSuccess) return set_last_error(KARMA_E_HIP, "hipSetDevice");
    if (hipGetDevice(&dev) != hipSuccess) return set_last_error(KARMA_E_HIP, "hipGetDevice");
    AppendCtx& C = ctx_for(dev);
    std::lock_guard<std::mutex> lk(C.mu);
    if (const int rc = C.init()) return rc;
    const uint8_t* src = static_cast<const uint8_t*>(h_src);
    uint8_t* wal = static_cast<uint8_t*>(h_wal);
    uint64_t cur = *h_cursor;
    size_t done = 0;
    while (done < n) {  // passes of at most kCallBytes of payload (at least one record)
        size_t m = 1;
        uint64_t bytes = h_len[done];
        uint32_t max_len = h_len[done];
        for (; done + m < n && bytes + h_len[done + m] <= kCallBytes; ++m) {
            bytes += h_len[done + m];
            max_len = std::max(max_len, h_len[done + m]);
        }
        size_t framed = 0;
        if (const int rc = append_pass(C, dev, src, h_src_off + done, h_len + done, m, bytes, max_len, wal, wal_bytes,
                                       seg_bytes, &cur, h_rec_off ? h_rec_off + done : nullptr, &framed))
            return rc;  // *h_cursor and *h_n_framed keep the passes already complete
        done += framed;
        *h_cursor = cur;
        *h_n_framed = done;
        if (framed < m) break;  // the image is full (or a record can never fit)
    }
    return 0;
}
