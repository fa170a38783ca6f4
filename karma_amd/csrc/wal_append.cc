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
// overlapped with the upload:
//   1. placement (sequential: can_hold, else footer + next segment), published
//      in blocks of records;
//   2. framing workers take the blocks as they are published: each writes its
//      records' length fields and payloads into the WAL image AND copies the
//      payloads, packed, into the library's pinned staging (the source bytes are
//      read once, the second copy comes from cache), then DMAs the block on its
//      stream and runs the block's CRC batch (one record per group of 8 lanes
//      when every payload <= 1 KiB) and the D2H of its CRCs there;
//   3. the CRC fields are written when every block's stream has drained.
// Nothing is page-locked per call: the staging is pinned once and grows.
#include <hip/hip_runtime_api.h>

#include <algorithm>
#include <atomic>
#include <cstring>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
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
constexpr size_t kBlockRecords = 16384;          // a published block: at most this many records
constexpr uint64_t kBlockBytes = uint64_t(4) << 20;  // ... or about this many payload bytes
constexpr uint64_t kCallBytes = uint64_t(1) << 30;   // payload bytes staged per pass (larger batches loop)
constexpr int kStreams = 8;                      // DMA / CRC streams the blocks rotate over
constexpr int kMaxWorkers = 15;                  // framing workers (+ the placing thread)

inline void put32(uint8_t* p, uint32_t v) {
    p[0] = uint8_t(v);
    p[1] = uint8_t(v >> 8);
    p[2] = uint8_t(v >> 16);
    p[3] = uint8_t(v >> 24);
}

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

// Per-device append context: the streams and the grow-only staging (pinned) and
// device copies of the packed payloads, their offsets, lengths and CRCs.
struct AppendCtx {
    std::mutex mu;
    bool ready = false;
    hipStream_t st[kStreams] = {};
    Buf h_pay, h_off, h_len, h_crc;  // pinned
    Buf d_pay, d_off, d_len, d_crc;  // device
    int init() {
        if (ready) return 0;
        for (auto& s : st)
            if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess)
                return set_last_error(KARMA_E_HIP, "wal_append: stream");
        ready = true;
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

// One pass over records [0, n) of the caller's arrays (payload total <= kCallBytes, or a
// single record): frames what fits from *cursor, returns the number framed.
int append_pass(AppendCtx& C, int dev, const uint8_t* src, const uint64_t* src_off, const uint32_t* len, size_t n,
                uint8_t* wal, size_t wal_bytes, size_t seg_bytes, uint64_t* cursor, uint64_t* rec_off,
                size_t* n_framed) {
    karma::engine::PhaseTimer T("wal_append");
    uint64_t pay_total = 0;
    uint32_t max_len = 0;
    for (size_t i = 0; i < n; ++i) {
        pay_total += len[i];
        max_len = std::max(max_len, len[i]);
    }
    if (const int rc = C.h_pay.ensure(pay_total + 16, true)) return rc;
    if (const int rc = C.d_pay.ensure(pay_total + 16, false)) return rc;
    if (const int rc = C.h_off.ensure(n * 8, true)) return rc;
    if (const int rc = C.d_off.ensure(n * 8, false)) return rc;
    if (const int rc = C.h_len.ensure(n * 4, true)) return rc;
    if (const int rc = C.d_len.ensure(n * 4, false)) return rc;
    if (const int rc = C.h_crc.ensure(n * 4, true)) return rc;
    if (const int rc = C.d_crc.ensure(n * 4, false)) return rc;
    T.mark("sizes + buffers");
    uint8_t* hp = C.h_pay.as<uint8_t>();
    uint64_t* ho = C.h_off.as<uint64_t>();
    uint32_t* hl = C.h_len.as<uint32_t>();
    uint32_t* hc = C.h_crc.as<uint32_t>();

    // 1. placement, published block by block: bstart[k] = first record of block k
    std::vector<uint64_t> at(n);
    std::vector<size_t> bstart(n + 2, 0);
    std::atomic<size_t> published{0};  // blocks whose end is known (bstart[k + 1] valid)
    std::atomic<bool> placing{true};
    std::atomic<size_t> next_block{0};
    std::atomic<int> crc_rc{0};
    const int nwork = (int)std::min<size_t>(kMaxWorkers, std::max<size_t>(1, n / 2048));
    std::vector<std::thread> workers;
    for (int t = 0; t < nwork; ++t)
        workers.emplace_back([&] {
            if (hipSetDevice(dev) != hipSuccess) {
                crc_rc = KARMA_E_HIP;
                return;
            }
            while (true) {
                const size_t k = next_block.fetch_add(1);
                size_t pub;
                while ((pub = published.load(std::memory_order_acquire)) <= k && placing.load(std::memory_order_acquire))
                    std::this_thread::yield();
                pub = published.load(std::memory_order_acquire);
                if (k >= pub) return;  // placement ended before this block
                const size_t lo = bstart[k], hi = bstart[k + 1];
                // 2. frame (segment_file::append_record) and pack the payloads for the device
                for (size_t i = lo; i < hi; ++i) {
                    uint8_t* p = wal + at[i];
                    const uint32_t L = len[i];
                    put32(p + 4, L << 8 | 0u);
                    std::memcpy(p + kHeader, src + src_off[i], L);
                    std::memcpy(hp + ho[i], p + kHeader, L);  // from cache
                    hl[i] = L;
                }
                const uint64_t plo = ho[lo], phi = ho[hi - 1] + hl[hi - 1];
                hipStream_t s = C.st[k % kStreams];
                const size_t nr = hi - lo;
                uint8_t* dp = C.d_pay.as<uint8_t>();
                uint64_t* doff = C.d_off.as<uint64_t>() + lo;
                for (size_t i = lo; i < hi; ++i) ho[i] -= plo;  // the block's kernel sees its own slice
                if (hipMemcpyAsync(dp + plo, hp + plo, phi - plo, hipMemcpyHostToDevice, s) != hipSuccess ||
                    hipMemcpyAsync(doff, ho + lo, nr * 8, hipMemcpyHostToDevice, s) != hipSuccess ||
                    hipMemcpyAsync(C.d_len.as<uint32_t>() + lo, hl + lo, nr * 4, hipMemcpyHostToDevice, s) !=
                        hipSuccess) {
                    crc_rc = KARMA_E_HIP;
                    return;
                }
                if (const int rc = karma_crc32c_batch_ragged_bounded(dp + plo, doff, C.d_len.as<uint32_t>() + lo, nr,
                                                                     phi - plo, max_len, nullptr, 0,
                                                                     C.d_crc.as<uint32_t>() + lo, s)) {
                    crc_rc = rc;
                    return;
                }
                if (hipMemcpyAsync(hc + lo, C.d_crc.as<uint32_t>() + lo, nr * 4, hipMemcpyDeviceToHost, s) !=
                    hipSuccess) {
                    crc_rc = KARMA_E_HIP;
                    return;
                }
            }
        });
    karma::engine::WalPlacer place(seg_bytes, wal_bytes, *cursor);
    size_t framed = 0, nb = 0;
    uint64_t packed = 0, bbytes = 0;
    std::vector<std::pair<uint64_t, uint64_t>> footers;  // (wal offset, segment end)
    for (; framed < n; ++framed) {
        const uint64_t L = len[framed];
        uint64_t f0, f1;
        const bool ok = place.place(L, &at[framed], &f0, &f1);
        if (f1 > f0) footers.emplace_back(f0, f1);
        if (!ok) break;
        ho[framed] = packed;
        packed += L;
        bbytes += L;
        if (framed + 1 - bstart[nb] == kBlockRecords || bbytes >= kBlockBytes) {
            bstart[++nb] = framed + 1;
            bbytes = 0;
            published.store(nb, std::memory_order_release);
        }
    }
    if (bstart[nb] < framed) {
        bstart[++nb] = framed;
        published.store(nb, std::memory_order_release);
    }
    placing.store(false, std::memory_order_release);
    T.mark("placement");
    for (const auto& f : footers) {  // segment_file::append_footer
        const uint64_t room = f.second - f.first;
        if (room < kHeader) {
            std::memset(wal + f.first, '0', room);
        } else {
            put32(wal + f.first, 0);
            put32(wal + f.first + 4, uint32_t((room - kHeader) << 8 | 1u));
            std::memset(wal + f.first + kHeader, '0', room - kHeader);
        }
    }
    for (auto& x : workers) x.join();
    T.mark("framing + uploads enqueued");
    for (auto& s : C.st)
        if (hipStreamSynchronize(s) != hipSuccess && !crc_rc) crc_rc = KARMA_E_HIP;
    T.mark("CRC batches");
    if (const int rc = crc_rc.load()) {  // payloads and length fields are written; no CRC field is
        return rc == KARMA_E_HIP ? set_last_error(rc, "wal_append: device pipeline") : rc;
    }
    // 3. the CRC fields
    const int nthr = (int)std::min<size_t>(16, std::max<size_t>(1, framed / 65536));
    karma::engine::run_threads(nthr, [&](int t) {
        for (size_t i = framed * t / nthr; i < framed * (t + 1) / nthr; ++i) put32(wal + at[i], hc[i]);
    });
    T.mark("CRC fields");
    if (rec_off) std::memcpy(rec_off, at.data(), framed * sizeof(uint64_t));
    *cursor = place.cur;
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
        for (uint64_t bytes = h_len[done]; done + m < n && bytes + h_len[done + m] <= kCallBytes; ++m)
            bytes += h_len[done + m];
        size_t framed = 0;
        if (const int rc = append_pass(C, dev, src, h_src_off + done, h_len + done, m, wal, wal_bytes, seg_bytes, &cur,
                                       h_rec_off ? h_rec_off + done : nullptr, &framed))
            return rc;  // *h_cursor and *h_n_framed keep the passes already complete
        done += framed;
        *h_cursor = cur;
        *h_n_framed = done;
        if (framed < m) break;  // the image is full (or a record can never fit)
    }
    return 0;
}
