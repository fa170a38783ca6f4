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
//   1. a parallel prefix sum of the record sizes, cut into blocks of records (small
//      blocks first, so the pipeline fills fast), then sivir's loop in run form (one
//      binary search per segment, wal_place.h) on one thread while the others start 2.;
//   2. the threads take the blocks in turn: each packs its payloads into the library's
//      pinned staging (one copy when they are contiguous in the source) and enqueues the
//      block's DMA, its CRC batch (one record per group of 8 lanes when every payload
//      <= 1 KiB) and the D2H of its CRCs on one of 8 streams;
//   3. block by block, in order, as each block's CRCs come back: the records are written
//      into the image, CRC field, length field and payload in one pass (between blocks
//      of 2., and the rest once every block is enqueued).
// No thread spins (the box's CPU quota is shared by every thread of the process).
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

#include "ab.h"
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
constexpr uint32_t kZeroCopyMaxLen = 1024;           // the bounded ABI's one-record-per-group limit (capi.cc)

inline void put32(uint8_t* p, uint32_t v) { std::memcpy(p, &v, 4); }  // little-endian host

// One record's payload: 16-byte moves (the last one overlapping) for the small records of a
// log; a library call per 180-byte record cost about as much as the copy itself.
inline void copy_payload(uint8_t* d, const uint8_t* s, size_t L) {
    if (L < 16 || L > 1024) {
        std::memcpy(d, s, L);
        return;
    }
    size_t k = 0;
    for (; k + 16 <= L; k += 16) std::memcpy(d + k, s + k, 16);
    if (k < L) std::memcpy(d + L - 16, s + L - 16, 16);
}

struct Buf {
    void* p = nullptr;
    size_t bytes = 0;
    bool host = false;
    // pinned_host: page-locked host memory; coherent: fine-grained (the GPU reads and writes it
    // over PCIe uncached, so a kernel sees what the host wrote just before the launch)
    int ensure(size_t want, bool pinned_host, bool coherent = false) {
        if (p && bytes >= want) return 0;
        if (p) (void)(host ? hipHostFree(p) : hipFree(p));
        p = nullptr;
        bytes = 0;
        want = std::max<size_t>(want + want / 8, 4096);
        const hipError_t e = pinned_host ? hipHostMalloc(&p, want, coherent ? hipHostMallocCoherent : hipHostMallocDefault)
                                         : hipMalloc(&p, want);
        if (e != hipSuccess) {
            p = nullptr;
            return set_last_error(e == hipErrorOutOfMemory ? KARMA_E_NOMEM : KARMA_E_HIP, "wal_append: allocation");
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
    void reset(int dev) {  // karma_crc32c_trim (the caller holds mu)
        if (!ready) return;
        for (auto& s : st) {
            (void)hipStreamSynchronize(s);
            (void)karma::engine::release_internal_stream(dev, s);
            (void)hipStreamDestroy(s);
            s = nullptr;
        }
        for (hipEvent_t e : ev) (void)hipEventDestroy(e);
        ev.clear();
        for (Buf* b : {&h_pay, &h_off, &h_len, &h_crc, &d_pay, &d_off, &d_len, &d_crc}) b->release();
        std::vector<uint64_t>().swap(at);
        std::vector<size_t>().swap(bstart);
        ready = false;
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

// A reusable barrier for the threads of one run_pool call.
struct Barrier {
    std::mutex mu;
    std::condition_variable cv;
    int n, left;
    uint64_t gen = 0;
    explicit Barrier(int n_) : n(n_), left(n_) {}
    void wait() {
        std::unique_lock<std::mutex> lk(mu);
        const uint64_t g = gen;
        if (--left == 0) {
            left = n;
            ++gen;
            cv.notify_all();
        } else {
            cv.wait(lk, [&] { return gen != g; });
        }
    }
};

// One pass over records [0, n) of the caller's arrays (payload total pay_total <= kCallBytes,
// or a single record): frames what fits from *cursor, returns the number framed.
//
// Every stage runs on all the pool's threads:
//   a. V(i) = sum_{j<i} (len_j + 8), a parallel prefix sum (kept in at[], turned into WAL
//      offsets in place when the record is framed) and the packed payload offsets V(i) - 8 i;
//   b. thread 0: placement in run form (wal_place.h place_runs, one binary search per
//      segment: WalPlacer's result), the footers and the blocks (small first, doubling);
//   c. per block: its records framed into the image (length field + payload) and their
//      payloads packed into pinned staging in the same pass, then its DMA, CRC batch and
//      CRC readback enqueued on one of 8 streams;
//   d. per block, in order, once its CRCs are back: the CRC fields -- between blocks of c.
//      (the block's image lines are then still in the caches), and the rest once every
//      block is enqueued.
// img: the image [*cursor, wal_bytes) is page-locked (the caller's io_uring-registered or
// hipHostMalloc'd WAL buffer): no payload is packed.  Each block's framed image span -- headers,
// payloads and any footer between them, the bytes the reference writes with its one copy
// (segment_file.cc:25-27) -- is DMAed straight from the image, and the CRC batch reads the
// payloads in that device copy (d_pay holds [cur0, end_cursor) of the image).
int append_pass(AppendCtx& C, int dev, const uint8_t* src, const uint64_t* src_off, const uint32_t* len, size_t n,
                uint64_t pay_total, uint32_t max_len, uint8_t* wal, size_t wal_bytes, size_t seg_bytes,
                uint64_t* cursor, uint64_t* rec_off, size_t* n_framed, bool img) {
    karma::engine::PhaseTimer T("wal_append");
    // blocks: at most n / kBlockRecords + (payload / smallest block) + the doubling steps
    const size_t max_blocks = n / kBlockRecords + pay_total / kBlockBytesFirst + 32;
    const uint64_t cur0 = *cursor;
    if (!img) {
        if (const int rc = C.h_pay.ensure(pay_total + 16, true)) return rc;
        if (const int rc = C.d_pay.ensure(pay_total + 16, false)) return rc;
    }
    if (const int rc = C.h_off.ensure(n * 8, true, true)) return rc;
    if (const int rc = C.d_off.ensure(n * 8, false)) return rc;
    if (const int rc = C.h_len.ensure(n * 4, true, true)) return rc;
    if (const int rc = C.d_len.ensure(n * 4, false)) return rc;
    if (const int rc = C.h_crc.ensure(n * 4, true, true)) return rc;
    if (const int rc = C.d_crc.ensure(n * 4, false)) return rc;
    if (const int rc = C.events(max_blocks)) return rc;
    if (C.at.size() < n) C.at.resize(n);
    if (C.bstart.size() < max_blocks + 2) C.bstart.resize(max_blocks + 2);
    T.mark("buffers");
    uint8_t* hp = img ? nullptr : C.h_pay.as<uint8_t>();
    uint64_t* ho = C.h_off.as<uint64_t>();
    uint32_t* hl = C.h_len.as<uint32_t>();
    uint32_t* hc = C.h_crc.as<uint32_t>();
    uint64_t* at = C.at.data();
    size_t* bstart = C.bstart.data();

    const int nthr = (int)std::min<size_t>(karma::engine::kPoolThreads + 1, std::max<size_t>(1, n / 4096));
    Barrier bar(nthr);
    std::vector<uint64_t> csum(nthr + 1, 0);
    std::vector<size_t> cbad(nthr, n);
    std::vector<karma::engine::WalRun> runs;
    std::vector<karma::engine::WalFooter> footers;
    size_t n_valid = 0, framed = 0, nb = 0;
    uint64_t vtotal = 0, end_cursor = *cursor;
    std::atomic<size_t> next_block{0}, next_fill{0};
    std::atomic<int> crc_rc{0};
    std::unique_ptr<std::atomic<uint8_t>[]> enq(new std::atomic<uint8_t>[max_blocks]);
    for (size_t k = 0; k < max_blocks; ++k) enq[k].store(0, std::memory_order_relaxed);
    auto set_rc = [&](int rc) {
        int zero = 0;
        crc_rc.compare_exchange_strong(zero, rc);
    };
    auto chunk = [&](int t, size_t m) { return std::make_pair(m * t / nthr, m * (t + 1) / nthr); };
    // V(i) for i <= n_valid (V(n_valid) = vtotal; at[i] holds V(i) until the block is framed)
    auto V = [&](size_t i) { return i < n_valid ? at[i] : vtotal; };

    // c. one block: its records framed into the image (WAL offset, length field, payload) and
    // their payloads packed into pinned staging in the same pass (the source is read once;
    // the packing copy comes from the caches), then its DMA, CRC batch and CRC readback
    auto frame_block = [&](size_t k) {
        const size_t lo = bstart[k], hi = bstart[k + 1];
        size_t r = std::upper_bound(runs.begin(), runs.end(), lo,
                                    [](size_t i, const karma::engine::WalRun& w) { return i < w.i0; }) -
                   runs.begin() - 1;  // the run holding record lo
        // the block's packed payloads [plo, phi) (V(i) - 8 i: read before this loop turns at[]
        // into WAL offsets; at[hi] belongs to the next block, which may be converting it)
        const uint64_t plo = at[lo] - kHeader * lo, phi = at[hi - 1] - kHeader * (hi - 1) + len[hi - 1];
        bool contiguous = !img;
        for (size_t i = lo + 1; i < hi && contiguous; ++i) contiguous = src_off[i] == src_off[i - 1] + len[i - 1];
        uint64_t ibase = 0;  // img: the block's first header (WAL offset)
        for (size_t i = lo; i < hi; ++i) {  // segment_file::append_record: length field + payload
            while (i >= runs[r].i1) ++r;
            const uint64_t v = at[i], pk = v - kHeader * i;  // V(i), packed payload offset
            at[i] = v + runs[r].base;                         // V(i) -> WAL offset
            uint8_t* p = wal + at[i];
            const uint32_t L = len[i];
            put32(p + 4, L << 8 | 0u);
            copy_payload(p + kHeader, src + src_off[i], L);
            if (img) {
                if (i == lo) ibase = at[i];
                ho[i] = at[i] + kHeader - ibase;  // the payload in the block's image span
            } else {
                if (!contiguous) copy_payload(hp + pk, src + src_off[i], L);
                ho[i] = pk - plo;  // the block's kernel sees its own slice: offsets rebased onto dp + plo
            }
            hl[i] = L;
        }
        if (contiguous) std::memcpy(hp + plo, src + src_off[lo], phi - plo);
        hipStream_t s = C.st[k % kStreams];
        const size_t nr = hi - lo;
        uint64_t* hoff = ho + lo;
        uint64_t* doff = C.d_off.as<uint64_t>() + lo;
        uint32_t* dlen = C.d_len.as<uint32_t>() + lo;
        // the bytes the block's kernel reads: its packed payloads, or (img) its image span
        uint8_t* dp = img ? C.d_pay.as<uint8_t>() + (ibase - cur0) : C.d_pay.as<uint8_t>() + plo;
        const uint8_t* hsrc = img ? wal + ibase : hp + plo;
        const uint64_t dma = img ? at[hi - 1] + kHeader + len[hi - 1] - ibase : phi - plo;
        if (hipMemcpyAsync(dp, hsrc, dma, hipMemcpyHostToDevice, s) != hipSuccess) return (int)KARMA_E_HIP;
        if (max_len <= kZeroCopyMaxLen) {
            // the small-record kernel reads each record's offset and length once and writes its CRC
            // once: it does so over PCIe, from and into the fine-grained host arrays, so the block's
            // only copy is its payload DMA (the small copies each cost the DMA engine ~10 us)
            // (a block of empty payloads has max_len 0, which the ABI reads as "no bound": bound it
            // by 1 so it too takes the small-record kernel and not the unknown-total plan)
            if (const int rc = karma_crc32c_batch_ragged_bounded(dp, hoff, hl + lo, nr, phi - plo,
                                                                 std::max<uint32_t>(max_len, 1), nullptr, 0, hc + lo, s))
                return rc;
        } else {
            if (hipMemcpyAsync(doff, hoff, nr * 8, hipMemcpyHostToDevice, s) != hipSuccess ||
                hipMemcpyAsync(dlen, hl + lo, nr * 4, hipMemcpyHostToDevice, s) != hipSuccess)
                return (int)KARMA_E_HIP;
            if (const int rc = karma_crc32c_batch_ragged_bounded(dp, doff, dlen, nr, phi - plo, max_len, nullptr,
                                                                 0, C.d_crc.as<uint32_t>() + lo, s))
                return rc;
            if (hipMemcpyAsync(hc + lo, C.d_crc.as<uint32_t>() + lo, nr * 4, hipMemcpyDeviceToHost, s) != hipSuccess)
                return (int)KARMA_E_HIP;
        }
        if (hipEventRecord(C.ev[k], s) != hipSuccess) return (int)KARMA_E_HIP;
        return 0;
    };
    // d. the CRC fields of the oldest blocks whose CRCs are back (every such event is this
    // call's: enq); wait = block on the next one instead of returning
    auto fill_ready = [&](bool wait) {
        while (!crc_rc.load(std::memory_order_relaxed)) {
            size_t f = next_fill.load();
            if (f >= nb) return;
            if (!wait && (!enq[f].load(std::memory_order_acquire) || hipEventQuery(C.ev[f]) != hipSuccess)) return;
            if (!next_fill.compare_exchange_strong(f, f + 1)) continue;
            if (wait && hipEventSynchronize(C.ev[f]) != hipSuccess) {
                set_rc(KARMA_E_HIP);
                return;
            }
            for (size_t i = bstart[f]; i < bstart[f + 1]; ++i) put32(wal + at[i], hc[i]);
        }
    };

    auto worker = [&](int t) {
        if (t > 0 && hipSetDevice(dev) != hipSuccess) set_rc(KARMA_E_HIP);  // thread 0 is the caller's
        // a. chunk sums of len + 8 and the first record that can never be placed
        {
            const auto [c0, c1] = chunk(t, n);
            uint64_t sum = 0;
            for (size_t i = c0; i < c1; ++i) {
                const uint64_t L = len[i];
                if (L + kHeader > seg_bytes || (L >> 24)) {  // WalPlacer::place refuses it
                    cbad[t] = i;
                    break;
                }
                sum += L + kHeader;
            }
            csum[t + 1] = sum;
        }
        bar.wait();
        if (t == 0) {
            n_valid = n;
            for (int c = 0; c < nthr; ++c) n_valid = std::min(n_valid, cbad[c]);
            for (int c = 0; c < nthr; ++c) csum[c + 1] += csum[c];
        }
        bar.wait();
        {
            const auto [c0, c1] = chunk(t, n);
            uint64_t v = csum[t];
            for (size_t i = c0; i < std::min(c1, n_valid); ++i) {
                at[i] = v;
                v += len[i] + kHeader;
            }
            if ((c0 <= n_valid && n_valid < c1) || (n_valid == n && t == nthr - 1)) vtotal = v;  // V(n_valid)
        }
        bar.wait();
        if (t == 0) T.mark("a. prefix");
        // b. placement (sivir::build_sqe's loop in run form), the footers and the blocks
        if (t == 0) {
            framed = karma::engine::place_runs(seg_bytes, wal_bytes, &end_cursor, n_valid, V,
                                               [&](size_t i) { return (uint64_t)len[i]; }, &runs, &footers);
            for (const auto& f : footers) {  // segment_file::append_footer
                const uint64_t room = f.f1 - f.f0;
                if (room < kHeader) {
                    std::memset(wal + f.f0, '0', room);
                } else {
                    put32(wal + f.f0, 0);
                    put32(wal + f.f0 + 4, uint32_t((room - kHeader) << 8 | 1u));
                    std::memset(wal + f.f0 + kHeader, '0', room - kHeader);
                }
            }
            bstart[0] = 0;  // [b, e): payload bytes <= blimit, or kBlockRecords records
            uint64_t blimit = kBlockBytesFirst;
            for (size_t b = 0; b < framed;) {
                size_t lo = b + 1, hi = std::min(framed, b + kBlockRecords);
                while (lo < hi) {
                    const size_t mid = lo + (hi - lo + 1) / 2;
                    if (V(mid) - V(b) - kHeader * (mid - b) <= blimit) lo = mid;  // payload bytes of [b, mid)
                    else hi = mid - 1;
                }
                bstart[++nb] = lo;
                b = lo;
                blimit = std::min(2 * blimit, kBlockBytesMax);
            }
            // img: the device copy of the image span this pass frames
            if (img) {
                if (const int rc = C.d_pay.ensure(end_cursor - cur0 + 16, false)) set_rc(rc);
            }
            T.mark("b. placement + blocks");
        }
        bar.wait();
        // c. + d.: frame, pack and enqueue blocks; between blocks, the CRC fields of the blocks
        // whose CRCs are back (their image lines are then still in the caches)
        for (size_t k; !crc_rc.load(std::memory_order_relaxed) && (k = next_block.fetch_add(1)) < nb;) {
            if (const int rc = frame_block(k)) {
                set_rc(rc);
                break;
            }
            enq[k].store(1, std::memory_order_release);
            fill_ready(false);
        }
        bar.wait();  // every block enqueued (an event not recorded in this call would not wait)
        if (t == 0) T.mark("c. frame + enqueue");
        fill_ready(true);
    };
    karma::engine::run_pool(nthr, worker);
    T.mark("d. CRC fields");
    for (auto& s : C.st)  // nothing of this call may be in flight when it returns
        if (hipStreamSynchronize(s) != hipSuccess) set_rc(KARMA_E_HIP);
    T.mark("e. stream syncs");
    if (const int rc = crc_rc.load())  // payloads and length fields are written; CRC fields may not be
        return rc == KARMA_E_HIP ? set_last_error(rc, "wal_append: device pipeline") : rc;
    if (rec_off) std::memcpy(rec_off, at, framed * sizeof(uint64_t));
    *cursor = end_cursor;
    *n_framed = framed;
    return 0;
}

}  // namespace

int karma::engine::trim_append_ctx(int dev) {
    AppendCtx& c = ctx_for(dev);
    std::lock_guard<std::mutex> lk(c.mu);
    c.reset(dev);
    return 0;
}

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
    karma::engine::PhaseTimer T("wal_append call");
    AppendCtx& C = ctx_for(dev);
    std::lock_guard<std::mutex> lk(C.mu);
    if (const int rc = C.init()) return rc;
    const uint8_t* src = static_cast<const uint8_t*>(h_src);
    uint8_t* wal = static_cast<uint8_t*>(h_wal);
    uint64_t cur = *h_cursor;
    size_t done = 0;
    // (the tools build's KARMA_APPEND_CALL_BYTES lowers the pass size, so tests cross passes)
    const uint64_t call_bytes = (uint64_t)KARMA_AB_KNOB("KARMA_APPEND_CALL_BYTES", (long)kCallBytes);
    while (done < n) {  // passes of at most call_bytes of payload (at least one record)
        size_t m = 1;
        uint64_t bytes = h_len[done];
        uint32_t max_len = h_len[done];
        // whole runs of kSumRun records while they fit (a loop the compiler vectorises: the
        // record-by-record form cost ~1 ms per million records), then record by record
        constexpr size_t kSumRun = 4096;
        while (done + m + kSumRun <= n) {
            uint64_t s = 0;
            uint32_t mx = 0;
            const uint32_t* l = h_len + done + m;
            for (size_t k = 0; k < kSumRun; ++k) {
                s += l[k];
                mx = std::max(mx, l[k]);
            }
            if (bytes + s > call_bytes) break;
            bytes += s;
            max_len = std::max(max_len, mx);
            m += kSumRun;
        }
        for (; done + m < n && bytes + h_len[done + m] <= call_bytes; ++m) {
            bytes += h_len[done + m];
            max_len = std::max(max_len, h_len[done + m]);
        }
        size_t framed = 0;
        const bool img = cur < wal_bytes && karma::engine::host_range_pinned(wal + cur, wal_bytes - cur) &&
                         KARMA_AB_KNOB("KARMA_APPEND_IMAGE_DMA", 1);
        if (const int rc = append_pass(C, dev, src, h_src_off + done, h_len + done, m, bytes, max_len, wal, wal_bytes,
                                       seg_bytes, &cur, h_rec_off ? h_rec_off + done : nullptr, &framed, img))
            return rc;  // *h_cursor and *h_n_framed keep the passes already complete
        done += framed;
        *h_cursor = cur;
        *h_n_framed = done;
        if (framed < m) break;  // the image is full (or a record can never fit)
    }
    T.mark("whole call");
    return 0;
}
