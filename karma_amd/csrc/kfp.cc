// karma_amd/csrc/kfp.cc -- batched KFP frame encode / parse on top of the GPU
// CRC batches.
//
// Frame layout (karma-transport/frame.cc:29-60, frame.h:20-23), native
// little-endian integers:
//   [frame_length u32][magic u8 = 123][operation_code i16][flag u8][seq u32]
//   [header_length u32][header][payload][crc u32]
// frame_length = 16 + header + payload + 4, and
// crc = Extend(Value(header), payload) (frame.cc:56-57).  Header and payload
// are adjacent in the frame, so crc = Value(frame[16, frame_length - 4)): one
// span per frame, which is what the ragged batch checksums.
//
// karma_kfp_encode_batch = frame::encode for n frames written back to back.
// karma_kfp_parse_batch  = connection::read_frame's loop over a receive buffer
//   (connection.cc:20-27): frame::parse at the cursor (frame.cc:62-130), erase
//   frame->size() bytes, repeat.  It stops where parse returns nullopt
//   (incomplete frame) or throws (bad size / magic / header length / crc).
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
#include "karma_crc32c.h"

namespace karma::engine {
int set_last_error(int code, const std::string& what);  // capi.cc

namespace {
// crc_spans' grow-only device copies of the span lists, per device.
struct SpanBufs {
    std::mutex mu;
    void *off = nullptr, *len = nullptr, *out = nullptr;
    size_t cap = 0;  // records
    void release() {  // the caller holds mu
        (void)hipFree(off);
        (void)hipFree(len);
        (void)hipFree(out);
        off = len = out = nullptr;
        cap = 0;
    }
};
std::mutex g_span_mu;
std::vector<std::unique_ptr<SpanBufs>> g_span_bufs;
SpanBufs* span_bufs(int dev) {
    std::lock_guard<std::mutex> g(g_span_mu);
    if ((int)g_span_bufs.size() <= dev) g_span_bufs.resize(dev + 1);
    if (!g_span_bufs[dev]) g_span_bufs[dev] = std::make_unique<SpanBufs>();
    return g_span_bufs[dev].get();
}
}  // namespace

// CRCs of the spans (off[i], len[i]) of a buffer in one ragged GPU batch: from host
// memory (batch_ragged_host), or over the caller's device copy d_buf.
int crc_spans(const void* h_buf, const void* d_buf, size_t buf_bytes, const std::vector<uint64_t>& off,
              const std::vector<uint32_t>& len, std::vector<uint32_t>& out, int device) {
    out.resize(off.size());
    if (off.empty()) return 0;
    if (!d_buf) return karma_crc32c_batch_ragged_host(h_buf, buf_bytes, off.data(), len.data(), off.size(), 0,
                                                      out.data(), device);
    // device copy supplied: stage the offsets/lengths and run the device batch (grow-only
    // device buffers kept per device: no allocation per call)
    uint64_t total = 0;
    uint32_t max_len = 0;
    for (uint32_t l : len) {
        total += l;
        max_len = std::max(max_len, l);
    }
    int dev = 0;
    if (device >= 0 && hipSetDevice(device) != hipSuccess) return set_last_error(KARMA_E_HIP, "hipSetDevice");
    if (hipGetDevice(&dev) != hipSuccess) return set_last_error(KARMA_E_HIP, "hipGetDevice");
    SpanBufs* B = span_bufs(dev);
    std::lock_guard<std::mutex> lk(B->mu);
    if (B->cap < off.size()) {
        B->release();
        const size_t cap = off.size() + off.size() / 8;
        if (hipMalloc(&B->off, cap * 8) != hipSuccess || hipMalloc(&B->len, cap * 4) != hipSuccess ||
            hipMalloc(&B->out, cap * 4) != hipSuccess)
            return set_last_error(KARMA_E_NOMEM, "crc_spans: hipMalloc");
        B->cap = cap;
    }
    int rc = 0;
    if (hipMemcpy(B->off, off.data(), off.size() * 8, hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(B->len, len.data(), len.size() * 4, hipMemcpyHostToDevice) != hipSuccess)
        rc = set_last_error(KARMA_E_HIP, "crc_spans: hipMemcpy H2D");
    else if ((rc = karma_crc32c_batch_ragged_bounded(d_buf, static_cast<uint64_t*>(B->off),
                                                     static_cast<uint32_t*>(B->len), off.size(), total, std::max<uint32_t>(max_len, 1),
                                                     nullptr, 0, static_cast<uint32_t*>(B->out), nullptr)))
        ;
    else if (hipMemcpy(out.data(), B->out, out.size() * 4, hipMemcpyDeviceToHost) != hipSuccess)
        rc = set_last_error(KARMA_E_HIP, "crc_spans: hipMemcpy D2H");
    return rc;
}

// frame::parse at the cursor, advance by frame_length, repeat (connection::read_frame,
// connection.cc:20-27): the structural checks in parse's order (frame.cc:64-116), without
// the CRC, which the caller verifies for all frames at once.
int kfp_walk(const uint8_t* b, size_t buf_bytes, size_t max_frames, KfpWalk* W) {
    constexpr uint32_t kFixed = KARMA_KFP_FIXED_HEADER, kCrcLen = 4;  // frame.h:21-22
    auto le32 = [](const uint8_t* p) {
        uint32_t v;
        std::memcpy(&v, p, 4);
        return v;
    };
    uint64_t cur = 0;
    int status = KARMA_KFP_OK;
    while (W->frame.size() < max_frames) {
        const uint64_t avail = buf_bytes - cur;
        if (avail < kFixed + kCrcLen) break;  // nullopt: wait for more bytes (:64-66)
        const uint32_t fl = le32(b + cur);
        if (fl > KARMA_KFP_MAX_FRAME) {  // throws "decoded frame size is larger than the limit" (:70-73)
            status = KARMA_KFP_BAD_SIZE;
            break;
        }
        if (avail < fl) break;                  // nullopt: incomplete frame (:75-77)
        if (b[cur + 4] != KARMA_KFP_MAGIC) {    // throws "Wrong magic code" (:86-89)
            status = KARMA_KFP_BAD_MAGIC;
            break;
        }
        if (fl < kFixed + kCrcLen) {  // unsigned wrap in :101 and :111-113: undefined in the reference
            status = KARMA_KFP_BAD_LENGTH;
            break;
        }
        const uint32_t hl = le32(b + cur + 12);
        if (hl > fl - kFixed - kCrcLen) {  // throws "Wrong header length" (:101-104)
            status = KARMA_KFP_BAD_HEADER_LEN;
            break;
        }
        W->frame.push_back(cur);
        W->span_off.push_back(cur + kFixed);
        W->span_len.push_back(fl - kFixed - kCrcLen);
        W->stored.push_back(le32(b + cur + fl - kCrcLen));
        cur += fl;  // read_frame erases frame->size() == frame_length bytes (connection.cc:25)
    }
    W->consumed = cur;
    return status;
}
}  // namespace karma::engine

namespace {

constexpr uint32_t kFixed = KARMA_KFP_FIXED_HEADER;  // frame.h:21
constexpr uint32_t kCrcLen = 4;                      // frame.h:22

inline uint32_t le32(const uint8_t* p) {
    uint32_t v;
    std::memcpy(&v, p, 4);
    return v;
}

int fail(int code, const char* what) { return karma::engine::set_last_error(code, what); }

// ---- the encoder's pipeline (the structure of wal_append.cc) ------------------------------
constexpr int kEncStreams = 8;                          // DMA / CRC streams the blocks rotate over
constexpr size_t kEncBlockFrames = 16384;               // a block: at most this many frames,
constexpr uint64_t kEncBlockBytesFirst = uint64_t(256) << 10;  // or about this many span bytes
constexpr uint64_t kEncBlockBytesMax = uint64_t(4) << 20;      // (doubling from the first block)
constexpr uint64_t kEncCallBytes = uint64_t(1) << 30;   // span bytes staged per pass

struct EncBuf {
    void* p = nullptr;
    size_t bytes = 0;
    bool host = false;
    int ensure(size_t want, bool pinned_host) {
        if (p && bytes >= want) return 0;
        if (p) (void)(host ? hipHostFree(p) : hipFree(p));
        p = nullptr;
        bytes = 0;
        want = std::max<size_t>(want + want / 8, 4096);
        if ((pinned_host ? hipHostMalloc(&p, want, hipHostMallocDefault) : hipMalloc(&p, want)) != hipSuccess) {
            p = nullptr;
            return fail(KARMA_E_NOMEM, "kfp_encode_batch: allocation");
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

// Per-device encoder context: streams, one event per block, grow-only pinned staging and device
// copies of the packed CRC spans, their offsets, lengths and CRCs.
struct EncCtx {
    std::mutex mu;
    bool ready = false;
    hipStream_t st[kEncStreams] = {};
    std::vector<hipEvent_t> ev;
    EncBuf h_span, h_off, h_len, h_crc, d_span, d_off, d_len, d_crc;
    std::vector<size_t> bstart;
    int init() {
        if (ready) return 0;
        for (auto& x : st)
            if (hipStreamCreateWithFlags(&x, hipStreamNonBlocking) != hipSuccess)
                return fail(KARMA_E_HIP, "kfp_encode_batch: stream");
        ready = true;
        return 0;
    }
    int events(size_t k) {
        while (ev.size() < k) {
            hipEvent_t e;
            if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess)
                return fail(KARMA_E_HIP, "kfp_encode_batch: event");
            ev.push_back(e);
        }
        return 0;
    }
    void reset(int dev) {  // karma_crc32c_trim (the caller holds mu)
        if (!ready) return;
        for (auto& x : st) {
            (void)hipStreamSynchronize(x);
            (void)karma::engine::release_internal_stream(dev, x);
            (void)hipStreamDestroy(x);
            x = nullptr;
        }
        for (hipEvent_t e : ev) (void)hipEventDestroy(e);
        ev.clear();
        for (EncBuf* b : {&h_span, &h_off, &h_len, &h_crc, &d_span, &d_off, &d_len, &d_crc}) b->release();
        std::vector<size_t>().swap(bstart);
        ready = false;
    }
};

std::mutex g_enc_mu;
std::vector<std::unique_ptr<EncCtx>> g_enc;

EncCtx& enc_ctx(int dev) {
    std::lock_guard<std::mutex> g(g_enc_mu);
    if ((int)g_enc.size() <= dev) g_enc.resize(dev + 1);
    if (!g_enc[dev]) g_enc[dev] = std::make_unique<EncCtx>();
    return *g_enc[dev];
}

struct EncFrames {
    const uint8_t* hdr;
    const uint64_t* hdr_off;
    const uint32_t* hdr_len;
    const uint8_t* pay;
    const uint64_t* pay_off;
    const uint32_t* pay_len;
    const int16_t* op;
    const uint8_t* flag;
    const uint32_t* seq;
    uint8_t* out;
    const uint64_t* at;  // frame offsets in out
};

// Frames [f0, f0 + m) (span bytes `span`, <= kEncCallBytes unless one frame), on the library's
// host threads: the threads take blocks of frames in turn, write each frame
// (frame::encode's fields, header, payload) and pack its CRC span -- header + payload,
// Value(frame[16, frame_length - 4)) = Extend(Value(header), payload), frame.cc:56-57 -- into
// pinned staging in the same pass, then enqueue the block's DMA, CRC batch and CRC readback on
// one of 8 streams; between blocks, and once every block is enqueued, they write the CRC fields
// of the blocks whose CRCs are back, in order.
int encode_pass(EncCtx& C, int dev, const EncFrames& F, size_t f0, size_t m, uint64_t span) {
    const size_t max_blocks = m / kEncBlockFrames + span / kEncBlockBytesFirst + 32;
    if (const int rc = C.h_span.ensure(span + 16, true)) return rc;
    if (const int rc = C.d_span.ensure(span + 16, false)) return rc;
    if (const int rc = C.h_off.ensure(m * 8, true)) return rc;
    if (const int rc = C.d_off.ensure(m * 8, false)) return rc;
    if (const int rc = C.h_len.ensure(m * 4, true)) return rc;
    if (const int rc = C.d_len.ensure(m * 4, false)) return rc;
    if (const int rc = C.h_crc.ensure(m * 4, true)) return rc;
    if (const int rc = C.d_crc.ensure(m * 4, false)) return rc;
    if (const int rc = C.events(max_blocks)) return rc;
    if (C.bstart.size() < max_blocks + 2) C.bstart.resize(max_blocks + 2);
    uint64_t* so = C.h_off.as<uint64_t>();  // packed span offset per frame (rebased per block when enqueued)
    uint32_t* sl = C.h_len.as<uint32_t>();
    uint32_t* hc = C.h_crc.as<uint32_t>();
    uint8_t* hs = C.h_span.as<uint8_t>();
    size_t* bstart = C.bstart.data();
    // the blocks, and the packed span offsets
    size_t nb = 0;
    uint32_t max_len = 0;
    {
        uint64_t packed = 0, bbytes = 0, blimit = kEncBlockBytesFirst;
        bstart[0] = 0;
        for (size_t i = 0; i < m; ++i) {
            const uint32_t L = F.hdr_len[f0 + i] + F.pay_len[f0 + i];
            so[i] = packed;
            sl[i] = L;
            max_len = std::max(max_len, L);
            packed += L;
            bbytes += L;
            if (i + 1 - bstart[nb] == kEncBlockFrames || bbytes >= blimit || i + 1 == m) {
                bstart[++nb] = i + 1;
                bbytes = 0;
                blimit = std::min(2 * blimit, kEncBlockBytesMax);
            }
        }
    }
    std::atomic<size_t> next_block{0}, next_fill{0};
    std::atomic<int> crc_rc{0};
    std::unique_ptr<std::atomic<uint8_t>[]> enq(new std::atomic<uint8_t>[nb]);
    for (size_t k = 0; k < nb; ++k) enq[k].store(0, std::memory_order_relaxed);
    auto set_rc = [&](int rc) {
        int zero = 0;
        crc_rc.compare_exchange_strong(zero, rc);
    };
    auto frame_block = [&](size_t k) {
        const size_t lo = bstart[k], hi = bstart[k + 1];
        for (size_t i = lo; i < hi; ++i) {  // frame::encode (frame.cc:29-60)
            const size_t g = f0 + i;
            const uint32_t hl = F.hdr_len[g], pl = F.pay_len[g];
            const uint32_t fl = kFixed + hl + pl + kCrcLen;
            uint8_t* f = F.out + F.at[g];
            std::memcpy(f, &fl, 4);
            f[4] = KARMA_KFP_MAGIC;
            std::memcpy(f + 5, &F.op[g], 2);
            f[7] = F.flag[g];
            std::memcpy(f + 8, &F.seq[g], 4);
            std::memcpy(f + 12, &hl, 4);
            if (hl) std::memcpy(f + kFixed, F.hdr + F.hdr_off[g], hl);
            if (pl) std::memcpy(f + kFixed + hl, F.pay + F.pay_off[g], pl);
            if (hl + pl) std::memcpy(hs + so[i], f + kFixed, hl + pl);  // the span, from the caches
        }
        const uint64_t plo = so[lo], phi = so[hi - 1] + sl[hi - 1];
        for (size_t i = lo; i < hi; ++i) so[i] -= plo;  // the block's kernel sees its own slice
        hipStream_t s = C.st[k % kEncStreams];
        const size_t nr = hi - lo;
        uint8_t* dp = C.d_span.as<uint8_t>();
        uint64_t* doff = C.d_off.as<uint64_t>() + lo;
        uint32_t* dlen = C.d_len.as<uint32_t>() + lo;
        if ((phi > plo && hipMemcpyAsync(dp + plo, hs + plo, phi - plo, hipMemcpyHostToDevice, s) != hipSuccess) ||
            hipMemcpyAsync(doff, so + lo, nr * 8, hipMemcpyHostToDevice, s) != hipSuccess ||
            hipMemcpyAsync(dlen, sl + lo, nr * 4, hipMemcpyHostToDevice, s) != hipSuccess)
            return (int)KARMA_E_HIP;
        // (max_len 0, every span empty, would read as "no bound" and take the unknown-total plan)
        if (const int rc = karma_crc32c_batch_ragged_bounded(dp + plo, doff, dlen, nr, phi - plo,
                                                             std::max<uint32_t>(max_len, 1), nullptr, 0,
                                                             C.d_crc.as<uint32_t>() + lo, s))
            return rc;
        if (hipMemcpyAsync(hc + lo, C.d_crc.as<uint32_t>() + lo, nr * 4, hipMemcpyDeviceToHost, s) != hipSuccess ||
            hipEventRecord(C.ev[k], s) != hipSuccess)
            return (int)KARMA_E_HIP;
        return 0;
    };
    auto fill = [&](size_t k) {  // the CRC fields of block k (frame.cc:58-59)
        for (size_t i = bstart[k]; i < bstart[k + 1]; ++i) {
            const size_t g = f0 + i;
            std::memcpy(F.out + F.at[g] + kFixed + sl[i], &hc[i], 4);
        }
    };
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
            fill(f);
        }
    };
    const int nthr = (int)std::min<size_t>(karma::engine::kPoolThreads + 1, std::max<size_t>(1, m / 1024));
    std::mutex bmu;
    std::condition_variable bcv;
    int framing = nthr;
    karma::engine::run_pool(nthr, [&](int t) {
        if (t > 0 && hipSetDevice(dev) != hipSuccess) set_rc(KARMA_E_HIP);  // thread 0 is the caller's
        for (size_t k; !crc_rc.load(std::memory_order_relaxed) && (k = next_block.fetch_add(1)) < nb;) {
            if (const int rc = frame_block(k)) {
                set_rc(rc);
                break;
            }
            enq[k].store(1, std::memory_order_release);
            fill_ready(false);
        }
        {  // every block enqueued (an event not recorded in this call would not wait)
            std::unique_lock<std::mutex> lk(bmu);
            if (--framing == 0) bcv.notify_all();
            bcv.wait(lk, [&] { return framing == 0; });
        }
        fill_ready(true);
    });
    for (auto& x : C.st)  // nothing of this call may be in flight when it returns
        if (hipStreamSynchronize(x) != hipSuccess) set_rc(KARMA_E_HIP);
    if (const int rc = crc_rc.load())
        return rc == KARMA_E_HIP ? fail(rc, "kfp_encode_batch: device pipeline") : rc;
    return 0;
}

}  // namespace

int karma::engine::trim_kfp_ctx(int dev) {
    {
        EncCtx& c = enc_ctx(dev);
        std::lock_guard<std::mutex> lk(c.mu);
        c.reset(dev);
    }
    SpanBufs* B = span_bufs(dev);
    std::lock_guard<std::mutex> lk(B->mu);
    B->release();
    return 0;
}


extern "C" {

int karma_kfp_encode_batch(const void* h_hdr, const uint64_t* h_hdr_off, const uint32_t* h_hdr_len,
                           const void* h_pay, const uint64_t* h_pay_off, const uint32_t* h_pay_len,
                           const int16_t* h_op, const uint8_t* h_flag, const uint32_t* h_seq, size_t n, void* h_out,
                           size_t out_bytes, uint64_t* h_frame_off, size_t* h_n_encoded, uint64_t* h_bytes,
                           int device) {
    if (!h_n_encoded || !h_bytes || (n && (!h_hdr_len || !h_pay_len || !h_op || !h_flag || !h_seq || !h_out)))
        return fail(KARMA_E_INVALID, "kfp_encode_batch: null argument");
    const uint8_t* hdr = static_cast<const uint8_t*>(h_hdr);
    const uint8_t* pay = static_cast<const uint8_t*>(h_pay);
    uint8_t* out = static_cast<uint8_t*>(h_out);
    // 1. frame offsets (frame::encode writes frames back to back) and argument checks
    std::vector<uint64_t> at;
    at.reserve(n);
    uint64_t cur = 0;
    size_t ne = 0;
    for (; ne < n; ++ne) {
        const uint64_t hl = h_hdr_len[ne], pl = h_pay_len[ne];
        const uint64_t fl = kFixed + hl + pl + kCrcLen;
        if (fl > 0xFFFFFFFFull) return fail(KARMA_E_INVALID, "kfp_encode_batch: frame_length overflows u32");
        if ((hl && (!hdr || !h_hdr_off)) || (pl && (!pay || !h_pay_off)))
            return fail(KARMA_E_INVALID, "kfp_encode_batch: null header/payload source");
        if (cur + fl > out_bytes) break;  // the rest does not fit: caller flushes and continues
        at.push_back(cur);
        cur += fl;
    }
    if (ne) {
        int dev = 0, nd = 0;
        if (hipGetDeviceCount(&nd) != hipSuccess || nd <= 0) return fail(KARMA_E_NO_DEVICE, "no HIP device visible");
        if (device >= nd) return fail(KARMA_E_INVALID, "kfp_encode_batch: device index out of range");
        if (device >= 0 && hipSetDevice(device) != hipSuccess) return fail(KARMA_E_HIP, "hipSetDevice");
        if (hipGetDevice(&dev) != hipSuccess) return fail(KARMA_E_HIP, "hipGetDevice");
        EncCtx& C = enc_ctx(dev);
        std::lock_guard<std::mutex> lk(C.mu);
        if (const int rc = C.init()) return rc;
        // 2. passes of at most kEncCallBytes of CRC span (header + payload) per pass
        for (size_t done = 0; done < ne;) {
            size_t m = 1;
            uint64_t span = h_hdr_len[done] + (uint64_t)h_pay_len[done];
            for (; done + m < ne && span + h_hdr_len[done + m] + h_pay_len[done + m] <= kEncCallBytes; ++m)
                span += h_hdr_len[done + m] + (uint64_t)h_pay_len[done + m];
            const EncFrames F{hdr, h_hdr_off, h_hdr_len, pay, h_pay_off, h_pay_len, h_op, h_flag, h_seq, out, at.data()};
            if (const int rc = encode_pass(C, dev, F, done, m, span)) return rc;
            done += m;
        }
        if (h_frame_off) std::memcpy(h_frame_off, at.data(), ne * sizeof(uint64_t));
    }
    *h_n_encoded = ne;
    *h_bytes = cur;
    return 0;
}

int karma_kfp_parse_batch(const void* h_buf, const void* d_buf, size_t buf_bytes, size_t max_frames,
                          uint64_t* h_frame_off, size_t* h_n_frames, uint64_t* h_consumed, int* h_status,
                          int device) {
    if (!h_n_frames || !h_consumed || !h_status || (buf_bytes && !h_buf))
        return fail(KARMA_E_INVALID, "kfp_parse_batch: null argument");
    // 1. structural walk: parse's checks in its order (frame.cc:64-116)
    karma::engine::KfpWalk W;
    int status = karma::engine::kfp_walk(static_cast<const uint8_t*>(h_buf), buf_bytes, max_frames, &W);
    uint64_t cur = W.consumed;
    const std::vector<uint64_t>& frame = W.frame;
    // 2. every frame's crc in one GPU batch; the first mismatch throws "Wrong crc32" (:125-128)
    std::vector<uint32_t> got;
    if (const int rc = karma::engine::crc_spans(h_buf, d_buf, buf_bytes, W.span_off, W.span_len, got, device))
        return rc;
    size_t ok = frame.size();
    for (size_t k = 0; k < got.size(); ++k)
        if (got[k] != W.stored[k]) {
            ok = k;
            status = KARMA_KFP_BAD_CRC;
            cur = frame[k];
            break;
        }
    if (h_frame_off)
        for (size_t k = 0; k < ok; ++k) h_frame_off[k] = frame[k];
    *h_n_frames = ok;
    *h_consumed = cur;
    *h_status = status;
    return 0;
}

}  // extern "C"
