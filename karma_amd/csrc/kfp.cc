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
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "engine.h"
#include "karma_crc32c.h"

namespace karma::engine {
int set_last_error(int code, const std::string& what);  // capi.cc

// CRCs of the spans (off[i], len[i]) of a buffer in one ragged GPU batch: from host
// memory (batch_ragged_host), or over the caller's device copy d_buf.
int crc_spans(const void* h_buf, const void* d_buf, size_t buf_bytes, const std::vector<uint64_t>& off,
              const std::vector<uint32_t>& len, std::vector<uint32_t>& out, int device) {
    out.resize(off.size());
    if (off.empty()) return 0;
    if (!d_buf) return karma_crc32c_batch_ragged_host(h_buf, buf_bytes, off.data(), len.data(), off.size(), 0,
                                                      out.data(), device);
    // device copy supplied: stage the offsets/lengths and run the device batch
    uint64_t total = 0;
    uint32_t max_len = 0;
    for (uint32_t l : len) {
        total += l;
        max_len = std::max(max_len, l);
    }
    if (device >= 0 && hipSetDevice(device) != hipSuccess) return set_last_error(KARMA_E_HIP, "hipSetDevice");
    void *doff = nullptr, *dlen = nullptr, *dout = nullptr;
    int rc = 0;
    if (hipMalloc(&doff, off.size() * 8) != hipSuccess || hipMalloc(&dlen, len.size() * 4) != hipSuccess ||
        hipMalloc(&dout, out.size() * 4) != hipSuccess)
        rc = set_last_error(KARMA_E_NOMEM, "crc_spans: hipMalloc");
    else if (hipMemcpy(doff, off.data(), off.size() * 8, hipMemcpyHostToDevice) != hipSuccess ||
             hipMemcpy(dlen, len.data(), len.size() * 4, hipMemcpyHostToDevice) != hipSuccess)
        rc = set_last_error(KARMA_E_HIP, "crc_spans: hipMemcpy H2D");
    else if ((rc = karma_crc32c_batch_ragged_bounded(d_buf, static_cast<uint64_t*>(doff), static_cast<uint32_t*>(dlen),
                                                     off.size(), total, max_len, nullptr, 0,
                                                     static_cast<uint32_t*>(dout), nullptr)))
        ;
    else if (hipMemcpy(out.data(), dout, out.size() * 4, hipMemcpyDeviceToHost) != hipSuccess)
        rc = set_last_error(KARMA_E_HIP, "crc_spans: hipMemcpy D2H");
    (void)hipFree(doff);
    (void)hipFree(dlen);
    (void)hipFree(dout);
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

}  // namespace

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
    // 2. frames written by 16 threads, piece by piece; 3. each written piece's
    //    CRCs (streamed to the device through the pinned staging, host_stage.h), Extend(Value(header), payload) = Value(frame[16, 16 + hl + pl)), in one
    //    GPU batch on a worker thread while the next piece is written
    constexpr size_t kPieces = 4;
    const size_t npc = ne >= 4 * 4096 ? kPieces : 1;
    std::atomic<size_t> written{0};
    int crc_rc = 0;
    std::thread gpu([&] {
        for (size_t p = 0; p < npc && !crc_rc; ++p) {
            const size_t lo = ne * p / npc, hi = ne * (p + 1) / npc;
            while (written.load(std::memory_order_acquire) <= p) std::this_thread::yield();
            if (lo == hi) continue;
            std::vector<uint64_t> so(hi - lo);
            std::vector<uint32_t> sl(hi - lo), crc;
            for (size_t k = lo; k < hi; ++k) {
                so[k - lo] = at[k] + kFixed;
                sl[k - lo] = h_hdr_len[k] + h_pay_len[k];
            }
            if ((crc_rc = karma::engine::crc_spans(out, nullptr, cur, so, sl, crc, device))) break;
            for (size_t k = 0; k < crc.size(); ++k) std::memcpy(out + so[k] + sl[k], &crc[k], 4);
        }
    });
    for (size_t p = 0; p < npc; ++p) {
        const size_t lo = ne * p / npc, hi = ne * (p + 1) / npc;
        const size_t nthr = std::min<size_t>(16, std::max<size_t>(1, (hi - lo) / 1024));
        std::vector<std::thread> th;
        for (size_t t = 0; t < nthr; ++t)
            th.emplace_back([&, t] {
                for (size_t i = lo + (hi - lo) * t / nthr; i < lo + (hi - lo) * (t + 1) / nthr; ++i) {
                    const uint32_t hl = h_hdr_len[i], pl = h_pay_len[i];
                    const uint32_t fl = kFixed + hl + pl + kCrcLen;
                    uint8_t* f = out + at[i];
                    std::memcpy(f, &fl, 4);
                    f[4] = KARMA_KFP_MAGIC;
                    std::memcpy(f + 5, &h_op[i], 2);
                    f[7] = h_flag[i];
                    std::memcpy(f + 8, &h_seq[i], 4);
                    std::memcpy(f + 12, &hl, 4);
                    if (hl) std::memcpy(f + kFixed, hdr + h_hdr_off[i], hl);
                    if (pl) std::memcpy(f + kFixed + hl, pay + h_pay_off[i], pl);
                    if (h_frame_off) h_frame_off[i] = at[i];
                }
            });
        for (auto& x : th) x.join();
        written.store(p + 1, std::memory_order_release);
    }
    gpu.join();
    if (crc_rc) return crc_rc;
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
