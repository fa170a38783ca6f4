// karma_amd/csrc/wal.cc -- batched WAL framing and replay on top of the GPU
// CRC batches.
//
// Record format (karma-store/segment_file.cc:21-31, common.h:11):
//   [crc u32 LE = Value(payload)][len << 8 | type u32 LE][payload]
// type 1 = padding to the segment end with '0' bytes and crc field 0
// (segment_file.cc:33-49); a segment tail shorter than a header is padded
// with '0' bytes only (:34-39).
//
// karma_wal_append_batch  = sivir::build_sqe's loop (sivir.cc:276-317): for
//   each payload, segment.can_hold (segment_file.cc:74-77) or close the
//   segment with append_footer and move on; then append_record.  The
//   payload CRCs of the whole batch are computed in one GPU ragged batch.
// karma_wal_replay        = sivir::open's loop over wal::scan_record
//   (sivir.cc:31-41, wal.cc:34-87): headers are walked on the host, every
//   payload CRC is verified in one GPU ragged batch, and replay stops where
//   scan_record would return false.  The reference's quirk for a type-0
//   record of size 0 is kept: read_exact_at returns early for size 0
//   (segment_file.cc:8) so the CRC is taken over the stale 4-byte len/type
//   word just read (wal.cc:50-60).  It is load-bearing: it is what ends replay
//   at the zero-filled, never-written part of the last segment.
#include <hip/hip_runtime_api.h>

#include <algorithm>
#include <cstring>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "karma-util/crc32c.h"
#include "host_trace.h"
#include "karma_crc32c.h"

namespace karma::engine {
int set_last_error(int code, const std::string& what);  // capi.cc

int crc_spans(const void* h_buf, const void* d_buf, size_t buf_bytes, const std::vector<uint64_t>& off,
              const std::vector<uint32_t>& len, std::vector<uint32_t>& out, int device) {
    out.resize(off.size());
    if (off.empty()) return 0;
    if (!d_buf) return karma_crc32c_batch_ragged_host(h_buf, buf_bytes, off.data(), len.data(), off.size(), 0,
                                                      out.data(), device);
    // device copy supplied: stage the offsets/lengths and run the device batch
    uint64_t total = 0;
    for (uint32_t l : len) total += l;
    if (device >= 0 && hipSetDevice(device) != hipSuccess) return set_last_error(KARMA_E_HIP, "hipSetDevice");
    void *doff = nullptr, *dlen = nullptr, *dout = nullptr;
    int rc = 0;
    if (hipMalloc(&doff, off.size() * 8) != hipSuccess || hipMalloc(&dlen, len.size() * 4) != hipSuccess ||
        hipMalloc(&dout, out.size() * 4) != hipSuccess)
        rc = set_last_error(KARMA_E_NOMEM, "crc_spans: hipMalloc");
    else if (hipMemcpy(doff, off.data(), off.size() * 8, hipMemcpyHostToDevice) != hipSuccess ||
             hipMemcpy(dlen, len.data(), len.size() * 4, hipMemcpyHostToDevice) != hipSuccess)
        rc = set_last_error(KARMA_E_HIP, "crc_spans: hipMemcpy H2D");
    else if ((rc = karma_crc32c_batch_ragged(d_buf, static_cast<uint64_t*>(doff), static_cast<uint32_t*>(dlen),
                                             off.size(), total, nullptr, 0, static_cast<uint32_t*>(dout), nullptr)))
        ;
    else if (hipMemcpy(out.data(), dout, out.size() * 4, hipMemcpyDeviceToHost) != hipSuccess)
        rc = set_last_error(KARMA_E_HIP, "crc_spans: hipMemcpy D2H");
    (void)hipFree(doff);
    (void)hipFree(dlen);
    (void)hipFree(dout);
    return rc;
}
}  // namespace karma::engine

namespace {

inline uint32_t le32(const uint8_t* p) {
    return uint32_t(p[0]) | uint32_t(p[1]) << 8 | uint32_t(p[2]) << 16 | uint32_t(p[3]) << 24;
}
inline void put32(uint8_t* p, uint32_t v) {
    p[0] = uint8_t(v);
    p[1] = uint8_t(v >> 8);
    p[2] = uint8_t(v >> 16);
    p[3] = uint8_t(v >> 24);
}

constexpr uint64_t kHeader = 8;  // store::RECORD_HEADER_LENGTH (common.h:11)

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

// One replay candidate: payload span to checksum and the stored CRC.
struct Cand {
    uint64_t rec;      // WAL offset of the header
    uint64_t off;      // checksummed span (payload, or the len/type word for size 0)
    uint32_t len;
    uint32_t stored;
};

// Walk one segment's headers from `pos` (scan_record's structural checks).
// Returns the stop kind: 0 = reached the segment end (padding / short tail),
// 1 = corrupt (length past the segment end, or a size-0 record whose stale
// 4-byte CRC mismatches), 2 = unknown record type.
int walk_segment(const uint8_t* seg, uint64_t seg_base, uint64_t seg_bytes, uint64_t pos, std::vector<Cand>& out,
                 uint64_t* stop) {
    while (true) {
        if (pos + kHeader > seg_bytes) {  // wal.cc:40-45: the rest of the segment is skipped
            *stop = seg_base + seg_bytes;
            return 0;
        }
        const uint32_t crc = le32(seg + pos);
        const uint32_t st = le32(seg + pos + 4);
        const uint32_t type = st & 0xffu, size = st >> 8;
        if (type == 0) {
            if (pos + kHeader + size > seg_bytes) {  // wal.cc:71-74
                *stop = seg_base + pos;
                return 1;
            }
            if (size == 0) {  // stale len/type word (wal.cc:50, segment_file.cc:8)
                if (crc32c::Value(reinterpret_cast<const char*>(seg + pos + 4), 4) != crc) {
                    *stop = seg_base + pos;
                    return 1;
                }
                out.push_back(Cand{seg_base + pos, 0, 0, crc});
                pos += kHeader;
                continue;
            }
            out.push_back(Cand{seg_base + pos, seg_base + pos + kHeader, size, crc});
            pos += kHeader + size;
        } else if (type == 1) {  // padding: skip to the segment end (wal.cc:76-82)
            *stop = seg_base + seg_bytes;
            return 0;
        } else {
            *stop = seg_base + pos;
            return 2;
        }
    }
}

int fail(int code, const char* what) { return karma::engine::set_last_error(code, what); }

static_assert(KARMA_WAL_CORRUPT == 1 && KARMA_WAL_BAD_TYPE == 2, "walk_segment stop kinds");

// Device copy of a host WAL image, uploaded on a worker thread while the caller
// walks the headers.  One cached, grow-only device buffer per device; the
// device's lock is held from the upload until release() (the CRC batch that
// reads the copy has completed).
struct ImageCache {
    std::mutex mu;
    void* d = nullptr;
    size_t bytes = 0;
    hipStream_t st = nullptr;
};
std::mutex g_img_mu;
std::vector<std::unique_ptr<ImageCache>> g_img;

class ImageUpload {
  public:
    ImageUpload(const void* h, size_t bytes, int device) {
        int dev = device;  // resolved here: a new thread starts on device 0
        if (dev < 0 && hipGetDevice(&dev) != hipSuccess) dev = 0;
        th_ = std::thread([=] { rc_ = run(h, bytes, dev); });
    }
    ~ImageUpload() { release(); }
    // Wait for the copy; *d = the device image.
    int wait(const void** d) {
        if (th_.joinable()) th_.join();
        *d = cache_ ? cache_->d : nullptr;
        return rc_ ? fail(rc_, msg_.c_str()) : 0;  // the worker's error, reported on this thread
    }
    void release() {
        if (th_.joinable()) th_.join();
        if (lock_.owns_lock()) lock_.unlock();
    }

  private:
    int err(int code, const char* what) {
        msg_ = what;
        return code;
    }
    int run(const void* h, size_t bytes, int dev) {
        int n = 0;
        if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return err(KARMA_E_NO_DEVICE, "no HIP device visible");
        if (dev >= n || hipSetDevice(dev) != hipSuccess) return err(KARMA_E_INVALID, "wal image: bad device");
        {
            std::lock_guard<std::mutex> g(g_img_mu);
            if ((int)g_img.size() <= dev) g_img.resize(dev + 1);
            if (!g_img[dev]) g_img[dev] = std::make_unique<ImageCache>();
            cache_ = g_img[dev].get();
        }
        lock_ = std::unique_lock<std::mutex>(cache_->mu);
        ImageCache& ic = *cache_;
        if (!ic.st && hipStreamCreateWithFlags(&ic.st, hipStreamNonBlocking) != hipSuccess)
            return err(KARMA_E_HIP, "hipStreamCreate");
        if (ic.bytes < bytes) {
            if (ic.d) (void)hipFree(ic.d);
            ic.d = nullptr;
            ic.bytes = 0;
            if (hipMalloc(&ic.d, bytes) != hipSuccess) return err(KARMA_E_NOMEM, "wal image: hipMalloc");
            ic.bytes = bytes;
        }
        const bool reg = hipHostRegister(const_cast<void*>(h), bytes, hipHostRegisterDefault) == hipSuccess;
        if (!reg) (void)hipGetLastError();  // already pinned or not registrable: a staged copy still works
        hipError_t e = hipMemcpyAsync(ic.d, h, bytes, hipMemcpyHostToDevice, ic.st);
        if (e == hipSuccess) e = hipStreamSynchronize(ic.st);
        if (reg) (void)hipHostUnregister(const_cast<void*>(h));
        return e == hipSuccess ? 0 : err(KARMA_E_HIP, "wal image: H2D");
    }
    std::thread th_;
    int rc_ = 0;
    std::string msg_;
    ImageCache* cache_ = nullptr;
    std::unique_lock<std::mutex> lock_;
};

}  // namespace

extern "C" {

int karma_wal_append_batch(const void* h_src, const uint64_t* h_src_off, const uint32_t* h_len, size_t n,
                           void* h_wal, size_t wal_bytes, size_t seg_bytes, uint64_t* h_cursor, uint64_t* h_rec_off,
                           size_t* h_n_framed, int device) {
    if (!h_cursor || !h_n_framed || (n && (!h_src || !h_src_off || !h_len)) || !h_wal || seg_bytes < kHeader ||
        wal_bytes % seg_bytes)
        return fail(KARMA_E_INVALID, "wal_append_batch");
    uint8_t* wal = static_cast<uint8_t*>(h_wal);
    const uint8_t* src = static_cast<const uint8_t*>(h_src);
    karma::engine::PhaseTimer T("wal_append");
    // 1. CRCs of every payload: one GPU batch over the source buffer, on its own
    //    thread while the host places and frames the records (2, 3) around it.
    //    Records that end up not framed (image full) cost only their checksum.
    uint64_t extent = 0;  // source bytes the batch reads
    for (size_t i = 0; i < n; ++i) extent = std::max<uint64_t>(extent, h_src_off[i] + h_len[i]);
    std::vector<uint32_t> crc(n);
    int crc_rc = 0;
    std::thread gpu;
    if (n)
        gpu = std::thread([&, extent] {
            crc_rc = karma_crc32c_batch_ragged_host(src, extent, h_src_off, h_len, n, 0, crc.data(), device);
        });
    // 2. placement (sequential, cheap): can_hold or footer + next segment
    std::vector<uint64_t> at(n);
    uint64_t cur = *h_cursor;
    size_t framed = 0;
    std::vector<std::pair<uint64_t, uint64_t>> footers;  // (wal offset, segment end)
    uint64_t seg_end = (cur / seg_bytes + 1) * seg_bytes;  // end of the segment holding cur
    for (; framed < n; ++framed) {
        const uint64_t len = h_len[framed];
        if (len + kHeader > seg_bytes || (len >> 24)) break;  // never fits / 3-byte size field
        if (cur == seg_end) seg_end += seg_bytes;             // the last record filled its segment
        if (cur + kHeader + len > seg_end) {  // !can_hold -> append_footer, next segment
            footers.emplace_back(cur, seg_end);
            cur = seg_end;
            seg_end += seg_bytes;
        }
        if (cur + kHeader + len > wal_bytes) break;
        at[framed] = cur;
        cur += kHeader + len;
    }
    T.mark("placement");
    // 3. framing (segment_file::append_record / append_footer); the CRC fields last
    for (const auto& f : footers) {
        const uint64_t room = f.second - f.first;
        if (room < kHeader) {
            std::memset(wal + f.first, '0', room);
        } else {
            put32(wal + f.first, 0);
            put32(wal + f.first + 4, uint32_t((room - kHeader) << 8 | 1u));
            std::memset(wal + f.first + kHeader, '0', room - kHeader);
        }
    }
    const size_t nthr = std::min<size_t>(16, std::max<size_t>(1, framed / 4096));
    auto parallel = [&](auto&& body) {
        std::vector<std::thread> th;
        for (size_t t = 0; t < nthr; ++t) th.emplace_back(body, framed * t / nthr, framed * (t + 1) / nthr);
        for (auto& x : th) x.join();
    };
    parallel([&](size_t lo, size_t hi) {
        for (size_t i = lo; i < hi; ++i) {
            uint8_t* p = wal + at[i];
            put32(p + 4, h_len[i] << 8 | 0u);
            std::memcpy(p + kHeader, src + h_src_off[i], h_len[i]);
        }
    });
    T.mark("framing (payloads, lengths, footers)");
    if (gpu.joinable()) gpu.join();
    T.mark("wait for the CRC batch");
    if (crc_rc) return crc_rc;  // payloads and length fields are written; no CRC field is
    parallel([&](size_t lo, size_t hi) {
        for (size_t i = lo; i < hi; ++i) put32(wal + at[i], crc[i]);
    });
    if (h_rec_off)
        for (size_t i = 0; i < framed; ++i) h_rec_off[i] = at[i];
    *h_cursor = cur;
    *h_n_framed = framed;
    return 0;
}

int karma_wal_replay(const void* h_wal, const void* d_wal, size_t wal_bytes, size_t seg_bytes, uint64_t start,
                     uint64_t* h_n_records, uint64_t* h_stop, int* h_status, uint64_t* h_rec_off, size_t rec_cap,
                     int device) {
    if (!h_wal || !h_n_records || !h_stop || !h_status || seg_bytes < 1 || wal_bytes % seg_bytes || start > wal_bytes)
        return fail(KARMA_E_INVALID, "wal_replay");
    const uint8_t* wal = static_cast<const uint8_t*>(h_wal);
    const uint64_t nseg = wal_bytes / seg_bytes;
    const uint64_t s0 = std::min<uint64_t>(start / seg_bytes, nseg);
    const uint64_t nwork = nseg - s0;
    karma::engine::PhaseTimer T("wal_replay");
    // 0. no device copy given: upload the image while the headers are walked
    std::unique_ptr<ImageUpload> up;
    if (!d_wal && nwork) up = std::make_unique<ImageUpload>(wal + s0 * seg_bytes, nwork * seg_bytes, device);
    // 1. walk every segment from where replay would enter it, in parallel
    std::vector<std::vector<Cand>> cands(nseg);
    std::vector<uint64_t> stop(nseg);
    std::vector<int> kind(nseg);
    parallel_for(s0, nseg, 4, [&](uint64_t s) {
        const uint64_t base = s * seg_bytes;
        const uint64_t pos = s == s0 ? start - base : 0;
        kind[s] = walk_segment(wal + base, base, seg_bytes, pos, cands[s], &stop[s]);
    });
    T.mark("header walk");
    // replay enters segment s+1 only if segment s ended cleanly
    int status = 0;
    uint64_t end = nwork ? wal_bytes : start;
    uint64_t s1 = nseg;  // one past the last segment replay reads
    for (uint64_t s = s0; s < nseg; ++s)
        if (kind[s] != 0) {
            status = kind[s];
            end = stop[s];
            s1 = s + 1;
            break;
        }
    // candidate slots: gb = all candidates before segment s, nb = those with a payload
    std::vector<uint64_t> gb(nseg + 1, 0), nb(nseg + 1, 0);
    for (uint64_t s = s0; s < s1; ++s) {
        uint64_t nz = 0;
        for (const Cand& x : cands[s]) nz += x.len != 0;
        gb[s + 1] = gb[s] + cands[s].size();
        nb[s + 1] = nb[s] + nz;
    }
    const uint64_t n_all = gb[s1], n_nz = nb[s1];
    // 2. payload CRCs in one GPU batch (size-0 records were checked on the host)
    std::vector<uint64_t> off(n_nz);
    std::vector<uint32_t> len(n_nz);
    parallel_for(s0, s1, 8, [&](uint64_t s) {
        uint64_t j = nb[s];
        for (const Cand& x : cands[s])
            if (x.len) {
                off[j] = x.off;
                len[j] = x.len;
                ++j;
            }
    });
    T.mark("span lists");
    std::vector<uint32_t> got;
    if (up && off.empty()) {
        up->release();  // nothing to checksum: the upload (and any device error) does not matter
    } else if (up) {  // spans are WAL offsets; the uploaded copy starts at segment s0
        const void* d = nullptr;
        if (const int rc = up->wait(&d)) return rc;
        T.mark("image upload (rest of it)");
        const uint64_t base = s0 * seg_bytes;
        parallel_for(0, off.size(), 1 << 16, [&](uint64_t j) { off[j] -= base; });
        const int rc = karma::engine::crc_spans(wal + base, d, nwork * seg_bytes, off, len, got, device);
        up->release();
        if (rc) return rc;
    } else if (const int rc = karma::engine::crc_spans(h_wal, d_wal, wal_bytes, off, len, got, device)) {
        return rc;
    }
    T.mark("CRC batch");
    // 3. the first mismatch (in WAL order) is where scan_record logs "Corrupt record"
    std::vector<uint64_t> bad(nseg, UINT64_MAX);
    parallel_for(s0, s1, 8, [&](uint64_t s) {
        uint64_t j = nb[s];
        for (size_t i = 0; i < cands[s].size(); ++i) {
            const Cand& x = cands[s][i];
            if (x.len && got[j++] != x.stored) {
                bad[s] = gb[s] + i;
                return;
            }
        }
    });
    uint64_t accepted = n_all;
    for (uint64_t s = s0; s < s1; ++s)
        if (bad[s] != UINT64_MAX) {
            accepted = bad[s];
            status = KARMA_WAL_CORRUPT;
            end = cands[s][bad[s] - gb[s]].rec;
            break;
        }
    if (h_rec_off)
        parallel_for(s0, s1, 8, [&](uint64_t s) {
            for (size_t i = 0; i < cands[s].size(); ++i) {
                const uint64_t g = gb[s] + i;
                if (g < accepted && g < rec_cap) h_rec_off[g] = cands[s][i].rec;
            }
        });
    T.mark("compare + offsets");
    *h_n_records = accepted;
    *h_stop = end;
    *h_status = status;
    return 0;
}

}  // extern "C"
