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
#include <string>
#include <thread>
#include <vector>

#include "karma-util/crc32c.h"
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
    // 1. placement (sequential, cheap): can_hold or footer + next segment
    std::vector<uint64_t> at(n);
    uint64_t cur = *h_cursor;
    size_t framed = 0;
    std::vector<std::pair<uint64_t, uint64_t>> footers;  // (wal offset, segment end)
    for (; framed < n; ++framed) {
        const uint64_t len = h_len[framed];
        if (len + kHeader > seg_bytes || (len >> 24)) break;  // never fits / 3-byte size field
        uint64_t seg_end = (cur / seg_bytes + 1) * seg_bytes;
        if (cur + kHeader + len > seg_end) {  // !can_hold -> append_footer, next segment
            footers.emplace_back(cur, seg_end);
            cur = seg_end;
            seg_end += seg_bytes;
        }
        if (cur + kHeader + len > wal_bytes) break;
        at[framed] = cur;
        cur += kHeader + len;
    }
    // 2. CRCs of the framed payloads: one GPU batch over the source buffer, on its
    //    own thread while the host threads frame the records (3) around it
    std::vector<uint32_t> crc(framed);
    int crc_rc = 0;
    std::thread gpu;
    if (framed) {
        uint64_t extent = 0;
        for (size_t i = 0; i < framed; ++i) extent = std::max<uint64_t>(extent, h_src_off[i] + h_len[i]);
        gpu = std::thread([&, extent] {
            crc_rc = karma_crc32c_batch_ragged_host(src, extent, h_src_off, h_len, framed, 0, crc.data(), device);
        });
    }
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
    if (gpu.joinable()) gpu.join();
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
    const uint64_t s0 = start / seg_bytes;
    // 1. walk every segment from where replay would enter it, in parallel
    std::vector<std::vector<Cand>> cands(nseg);
    std::vector<uint64_t> stop(nseg);
    std::vector<int> kind(nseg);
    auto walk = [&](uint64_t lo, uint64_t hi) {
        for (uint64_t s = lo; s < hi; ++s) {
            const uint64_t base = s * seg_bytes;
            const uint64_t pos = s == s0 ? start - base : 0;
            kind[s] = walk_segment(wal + base, base, seg_bytes, pos, cands[s], &stop[s]);
        }
    };
    const uint64_t nwork = nseg - std::min(nseg, s0);
    const uint64_t nthr = std::min<uint64_t>(16, std::max<uint64_t>(1, nwork / 4));
    std::vector<std::thread> th;
    for (uint64_t t = 0; t < nthr; ++t) th.emplace_back(walk, s0 + nwork * t / nthr, s0 + nwork * (t + 1) / nthr);
    for (auto& x : th) x.join();
    // replay enters segment s+1 only if segment s ended cleanly
    std::vector<Cand> all;
    int status = 0;
    uint64_t end = wal_bytes;
    for (uint64_t s = s0; s < nseg; ++s) {
        all.insert(all.end(), cands[s].begin(), cands[s].end());
        if (kind[s] != 0) {
            status = kind[s];
            end = stop[s];
            break;
        }
    }
    if (s0 >= nseg) end = start;
    // 2. payload CRCs in one GPU batch (size-0 records were checked on the host)
    std::vector<uint64_t> off;
    std::vector<uint32_t> len;
    std::vector<size_t> idx;
    for (size_t i = 0; i < all.size(); ++i)
        if (all[i].len) {
            off.push_back(all[i].off);
            len.push_back(all[i].len);
            idx.push_back(i);
        }
    std::vector<uint32_t> got(off.size());
    if (const int rc = karma::engine::crc_spans(h_wal, d_wal, wal_bytes, off, len, got, device)) return rc;
    // 3. the first mismatch (in WAL order) is where scan_record logs "Corrupt record"
    size_t accepted = all.size();
    for (size_t j = 0; j < idx.size(); ++j)
        if (got[j] != all[idx[j]].stored) {
            accepted = idx[j];
            status = KARMA_WAL_CORRUPT;
            end = all[idx[j]].rec;
            break;
        }
    if (h_rec_off)
        for (size_t i = 0; i < accepted && i < rec_cap; ++i) h_rec_off[i] = all[i].rec;
    *h_n_records = accepted;
    *h_stop = end;
    *h_status = status;
    return 0;
}

}  // extern "C"
