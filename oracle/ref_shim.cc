// oracle/ref_shim.cc -- TEST INFRASTRUCTURE ONLY.
//
// C entry points around the reference's own crc32c::Extend, compiled from the
// sources where they lie (/root/reference/karma-util/crc32c.cc + coding.cc) by
// oracle/Makefile into oracle/_ref/libkarma_ref_crc32c.so.  Used to generate
// tests/golden/ and as bench.py's cpu_baseline (kind "reference").  No
// reference source is copied into this repository.
#include <cstddef>
#include <cstring>
#include <cstdint>
#include <thread>
#include <vector>

#include "karma-util/crc32c.h"  // /root/reference/karma-util/crc32c.h:16

extern "C" {

uint32_t ref_crc32c_extend(uint32_t init_crc, const void* data, size_t n) {
    return crc32c::Extend(init_crc, static_cast<const char*>(data), n);
}

// CRC of n_rec fixed-size records laid out back to back in host memory, split
// round-robin over nthreads std::threads (the survey's CPU-baseline shape).
int ref_crc32c_fixed_mt(const void* base, uint64_t rec_bytes, uint64_t n_rec, uint32_t* out, int nthreads) {
    if (nthreads < 1) nthreads = 1;
    const char* b = static_cast<const char*>(base);
    std::vector<std::thread> th;
    for (int t = 0; t < nthreads; ++t)
        th.emplace_back([=] {
            for (uint64_t r = t; r < n_rec; r += nthreads) out[r] = crc32c::Value(b + r * rec_bytes, rec_bytes);
        });
    for (auto& x : th) x.join();
    return 0;
}

// Ragged records: out[r] = Extend(init ? init[r] : 0, base + off[r], len[r]).
int ref_crc32c_ragged_mt(const void* base, const uint64_t* off, const uint32_t* len, const uint32_t* init,
                         uint64_t n_rec, uint32_t* out, int nthreads) {
    if (nthreads < 1) nthreads = 1;
    const char* b = static_cast<const char*>(base);
    std::vector<std::thread> th;
    for (int t = 0; t < nthreads; ++t)
        th.emplace_back([=] {
            for (uint64_t r = t; r < n_rec; r += nthreads)
                out[r] = crc32c::Extend(init ? init[r] : 0u, b + off[r], len[r]);
        });
    for (auto& x : th) x.join();
    return 0;
}

// Config 1 harness: segment_file::append_record / append_footer
// framing (karma-store/segment_file.cc:21-49, can_hold :74-77) with the
// reference's crc32c::Value, as sivir::build_sqe drives it (sivir.cc:276-317).
// Thread t frames records [n*t/T, n*(t+1)/T) into its own WAL image
// wal + t*wal_bytes (each thread its own writer).  Returns records framed.
uint64_t ref_wal_append_mt(const void* src, const uint64_t* off, const uint32_t* len, uint64_t n, void* wal,
                           uint64_t wal_bytes, uint64_t seg, int nthreads) {
    if (nthreads < 1) nthreads = 1;
    const char* s = static_cast<const char*>(src);
    std::vector<uint64_t> done(nthreads, 0);
    std::vector<std::thread> th;
    for (int t = 0; t < nthreads; ++t)
        th.emplace_back([=, &done] {
            char* w = static_cast<char*>(wal) + (uint64_t)t * wal_bytes;
            uint64_t cur = 0, cnt = 0;
            for (uint64_t i = n * t / nthreads; i < n * (t + 1) / nthreads; ++i) {
                const uint64_t l = len[i];
                uint64_t seg_end = (cur / seg + 1) * seg;
                if (cur + 8 + l > seg_end) {  // append_footer
                    const uint64_t room = seg_end - cur;
                    if (room < 8) {
                        std::memset(w + cur, '0', room);
                    } else {
                        const uint32_t z = 0, st = uint32_t((room - 8) << 8 | 1u);
                        std::memcpy(w + cur, &z, 4);
                        std::memcpy(w + cur + 4, &st, 4);
                        std::memset(w + cur + 8, '0', room - 8);
                    }
                    cur = seg_end;
                }
                if (cur + 8 + l > wal_bytes) break;
                const uint32_t crc = crc32c::Value(s + off[i], l), st = uint32_t(l << 8);
                std::memcpy(w + cur, &crc, 4);
                std::memcpy(w + cur + 4, &st, 4);
                std::memcpy(w + cur + 8, s + off[i], l);
                cur += 8 + l;
                ++cnt;
            }
            done[t] = cnt;
        });
    for (auto& x : th) x.join();
    uint64_t total = 0;
    for (uint64_t d : done) total += d;
    return total;
}

// Replay harness: sivir::open's loop over wal::scan_record (sivir.cc:31-41,
// wal.cc:34-87) with the reference's crc32c::Value, over nimg independent WAL
// images of wal_bytes each, image i on thread i % nthreads.  Returns records
// accepted over all images.
uint64_t ref_wal_replay_mt(const void* wal, uint64_t wal_bytes, uint64_t seg, int nimg, int nthreads) {
    if (nthreads < 1) nthreads = 1;
    std::vector<uint64_t> done(nthreads, 0);
    std::vector<std::thread> th;
    for (int t = 0; t < nthreads; ++t)
        th.emplace_back([=, &done] {
            uint64_t cnt = 0;
            for (int im = t; im < nimg; im += nthreads) {
                const unsigned char* w = static_cast<const unsigned char*>(wal) + (uint64_t)im * wal_bytes;
                uint64_t off = 0;
                while (off < wal_bytes) {
                    const uint64_t base = off / seg * seg, pos = off - base;
                    if (pos + 8 > seg) {
                        off = base + seg;
                        continue;
                    }
                    uint32_t crc, st;
                    std::memcpy(&crc, w + off, 4);
                    std::memcpy(&st, w + off + 4, 4);
                    const uint32_t type = st & 0xff, size = st >> 8;
                    if (type == 1) {
                        off = base + seg;
                        continue;
                    }
                    if (type != 0 || pos + 8 + size > seg) break;
                    const char* data = reinterpret_cast<const char*>(size ? w + off + 8 : w + off + 4);
                    if (crc32c::Value(data, size ? size : 4) != crc) break;
                    ++cnt;
                    off += 8 + (size ? size : 4);  // record.size(): + the 4 stale bytes (wal.cc:66, sivir.cc:38)
                }
            }
            done[t] = cnt;
        });
    for (auto& x : th) x.join();
    uint64_t total = 0;
    for (uint64_t d : done) total += d;
    return total;
}

}  // extern "C"
