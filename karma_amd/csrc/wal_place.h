// karma_amd/csrc/wal_place.h -- record placement of the WAL writer (library-internal;
// also compiled into tests/cpp/host_logic_test.cc under the sanitizers).
//
// sivir::build_sqe's loop (karma-store/sivir.cc:276-317): a record of L payload bytes
// goes at the cursor when the segment can hold it (segment_file::can_hold,
// segment_file.cc:74-77); otherwise the segment is closed with a footer
// (append_footer, :33-49: a type-1 padding record, or '0' bytes when fewer than 8
// remain) and the record starts the next segment.
#pragma once
#include <cstddef>
#include <cstdint>
#include <vector>

namespace karma::engine {

constexpr uint64_t kWalHeader = 8;  // store::RECORD_HEADER_LENGTH (common.h:11)

struct WalPlacer {
    uint64_t seg_bytes, wal_bytes, cur, seg_end;
    WalPlacer(uint64_t seg, uint64_t wal, uint64_t cursor)
        : seg_bytes(seg), wal_bytes(wal), cur(cursor), seg_end((cursor / seg + 1) * seg) {}
    // Places a record of L payload bytes.  When the segment has to be closed first,
    // [*f0, *f1) is the footer (else f0 == f1) and the cursor moves to the next segment.
    // Returns false when the record is not placed: it can never fit (L + 8 > seg_bytes, or
    // L >= 2^24: the 3-byte size field; no footer then) or the image is full (the footer,
    // if any, is still written, as the writer closes the segment before it runs out).
    bool place(uint64_t L, uint64_t* at, uint64_t* f0, uint64_t* f1) {
        *f0 = *f1 = 0;
        if (L + kWalHeader > seg_bytes || (L >> 24)) return false;
        if (cur == seg_end) seg_end += seg_bytes;  // the last record filled its segment exactly
        if (cur + kWalHeader + L > seg_end) {      // !can_hold -> append_footer, next segment
            *f0 = cur;
            *f1 = seg_end;
            cur = seg_end;
            seg_end += seg_bytes;
        }
        if (cur + kWalHeader + L > wal_bytes) return false;
        *at = cur;
        cur += kWalHeader + L;
        return true;
    }
};

// The same placement in run form, for a parallel writer.  With V(i) = sum_{j<i} (len_j + 8)
// (V(n_valid) the total, every len_j < n_valid valid: L + 8 <= seg_bytes and L < 2^24),
// records are placed in maximal runs that share a segment: run k holds records
// [i0, i1) at at[i] = base + V(i) (unsigned arithmetic).  Between runs the WalPlacer rules
// apply record by record (a footer, or no footer when a run filled its segment exactly;
// the image full), so the result -- every at[i], every footer, the cursor and the count
// placed -- is WalPlacer's (tests/cpp/host_logic_test.cc checks both on random batches).
// Each run's end is a binary search over V: O(segments x log n) instead of O(n).
struct WalRun {
    size_t i0, i1;
    uint64_t base;
};
struct WalFooter {
    uint64_t f0, f1;
};
template <typename VAt, typename LenAt>
size_t place_runs(uint64_t seg_bytes, uint64_t wal_bytes, uint64_t* cursor, size_t n_valid, VAt V, LenAt len,
                  std::vector<WalRun>* runs, std::vector<WalFooter>* footers) {
    uint64_t cur = *cursor, seg_end = (cur / seg_bytes + 1) * seg_bytes;
    size_t i = 0;
    while (i < n_valid) {
        const uint64_t L = len(i);
        if (cur == seg_end) seg_end += seg_bytes;       // the last run filled its segment exactly
        if (cur + kWalHeader + L > seg_end) {          // !can_hold -> append_footer, next segment
            footers->push_back(WalFooter{cur, seg_end});
            cur = seg_end;
            seg_end += seg_bytes;
        }
        if (cur + kWalHeader + L > wal_bytes) break;  // the image is full
        // records i .. j-1 fit at cur: cur + V(j) - V(i) <= seg_end (j = i + 1 does)
        const uint64_t vi = V(i);
        size_t lo = i + 1, hi = n_valid;  // the answer lies in [lo, hi]
        while (lo < hi) {
            const size_t mid = lo + (hi - lo + 1) / 2;
            if (cur + (V(mid) - vi) <= seg_end) lo = mid;
            else hi = mid - 1;
        }
        runs->push_back(WalRun{i, lo, cur - vi});
        cur += V(lo) - vi;
        i = lo;
    }
    *cursor = cur;
    return i;
}

}  // namespace karma::engine
