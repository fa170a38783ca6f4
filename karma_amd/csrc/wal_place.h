// karma_amd/csrc/wal_place.h -- record placement of the WAL writer (library-internal;
// also compiled into tests/cpp/host_logic_test.cc under the sanitizers).
//
// sivir::build_sqe's loop (karma-store/sivir.cc:276-317): a record of L payload bytes
// goes at the cursor when the segment can hold it (segment_file::can_hold,
// segment_file.cc:74-77); otherwise the segment is closed with a footer
// (append_footer, :33-49: a type-1 padding record, or '0' bytes when fewer than 8
// remain) and the record starts the next segment.
#pragma once
#include <cstdint>

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

}  // namespace karma::engine
