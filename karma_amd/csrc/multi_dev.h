// karma_amd/csrc/multi_dev.h -- one host batch spread over several devices of this process
// (karma_crc32c_batch_fixed_host_multi, karma_crc32c_batch_ragged_host_multi,
// karma_wal_replay_multi; include/karma_crc32c.h).
//
// From host memory one device is bound by its PCIe link (~50 GiB/s); records are
// independent (karma-store/segment_file.cc:22, wal.cc:60), so a batch is split into contiguous
// record (or segment) ranges, one per device, each streamed over its own link by the one-device
// entry point on a host thread of its own, the results written in record order.
//
// Templated on the one-device call, so tests/cpp/host_logic_test.cc drives the range arithmetic
// and the ordered merge under ASan through stubs (as gather_p2p.h is tested); host_multi.cc
// instantiates it with the library's one-device entry points.
#pragma once
#include <cstddef>
#include <cstdint>
#include <string>
#include <thread>
#include <vector>

namespace karma::engine {

// Share k of n items over parts: [n k / parts, n (k + 1) / parts).
inline size_t share_lo(size_t n, int parts, int k) { return (size_t)((unsigned __int128)n * (unsigned)k / (unsigned)parts); }

// Record ranges of equal byte counts (lengths in record order): cut k is the first record whose
// inclusive byte prefix reaches total * k / parts.  cuts has parts + 1 entries, cuts[0] = 0,
// cuts[parts] = n, non-decreasing.
inline std::vector<size_t> byte_balanced_cuts(const uint32_t* len, size_t n, int parts) {
    uint64_t total = 0;
    for (size_t r = 0; r < n; ++r) total += len[r];
    std::vector<size_t> cuts(parts + 1, n);
    cuts[0] = 0;
    uint64_t acc = 0;
    int k = 1;
    for (size_t r = 0; r < n && k < parts; ++r) {
        acc += len[r];
        while (k < parts && acc * (uint64_t)parts >= total * (uint64_t)k) cuts[k++] = r + 1;
    }
    for (; k < parts; ++k) cuts[k] = n;
    return cuts;
}

// Runs one(k) for k in [0, parts) on one host thread each (k = 0 on the caller's) and returns the
// first nonzero status in k order; *what gets that share's error detail (the one-device calls
// report theirs per thread: karma_crc32c_last_error).
template <class One, class Detail>
int run_shares(int parts, One&& one, Detail&& detail, std::string* what) {
    std::vector<int> rc(parts, 0);
    std::vector<std::string> msg(parts);
    std::vector<std::thread> th;
    for (int k = 1; k < parts; ++k)
        th.emplace_back([&, k] {
            rc[k] = one(k);
            if (rc[k]) msg[k] = detail();
        });
    rc[0] = one(0);
    if (rc[0]) msg[0] = detail();
    for (auto& t : th) t.join();
    for (int k = 0; k < parts; ++k)
        if (rc[k]) {
            if (what) *what = "device share " + std::to_string(k) + ": " + msg[k];
            return rc[k];
        }
    return 0;
}

// One device's replay of a range of segments (offsets relative to the whole image).
struct ReplayShare {
    uint64_t lo = 0, hi = 0;  // bytes of the image this share walks: [lo, hi), whole segments
    uint64_t start = 0;       // where its replay starts (lo, or the caller's start in share 0)
    uint64_t n = 0, stop = 0;
    int status = 0;
    std::vector<uint64_t> rec;  // its records' header offsets (relative to the whole image)
};

// The segments from start's segment to the image end, split into contiguous ranges.
inline std::vector<ReplayShare> replay_shares(uint64_t wal_bytes, uint64_t seg_bytes, uint64_t start, int parts) {
    const uint64_t nseg = wal_bytes / seg_bytes, s0 = start / seg_bytes;
    const uint64_t rest = nseg > s0 ? nseg - s0 : 0;
    if ((uint64_t)parts > rest) parts = rest ? (int)rest : 1;
    std::vector<ReplayShare> sh(parts);
    for (int k = 0; k < parts; ++k) {
        sh[k].lo = (s0 + share_lo(rest, parts, k)) * seg_bytes;
        sh[k].hi = (s0 + share_lo(rest, parts, k + 1)) * seg_bytes;
        sh[k].start = k ? sh[k].lo : start;
    }
    return sh;
}

// sivir::open's loop (sivir.cc:31-41) over the shares in order: a share's records count only when
// every share before it walked to its range's end and stopped there cleanly (END at its hi: the
// chain entered the next range at a segment start, as the shares assumed).  When a share stops
// cleanly PAST its range (an accepted size-0 record carried the chain 1-4 bytes into the next
// segment, wal.cc:66), only the next share is replayed again, from that stop: redo(k, start)
// re-runs share k from the absolute offset `start` (inside its first segment) and updates sh[k],
// returning a KARMA status.  The shares after it stay valid as long as the redone share ends at
// its own hi again, so each spill costs one share replay.  Returns the index of the share whose
// stop ends replay, or -1 when a redo failed (*redo_rc = its status).  *n, *stop, *status: the
// merged result.
template <class Redo>
inline int merge_replays(std::vector<ReplayShare>& sh, uint64_t* n, uint64_t* stop, int* status, uint64_t* rec_off,
                         size_t rec_cap, int end_status, Redo&& redo, int* redo_rc) {
    *n = 0;
    *redo_rc = 0;
    for (size_t k = 0; k < sh.size(); ++k) {
        const ReplayShare& s = sh[k];
        for (uint64_t i = 0; i < s.n; ++i) {
            if (rec_off && *n + i < rec_cap && i < s.rec.size()) rec_off[*n + i] = s.rec[i];
        }
        *n += s.n;
        *stop = s.stop;
        *status = s.status;
        const bool last = k + 1 == sh.size();
        if (s.status != end_status || s.stop < s.hi || last) return (int)k;
        if (s.stop > s.hi) {  // carried into the next share's range past its start: redo that share
            if (const int rc = redo((int)k + 1, s.stop)) {
                *redo_rc = rc;
                return -1;
            }
        }
    }
    return (int)sh.size() - 1;
}

}  // namespace karma::engine
