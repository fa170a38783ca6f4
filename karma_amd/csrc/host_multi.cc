// karma_amd/csrc/host_multi.cc -- host-memory batches over several devices of one process
// (include/karma_crc32c.h: karma_crc32c_batch_fixed_host_multi, _ragged_host_multi,
// karma_wal_replay_multi).  The split and the ordered merge are multi_dev.h; each share runs the
// one-device entry point on a host thread of its own, so every device's PCIe link, staging buffers
// and streams work at once.  The batching points these serve: sivir::build_sqe draining a batch
// (sivir.cc:276-317) and sivir::open's replay (sivir.cc:31-41).
#include <hip/hip_runtime_api.h>

#include <algorithm>
#include <cstring>
#include <string>
#include <vector>

#include "karma_crc32c.h"
#include "multi_dev.h"

namespace karma::engine {
int set_last_error(int code, const std::string& what);  // capi.cc
}

namespace {

using karma::engine::set_last_error;

int check_devices(const int* devices, int n_dev, const char* fn) {
    if (!devices || n_dev < 1) return set_last_error(KARMA_E_INVALID, std::string(fn) + ": no devices");
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess || count <= 0) return set_last_error(KARMA_E_NO_DEVICE, "no HIP device visible");
    for (int k = 0; k < n_dev; ++k)
        if (devices[k] < 0 || devices[k] >= count)
            return set_last_error(KARMA_E_INVALID, std::string(fn) + ": device index out of range");
    return 0;
}

std::string detail() { return karma_crc32c_last_error(); }

}  // namespace

extern "C" {

int karma_crc32c_batch_fixed_host_multi(const void* h_data, size_t rec_bytes, size_t n_rec, uint32_t init,
                                        uint32_t* h_out, const int* devices, int n_dev) {
    if (const int rc = check_devices(devices, n_dev, "batch_fixed_host_multi")) return rc;
    if (n_rec == 0) return KARMA_OK;
    if (!h_out || (!h_data && rec_bytes)) return set_last_error(KARMA_E_INVALID, "batch_fixed_host_multi: null pointer");
    const int parts = (int)std::min<size_t>((size_t)n_dev, n_rec);
    const char* src = static_cast<const char*>(h_data);
    std::string what;
    const int rc = karma::engine::run_shares(
        parts,
        [&](int k) {
            const size_t lo = karma::engine::share_lo(n_rec, parts, k), hi = karma::engine::share_lo(n_rec, parts, k + 1);
            return karma_crc32c_batch_fixed_host(src + lo * rec_bytes, rec_bytes, hi - lo, init, h_out + lo, devices[k]);
        },
        detail, &what);
    return rc ? set_last_error(rc, what) : KARMA_OK;
}

int karma_crc32c_batch_ragged_host_multi(const void* h_arena, size_t arena_bytes, const uint64_t* h_off,
                                         const uint32_t* h_len, size_t n_rec, uint32_t init, uint32_t* h_out,
                                         const int* devices, int n_dev) {
    if (const int rc = check_devices(devices, n_dev, "batch_ragged_host_multi")) return rc;
    if (n_rec == 0) return KARMA_OK;
    if (!h_out || !h_off || !h_len || (!h_arena && arena_bytes))
        return set_last_error(KARMA_E_INVALID, "batch_ragged_host_multi: null pointer");
    const int parts = (int)std::min<size_t>((size_t)n_dev, n_rec);
    const std::vector<size_t> cuts = karma::engine::byte_balanced_cuts(h_len, n_rec, parts);
    std::string what;
    const int rc = karma::engine::run_shares(
        parts,
        [&](int k) {
            const size_t lo = cuts[k], hi = cuts[k + 1];
            if (hi == lo) return 0;
            return karma_crc32c_batch_ragged_host(h_arena, arena_bytes, h_off + lo, h_len + lo, hi - lo, init, h_out + lo,
                                                  devices[k]);
        },
        detail, &what);
    return rc ? set_last_error(rc, what) : KARMA_OK;
}

int karma_wal_replay_multi(const void* h_wal, size_t wal_bytes, size_t seg_bytes, uint64_t start, uint64_t* h_n_records,
                           uint64_t* h_stop, int* h_status, uint64_t* h_rec_off, size_t rec_cap, const int* devices,
                           int n_dev) {
    if (const int rc = check_devices(devices, n_dev, "wal_replay_multi")) return rc;
    if (!h_wal || !h_n_records || !h_stop || !h_status || seg_bytes < 1 || wal_bytes % seg_bytes ||
        start > wal_bytes + 4 || seg_bytes >= (uint64_t(1) << 31))
        return set_last_error(KARMA_E_INVALID, "wal_replay_multi");
    const uint8_t* img = static_cast<const uint8_t*>(h_wal);
    std::vector<karma::engine::ReplayShare> sh = karma::engine::replay_shares(wal_bytes, seg_bytes, start, n_dev);
    if (sh.size() <= 1 || start >= wal_bytes)
        return karma_wal_replay(h_wal, nullptr, wal_bytes, seg_bytes, start, h_n_records, h_stop, h_status, h_rec_off,
                                rec_cap, devices[0]);
    // share k replayed from the absolute offset `from` (its lo, or a stop a spill carried 1-4 bytes
    // into its first segment), on its own device
    auto replay_share = [&](int k, uint64_t from) {
        karma::engine::ReplayShare& s = sh[k];
        const uint64_t bytes = s.hi - s.lo;
        s.start = from;
        s.rec.assign(h_rec_off ? std::min<uint64_t>(rec_cap, bytes / 8 + 2) : 0, 0);
        const int r = karma_wal_replay(img + s.lo, nullptr, bytes, seg_bytes, s.start - s.lo, &s.n, &s.stop, &s.status,
                                       s.rec.empty() ? nullptr : s.rec.data(), s.rec.size(), devices[k]);
        if (r) return r;
        s.stop += s.lo;
        if (s.rec.size() > s.n) s.rec.resize(s.n);
        for (uint64_t& o : s.rec) o += s.lo;
        return 0;
    };
    std::string what;
    const int parts = (int)sh.size();
    int rc = karma::engine::run_shares(parts, [&](int k) { return replay_share(k, sh[k].start); }, detail, &what);
    if (rc) return set_last_error(rc, what);
    int redo_rc = 0;
    const int end = karma::engine::merge_replays(
        sh, h_n_records, h_stop, h_status, h_rec_off, rec_cap, KARMA_WAL_END,
        [&](int k, uint64_t from) { return replay_share(k, from); }, &redo_rc);
    if (end < 0) return set_last_error(redo_rc, "wal_replay_multi: share replayed after a size-0 spill: " + detail());
    return KARMA_OK;
}

}  // extern "C"
