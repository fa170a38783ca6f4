// karma_amd/csrc/host_batch.cc -- batches whose bytes live in host memory
// (karma_crc32c_batch_fixed_host / _ragged_host): the path the north star
// measures end to end (io_uring-filled WAL buffers on write, segment pages on
// replay).
//
// Pageable caller memory is never page-locked per call: it is streamed into HBM
// through the library's persistent pinned staging buffers (host_stage.h), in
// slices of at most kSlice bytes, each slice checksummed by one device batch.
// Page-locked caller memory (hipHostMalloc'd, or registered once by its owner,
// e.g. io_uring fixed buffers) is DMAed directly, in 64 MiB chunks alternating
// over two streams so the H2D of chunk i+1 overlaps the kernel and D2H of
// chunk i.  Streams and device buffers are cached per device and reused by
// later calls (one call at a time per device; other threads wait on its lock).
#include <hip/hip_runtime_api.h>

#include <algorithm>
#include <cstring>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "engine.h"
#include "host_stage.h"
#include "host_trace.h"
#include "karma_crc32c.h"

namespace karma::engine {
int set_last_error(int code, const std::string& what);  // capi.cc
}

namespace {

using karma::engine::set_last_error;

constexpr size_t kChunkBytes = size_t(64) << 20;  // pinned caller memory: bytes per DMA chunk
constexpr size_t kSlice = size_t(1) << 30;        // pageable caller memory: bytes per staged slice
constexpr uint32_t kDirectMax = 1024;             // ragged records up to this: one record per group

int hip_fail(hipError_t e, const char* what) {
    return set_last_error(e == hipErrorOutOfMemory ? KARMA_E_NOMEM : KARMA_E_HIP,
                          std::string(what) + ": " + hipGetErrorString(e));
}

#define HB_HIP(expr)                                      \
    do {                                                  \
        hipError_t _e = (expr);                           \
        if (_e != hipSuccess) return hip_fail(_e, #expr); \
    } while (0)

// Grow-only device or pinned-host allocation.
struct Buf {
    void* p = nullptr;
    size_t bytes = 0;
    bool host = false;
    int ensure(size_t want, bool pinned_host) {
        if (bytes >= want && p) return 0;
        release();
        want = std::max<size_t>(want + want / 4, 256);
        hipError_t e = pinned_host ? hipHostMalloc(&p, want, hipHostMallocDefault) : hipMalloc(&p, want);
        if (e != hipSuccess) {
            p = nullptr;
            return hip_fail(e, pinned_host ? "hipHostMalloc" : "hipMalloc");
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

struct Slot {
    hipStream_t st = nullptr;
    hipEvent_t done = nullptr;
    Buf d_data, d_off, d_len, d_out;  // device
    Buf h_off, h_len, h_out;          // pinned host staging of the chunk's metadata / CRCs
    bool busy = false;                // work enqueued, results not yet collected
    size_t r0 = 0, nr = 0;            // the chunk's records
};

struct HostCtx {
    std::mutex mu;
    bool ready = false;
    Slot slot[2];
    int init(int dev) {
        if (ready) return 0;
        HB_HIP(hipSetDevice(dev));
        for (Slot& s : slot) {
            HB_HIP(hipStreamCreateWithFlags(&s.st, hipStreamNonBlocking));
            HB_HIP(hipEventCreateWithFlags(&s.done, hipEventDisableTiming));
        }
        ready = true;
        return 0;
    }
    void reset(int dev) {  // karma_crc32c_trim (the caller holds mu)
        if (!ready) return;
        for (Slot& s : slot) {
            (void)hipStreamSynchronize(s.st);
            (void)karma::engine::release_internal_stream(dev, s.st);
            for (Buf* b : {&s.d_data, &s.d_off, &s.d_len, &s.d_out, &s.h_off, &s.h_len, &s.h_out}) b->release();
            (void)hipEventDestroy(s.done);
            (void)hipStreamDestroy(s.st);
            s = Slot{};
        }
        ready = false;
    }
};

std::mutex g_ctx_mu;
std::vector<std::unique_ptr<HostCtx>> g_ctx;

HostCtx& ctx_for(int dev) {
    std::lock_guard<std::mutex> lk(g_ctx_mu);
    if ((int)g_ctx.size() <= dev) g_ctx.resize(dev + 1);
    if (!g_ctx[dev]) g_ctx[dev] = std::make_unique<HostCtx>();
    return *g_ctx[dev];
}

int pick_device(int device, int* dev) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return set_last_error(KARMA_E_NO_DEVICE, "no HIP device visible");
    if (device >= n) return set_last_error(KARMA_E_INVALID, "device index out of range");
    if (device >= 0) HB_HIP(hipSetDevice(device));
    HB_HIP(hipGetDevice(dev));
    return 0;
}

// Wait for a slot's chunk and hand its CRCs to the caller.
int collect(Slot& s, uint32_t* h_out) {
    if (!s.busy) return 0;
    s.busy = false;
    HB_HIP(hipEventSynchronize(s.done));
    std::memcpy(h_out + s.r0, s.h_out.p, s.nr * sizeof(uint32_t));
    return 0;
}

// Drain both slots (also on the error path, so no copy outlives the call).
int drain(HostCtx& c, uint32_t* h_out, int rc) {
    for (Slot& s : c.slot) {
        const int r = collect(s, h_out);
        if (!rc) rc = r;
    }
    return rc;
}

// Pinned caller memory: chunks DMAed straight from it, two streams in flight.
int fixed_pinned(HostCtx& c, const char* src, size_t rec_bytes, size_t n_rec, uint32_t init, uint32_t* h_out) {
    const size_t chunk = std::max<size_t>(1, kChunkBytes / std::max<size_t>(rec_bytes, 1));
    int rc = 0;
    for (size_t r0 = 0, i = 0; r0 < n_rec && !rc; r0 += chunk, ++i) {
        Slot& s = c.slot[i & 1];
        if ((rc = collect(s, h_out))) break;
        const size_t nr = std::min(chunk, n_rec - r0);
        if ((rc = s.d_data.ensure(std::max<size_t>(nr * rec_bytes, 16), false)) ||
            (rc = s.d_out.ensure(nr * sizeof(uint32_t), false)) || (rc = s.h_out.ensure(nr * sizeof(uint32_t), true)))
            break;
        hipError_t e = hipMemcpyAsync(s.d_data.p, src + r0 * rec_bytes, nr * rec_bytes, hipMemcpyHostToDevice, s.st);
        if (e != hipSuccess) {
            rc = hip_fail(e, "H2D");
            break;
        }
        if ((rc = karma_crc32c_batch_fixed(s.d_data.p, rec_bytes, nr, nullptr, init, s.d_out.as<uint32_t>(), s.st)))
            break;
        e = hipMemcpyAsync(s.h_out.p, s.d_out.p, nr * sizeof(uint32_t), hipMemcpyDeviceToHost, s.st);
        if (e == hipSuccess) e = hipEventRecord(s.done, s.st);
        if (e != hipSuccess) {
            rc = hip_fail(e, "D2H");
            break;
        }
        s.busy = true;
        s.r0 = r0;
        s.nr = nr;
    }
    return drain(c, h_out, rc);
}

}  // namespace

int karma::engine::trim_host_batch_ctx(int dev) {
    HostCtx& c = ctx_for(dev);
    std::lock_guard<std::mutex> lk(c.mu);
    c.reset(dev);
    return 0;
}

extern "C" {

int karma_crc32c_batch_fixed_host(const void* h_data, size_t rec_bytes, size_t n_rec, uint32_t init,
                                  uint32_t* h_out, int device) {
    if (n_rec == 0) return KARMA_OK;
    if (!h_out || (!h_data && rec_bytes)) return set_last_error(KARMA_E_INVALID, "batch_fixed_host: null pointer");
    int dev = 0;
    if (const int rc = pick_device(device, &dev)) return rc;
    HostCtx& c = ctx_for(dev);
    std::lock_guard<std::mutex> lk(c.mu);
    if (const int rc = c.init(dev)) return rc;
    const char* src = static_cast<const char*>(h_data);
    if (karma::engine::host_is_pinned(h_data)) return fixed_pinned(c, src, rec_bytes, n_rec, init, h_out);
    // pageable: slices of whole records streamed through the pinned staging
    Slot& s = c.slot[0];
    const size_t per = std::max<size_t>(1, kSlice / std::max<size_t>(rec_bytes, 1));
    for (size_t r0 = 0; r0 < n_rec; r0 += per) {
        const size_t nr = std::min(per, n_rec - r0);
        if (const int rc = s.d_data.ensure(std::max<size_t>(nr * rec_bytes, 16), false)) return rc;
        if (const int rc = s.d_out.ensure(nr * sizeof(uint32_t), false)) return rc;
        if (const int rc = karma::engine::staged_copy(dev, s.d_data.p, src + r0 * rec_bytes, nr * rec_bytes)) return rc;
        if (const int rc = karma_crc32c_batch_fixed(s.d_data.p, rec_bytes, nr, nullptr, init, s.d_out.as<uint32_t>(),
                                                    s.st))
            return rc;
        HB_HIP(hipMemcpyAsync(h_out + r0, s.d_out.p, nr * sizeof(uint32_t), hipMemcpyDeviceToHost, s.st));
        HB_HIP(hipStreamSynchronize(s.st));
    }
    return KARMA_OK;
}

int karma_crc32c_batch_ragged_host(const void* h_arena, size_t arena_bytes, const uint64_t* h_off,
                                   const uint32_t* h_len, size_t n_rec, uint32_t init, uint32_t* h_out, int device) {
    if (n_rec == 0) return KARMA_OK;
    if (!h_out || !h_off || !h_len || (!h_arena && arena_bytes))
        return set_last_error(KARMA_E_INVALID, "batch_ragged_host: null pointer");
    karma::engine::PhaseTimer T("ragged_host");
    bool monotone = true;
    for (size_t r = 0; r < n_rec; ++r) {
        if (h_off[r] + h_len[r] > arena_bytes)
            return set_last_error(KARMA_E_INVALID, "batch_ragged_host: record past arena");
        if (r && h_off[r] < h_off[r - 1]) monotone = false;
    }
    int dev = 0;
    if (const int rc = pick_device(device, &dev)) return rc;
    HostCtx& c = ctx_for(dev);
    std::lock_guard<std::mutex> lk(c.mu);
    if (const int rc = c.init(dev)) return rc;
    T.mark("validate");
    const char* src = static_cast<const char*>(h_arena);
    const bool pinned = karma::engine::host_is_pinned(h_arena);
    // Two slots on two streams, as the fixed path: slice i + 1's upload (a DMA from pinned caller
    // memory, or the staging threads' copy from pageable memory) runs while slice i's kernel and
    // CRC download are in flight on the other stream; a slot is collected before it is reused.
    int rc = 0;
    size_t i = 0;
    for (size_t r0 = 0; r0 < n_rec && !rc; ++i) {
        Slot& s = c.slot[i & 1];
        if ((rc = collect(s, h_out))) break;
        // slice = records [r0, r1) whose bytes span [lo, hi) <= kSlice (at least one record);
        // offsets out of order: one slice over every record
        uint64_t lo = h_off[r0], hi = h_off[r0] + h_len[r0];
        uint32_t max_len = h_len[r0];
        size_t r1 = r0 + 1;
        for (; r1 < n_rec; ++r1) {
            const uint64_t l2 = std::min<uint64_t>(lo, h_off[r1]), h2 = std::max<uint64_t>(hi, h_off[r1] + h_len[r1]);
            if (monotone && h2 - l2 > kSlice) break;
            lo = l2;
            hi = h2;
            max_len = std::max(max_len, h_len[r1]);
        }
        const size_t nr = r1 - r0;
        if ((rc = s.d_data.ensure(std::max<uint64_t>(hi - lo, 16), false)) ||
            (rc = s.d_off.ensure(nr * sizeof(uint64_t), false)) || (rc = s.d_len.ensure(nr * sizeof(uint32_t), false)) ||
            (rc = s.d_out.ensure(nr * sizeof(uint32_t), false)) || (rc = s.h_off.ensure(nr * sizeof(uint64_t), true)) ||
            (rc = s.h_len.ensure(nr * sizeof(uint32_t), true)) || (rc = s.h_out.ensure(nr * sizeof(uint32_t), true)))
            break;
        uint64_t* ho = s.h_off.as<uint64_t>();
        uint64_t total = 0;
        for (size_t k = 0; k < nr; ++k) {
            ho[k] = h_off[r0 + k] - lo;  // rebased onto the slice's device copy
            total += h_len[r0 + k];
        }
        std::memcpy(s.h_len.p, h_len + r0, nr * sizeof(uint32_t));
        hipError_t e = hipMemcpyAsync(s.d_off.p, s.h_off.p, nr * sizeof(uint64_t), hipMemcpyHostToDevice, s.st);
        if (e == hipSuccess) e = hipMemcpyAsync(s.d_len.p, s.h_len.p, nr * sizeof(uint32_t), hipMemcpyHostToDevice, s.st);
        if (e == hipSuccess && pinned) e = hipMemcpyAsync(s.d_data.p, src + lo, hi - lo, hipMemcpyHostToDevice, s.st);
        if (e != hipSuccess) {
            rc = hip_fail(e, "ragged_host: H2D");
            break;
        }
        if (!pinned && (rc = karma::engine::staged_copy(dev, s.d_data.p, src + lo, hi - lo))) break;
        T.mark("upload");
        if ((rc = karma_crc32c_batch_ragged_bounded(s.d_data.p, s.d_off.as<uint64_t>(), s.d_len.as<uint32_t>(), nr, total,
                                                    max_len, nullptr, init, s.d_out.as<uint32_t>(), s.st)))
            break;
        e = hipMemcpyAsync(s.h_out.p, s.d_out.p, nr * sizeof(uint32_t), hipMemcpyDeviceToHost, s.st);
        if (e == hipSuccess) e = hipEventRecord(s.done, s.st);
        if (e != hipSuccess) {
            rc = hip_fail(e, "ragged_host: D2H");
            break;
        }
        s.busy = true;
        s.r0 = r0;
        s.nr = nr;
        r0 = r1;
    }
    rc = drain(c, h_out, rc);
    T.mark("batches + D2H");
    return rc;
}

}  // extern "C"
