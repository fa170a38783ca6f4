// karma_amd/csrc/host_batch.cc -- batches whose bytes live in host memory
// (karma_crc32c_batch_fixed_host / _ragged_host): the path the north star
// measures end to end (io_uring-filled WAL buffers on write, segment pages on
// replay).
//
// The caller's buffer is page-locked for the call (hipHostRegister, skipped if
// it is already pinned) so every H2D copy is a DMA straight from it.  Work is
// cut into chunks of <= kStageBytes and alternates over two streams: the H2D
// of chunk i+1 overlaps the kernel and D2H of chunk i.  Streams, events and
// device slots are cached per device and reused by later calls (one call at a
// time per device; callers on other threads wait on the device's lock).
#include <hip/hip_runtime_api.h>

#include <algorithm>
#include <cstring>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "host_trace.h"
#include "karma_crc32c.h"

namespace karma::engine {
int set_last_error(int code, const std::string& what);  // capi.cc
}

namespace {

constexpr size_t kStageBytes = size_t(64) << 20;  // bytes per chunk and slot

int hip_fail(hipError_t e, const char* what) {
    return karma::engine::set_last_error(e == hipErrorOutOfMemory ? KARMA_E_NOMEM : KARMA_E_HIP,
                                         std::string(what) + ": " + hipGetErrorString(e));
}

#define HB_HIP(expr)                                      \
    do {                                                  \
        hipError_t _e = (expr);                           \
        if (_e != hipSuccess) return hip_fail(_e, #expr); \
    } while (0)

struct HostPin {
    void* p = nullptr;
    bool registered = false;
    HostPin(const void* ptr, size_t bytes) {
        hipPointerAttribute_t attr;
        if (!ptr || !bytes) return;
        if (hipPointerGetAttributes(&attr, ptr) == hipSuccess && attr.type == hipMemoryTypeHost) return;  // pinned
        (void)hipGetLastError();
        if (hipHostRegister(const_cast<void*>(ptr), bytes, hipHostRegisterDefault) == hipSuccess) {
            p = const_cast<void*>(ptr);
            registered = true;
        } else {
            (void)hipGetLastError();  // pageable copies still work, staged by the runtime
        }
    }
    ~HostPin() {
        if (registered) (void)hipHostUnregister(p);
    }
};

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
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0)
        return karma::engine::set_last_error(KARMA_E_NO_DEVICE, "no HIP device visible");
    if (device >= n) return karma::engine::set_last_error(KARMA_E_INVALID, "device index out of range");
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

}  // namespace

extern "C" {

int karma_crc32c_batch_fixed_host(const void* h_data, size_t rec_bytes, size_t n_rec, uint32_t init,
                                  uint32_t* h_out, int device) {
    if (n_rec == 0) return KARMA_OK;
    if (!h_out || (!h_data && rec_bytes))
        return karma::engine::set_last_error(KARMA_E_INVALID, "batch_fixed_host: null pointer");
    int dev = 0;
    if (const int rc = pick_device(device, &dev)) return rc;
    HostCtx& c = ctx_for(dev);
    std::lock_guard<std::mutex> lk(c.mu);
    if (const int rc = c.init(dev)) return rc;
    const size_t chunk = std::max<size_t>(1, rec_bytes ? kStageBytes / std::max<size_t>(rec_bytes, 1) : n_rec);
    HostPin pin(h_data, n_rec * rec_bytes);
    const char* src = static_cast<const char*>(h_data);
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
        if ((rc = karma_crc32c_batch_fixed(s.d_data.p, rec_bytes, nr, nullptr, init, static_cast<uint32_t*>(s.d_out.p),
                                           s.st)))
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

int karma_crc32c_batch_ragged_host(const void* h_arena, size_t arena_bytes, const uint64_t* h_off,
                                   const uint32_t* h_len, size_t n_rec, uint32_t init, uint32_t* h_out, int device) {
    if (n_rec == 0) return KARMA_OK;
    if (!h_out || !h_off || !h_len || (!h_arena && arena_bytes))
        return karma::engine::set_last_error(KARMA_E_INVALID, "batch_ragged_host: null pointer");
    karma::engine::PhaseTimer T("ragged_host");
    bool monotone = true;
    for (size_t r = 0; r < n_rec; ++r) {
        if (h_off[r] + h_len[r] > arena_bytes)
            return karma::engine::set_last_error(KARMA_E_INVALID, "batch_ragged_host: record past arena");
        if (r && h_off[r] < h_off[r - 1]) monotone = false;
    }
    int dev = 0;
    if (const int rc = pick_device(device, &dev)) return rc;
    HostCtx& c = ctx_for(dev);
    std::lock_guard<std::mutex> lk(c.mu);
    if (const int rc = c.init(dev)) return rc;
    T.mark("validate");
    HostPin pin(h_arena, arena_bytes);
    T.mark("hipHostRegister");
    const char* src = static_cast<const char*>(h_arena);
    int rc = 0;
    size_t r0 = 0;
    for (size_t i = 0; r0 < n_rec && !rc; ++i) {
        // chunk = records [r0, r1) whose bytes span [lo, hi) <= kStageBytes (at least one
        // record); offsets out of order: one chunk over every record
        uint64_t lo = h_off[r0], hi = h_off[r0] + h_len[r0];
        size_t r1 = r0 + 1;
        if (monotone) {
            while (r1 < n_rec && std::max<uint64_t>(hi, h_off[r1] + h_len[r1]) - lo <= kStageBytes) {
                hi = std::max<uint64_t>(hi, h_off[r1] + h_len[r1]);
                ++r1;
            }
        } else {
            for (; r1 < n_rec; ++r1) {
                lo = std::min<uint64_t>(lo, h_off[r1]);
                hi = std::max<uint64_t>(hi, h_off[r1] + h_len[r1]);
            }
        }
        const size_t nr = r1 - r0;
        Slot& s = c.slot[i & 1];
        if ((rc = collect(s, h_out))) break;
        if ((rc = s.d_data.ensure(std::max<uint64_t>(hi - lo, 16), false)) ||
            (rc = s.d_off.ensure(nr * sizeof(uint64_t), false)) || (rc = s.d_len.ensure(nr * sizeof(uint32_t), false)) ||
            (rc = s.d_out.ensure(nr * sizeof(uint32_t), false)) || (rc = s.h_off.ensure(nr * sizeof(uint64_t), true)) ||
            (rc = s.h_len.ensure(nr * sizeof(uint32_t), true)) || (rc = s.h_out.ensure(nr * sizeof(uint32_t), true)))
            break;
        uint64_t* ho = static_cast<uint64_t*>(s.h_off.p);
        uint64_t total = 0;
        for (size_t k = 0; k < nr; ++k) {
            ho[k] = h_off[r0 + k] - lo;  // rebased onto the chunk's device copy
            total += h_len[r0 + k];
        }
        std::memcpy(s.h_len.p, h_len + r0, nr * sizeof(uint32_t));
        hipError_t e = hipMemcpyAsync(s.d_data.p, src + lo, hi - lo, hipMemcpyHostToDevice, s.st);
        if (e == hipSuccess) e = hipMemcpyAsync(s.d_off.p, s.h_off.p, nr * sizeof(uint64_t), hipMemcpyHostToDevice, s.st);
        if (e == hipSuccess) e = hipMemcpyAsync(s.d_len.p, s.h_len.p, nr * sizeof(uint32_t), hipMemcpyHostToDevice, s.st);
        if (e != hipSuccess) {
            rc = hip_fail(e, "H2D");
            break;
        }
        if ((rc = karma_crc32c_batch_ragged(s.d_data.p, static_cast<uint64_t*>(s.d_off.p),
                                            static_cast<uint32_t*>(s.d_len.p), nr, total, nullptr, init,
                                            static_cast<uint32_t*>(s.d_out.p), s.st)))
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
        r0 = r1;
    }
    T.mark("enqueue chunks");
    rc = drain(c, h_out, rc);
    T.mark("drain");
    return rc;
}

}  // extern "C"
