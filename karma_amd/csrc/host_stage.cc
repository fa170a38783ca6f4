// karma_amd/csrc/host_stage.cc -- pinned staging uploads (host_stage.h).
#include "host_stage.h"

#include <algorithm>
#include <condition_variable>
#include <cstring>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "karma_crc32c.h"

namespace karma::engine {
int set_last_error(int code, const std::string& what);  // capi.cc

namespace {

constexpr int kWorkers = 8;                  // copy threads, one DMA stream each
constexpr size_t kChunk = size_t(8) << 20;   // bytes per pinned buffer (two per worker)

struct Stage {
    std::mutex mu;
    bool ready = false;
    hipStream_t st[kWorkers] = {};
    hipEvent_t ev[kWorkers][2] = {};
    void* buf[kWorkers][2] = {};
    int init() {
        if (ready) return 0;
        for (int t = 0; t < kWorkers; ++t) {
            if (hipStreamCreateWithFlags(&st[t], hipStreamNonBlocking) != hipSuccess)
                return set_last_error(KARMA_E_HIP, "staging: stream");
            for (int k = 0; k < 2; ++k) {
                if (hipEventCreateWithFlags(&ev[t][k], hipEventDisableTiming) != hipSuccess)
                    return set_last_error(KARMA_E_HIP, "staging: event");
                if (hipHostMalloc(&buf[t][k], kChunk, hipHostMallocDefault) != hipSuccess) {
                    buf[t][k] = nullptr;
                    return set_last_error(KARMA_E_NOMEM, "staging: pinned buffer");
                }
            }
        }
        ready = true;
        return 0;
    }
    void reset() {  // karma_crc32c_trim (the caller holds mu)
        if (!ready) return;
        for (int t = 0; t < kWorkers; ++t) {
            (void)hipStreamSynchronize(st[t]);
            (void)hipStreamDestroy(st[t]);
            st[t] = nullptr;
            for (int k = 0; k < 2; ++k) {
                (void)hipEventDestroy(ev[t][k]);
                (void)hipHostFree(buf[t][k]);
                ev[t][k] = nullptr;
                buf[t][k] = nullptr;
            }
        }
        ready = false;
    }
};

std::mutex g_mu;
std::vector<std::unique_ptr<Stage>> g_stage;

Stage& stage_for(int dev) {
    std::lock_guard<std::mutex> g(g_mu);
    if ((int)g_stage.size() <= dev) g_stage.resize(dev + 1);
    if (!g_stage[dev]) g_stage[dev] = std::make_unique<Stage>();
    return *g_stage[dev];
}

}  // namespace

void run_threads(int n, const std::function<void(int)>& body) {
    if (n <= 1) {
        if (n == 1) body(0);
        return;
    }
    std::vector<std::thread> th;
    th.reserve(n);
    for (int t = 0; t < n; ++t) th.emplace_back(body, t);
    for (auto& x : th) x.join();
}

namespace {

// Parked threads woken by a generation counter.  Never destroyed (the threads stay
// parked in a wait at process exit): no static-destruction order against the HIP runtime.
struct Pool {
    std::mutex run_mu;  // one run at a time
    std::mutex mu;
    std::condition_variable go, done;
    uint64_t gen = 0;
    int want = 0, finished = 0;
    const std::function<void(int)>* body = nullptr;
    std::vector<std::thread> th;
    void loop(int t) {  // pool thread t runs body(t + 1)
        uint64_t seen = 0;
        std::unique_lock<std::mutex> lk(mu);
        while (true) {
            go.wait(lk, [&] { return gen != seen; });
            seen = gen;
            if (t + 1 >= want) continue;
            const std::function<void(int)>* b = body;
            lk.unlock();
            (*b)(t + 1);
            lk.lock();
            if (++finished == want - 1) done.notify_one();
        }
    }
};

Pool& pool() {
    static Pool* p = [] {
        Pool* q = new Pool;
        for (int t = 0; t < kPoolThreads; ++t) q->th.emplace_back([q, t] { q->loop(t); });
        for (auto& x : q->th) x.detach();
        return q;
    }();
    return *p;
}

}  // namespace

void run_pool(int n, const std::function<void(int)>& body) {
    n = std::min(n, kPoolThreads + 1);
    if (n <= 1) {
        if (n == 1) body(0);
        return;
    }
    Pool& P = pool();
    std::lock_guard<std::mutex> one(P.run_mu);
    {
        std::lock_guard<std::mutex> lk(P.mu);
        P.body = &body;
        P.want = n;
        P.finished = 0;
        ++P.gen;
    }
    P.go.notify_all();
    body(0);
    std::unique_lock<std::mutex> lk(P.mu);
    P.done.wait(lk, [&] { return P.finished == P.want - 1; });
}

bool host_is_pinned(const void* h) {
    if (!h) return false;
    hipPointerAttribute_t attr;
    if (hipPointerGetAttributes(&attr, h) == hipSuccess) return attr.type == hipMemoryTypeHost;
    (void)hipGetLastError();  // pageable memory is unknown to the runtime
    return false;
}

bool host_range_pinned(const void* h, size_t bytes) {
    if (!host_is_pinned(h)) return false;
    hipDeviceptr_t base = nullptr;
    size_t sz = 0;
    if (hipMemGetAddressRange(&base, &sz, const_cast<void*>(h)) != hipSuccess) {
        (void)hipGetLastError();
        return false;
    }
    const uintptr_t b = reinterpret_cast<uintptr_t>(base), q = reinterpret_cast<uintptr_t>(h);
    return q >= b && q + bytes <= b + sz;
}

int staged_upload(int dev, void* d_dst, const HostFill& fill, uint64_t src_off, size_t bytes) {
    if (!bytes) return 0;
    Stage& S = stage_for(dev);
    std::lock_guard<std::mutex> lk(S.mu);
    if (const int rc = S.init()) return rc;
    const size_t nchunk = (bytes + kChunk - 1) / kChunk;
    const int nthr = (int)std::min<size_t>(kWorkers, nchunk);
    std::vector<int> rcs(nthr, 0);
    // worker t copies chunks t, t + T, ... into its two buffers (alternating) and DMAs each
    // one on its own stream; a buffer is refilled once its previous DMA has completed
    run_threads(nthr, [&](int t) {
        if (hipSetDevice(dev) != hipSuccess) {
            rcs[t] = KARMA_E_HIP;
            return;
        }
        int k = 0;
        for (size_t i = t; i < nchunk; i += nthr, k ^= 1) {
            const size_t o = i * kChunk, n = std::min(kChunk, bytes - o);
            if (hipEventSynchronize(S.ev[t][k]) != hipSuccess) {
                rcs[t] = KARMA_E_HIP;
                return;
            }
            if (const int rc = fill(static_cast<uint8_t*>(S.buf[t][k]), src_off + o, n)) {
                rcs[t] = rc;
                return;
            }
            if (hipMemcpyAsync(static_cast<uint8_t*>(d_dst) + o, S.buf[t][k], n, hipMemcpyHostToDevice, S.st[t]) !=
                    hipSuccess ||
                hipEventRecord(S.ev[t][k], S.st[t]) != hipSuccess) {
                rcs[t] = KARMA_E_HIP;
                return;
            }
        }
        if (hipStreamSynchronize(S.st[t]) != hipSuccess) rcs[t] = KARMA_E_HIP;
    });
    for (int rc : rcs)
        if (rc) return rc == KARMA_E_IO ? rc : set_last_error(rc, "staged upload");
    return 0;
}

int trim_stage(int dev) {
    Stage& S = stage_for(dev);
    std::lock_guard<std::mutex> lk(S.mu);
    S.reset();
    return 0;
}

int trim_host_contexts(int dev) {
    // the staging last: the other contexts' calls may be using it
    int rc = trim_replay_ctx(dev);
    for (int r : {trim_host_batch_ctx(dev), trim_append_ctx(dev), trim_kfp_ctx(dev), trim_stage(dev)})
        if (!rc) rc = r;
    return rc;
}

int staged_copy(int dev, void* d_dst, const void* h_src, size_t bytes) {
    const uint8_t* src = static_cast<const uint8_t*>(h_src);
    return staged_upload(
        dev, d_dst,
        [src](uint8_t* dst, uint64_t off, size_t n) {
            std::memcpy(dst, src + off, n);
            return 0;
        },
        0, bytes);
}

}  // namespace karma::engine
