// tools/segment_loop.cc -- the single-segment latency (configs[3]) seen from C++, without Python
// or torch in the way: how much of an isolated karma_crc32c_stream call is the library's own
// enqueue, and how much is the kernel.  Links the shipped library through its C ABI only.
//
//   hipcc -O2 -std=c++17 tools/segment_loop.cc -Iinclude -Lkarma_amd/lib -lkarma_crc32c \
//         -Wl,-rpath,$PWD/karma_amd/lib -o tools/bin/segment_loop
//   tools/bin/segment_loop [MiB=64] [calls=2000]
//
// Printed (one JSON line; microseconds, medians unless noted):
//   enqueue_us          host time of one call, calls back to back with no sync
//   back_to_back_us     wall time per call over `calls` calls issued back to back, then one sync
//   isolated_event_us   events recorded before / after one call on an idle stream, then a sync
//                       (bench.py --workload segment's single_segment_latency_us)
//   isolated_wall_us    host wall time of call + sync on an idle stream
//   launch_floor_us     the same events around an empty kernel launch (the HIP floor)
// 64 distinct segments rotate so every call reads HBM (64 x 64 MiB > the 256 MB MALL); the CRCs of
// the rotation are checked against karma_crc32c_extend_host at the end.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "karma_crc32c.h"

namespace {

__global__ void k_empty() {}

double now_us() {
    return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

double median(std::vector<double> v) {
    std::sort(v.begin(), v.end());
    return v.empty() ? 0.0 : v[v.size() / 2];
}

#define CK(x)                                                                        \
    do {                                                                             \
        if ((x) != hipSuccess) {                                                     \
            std::fprintf(stderr, "%s failed at line %d\n", #x, __LINE__);            \
            return 1;                                                                \
        }                                                                            \
    } while (0)

}  // namespace

int main(int argc, char** argv) {
    const size_t mib = argc > 1 ? std::strtoul(argv[1], nullptr, 10) : 64;
    const int calls = argc > 2 ? std::atoi(argv[2]) : 2000;
    const size_t seg = mib << 20;
    const int nseg = 64;
    uint8_t* arena = nullptr;
    uint32_t* out = nullptr;
    CK(hipMalloc(&arena, seg * nseg));
    CK(hipMalloc(&out, nseg * sizeof(uint32_t)));
    hipStream_t st;
    CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    if (karma_fill_splitmix64(arena, seg * nseg, 42, 0, st)) return 1;
    CK(hipStreamSynchronize(st));
    int i = 0;
    auto call = [&]() {
        const int k = i++ % nseg;
        return karma_crc32c_stream(0, arena + (size_t)k * seg, seg, out + k, st);
    };
    // pre-warm 500 ms (the clock ramp)
    for (double t0 = now_us(); now_us() - t0 < 5e5;) {
        for (int q = 0; q < 8; ++q)
            if (call()) return 1;
        CK(hipStreamSynchronize(st));
    }
    // enqueue: calls back to back, host time per call; back to back: wall per call incl. the drain
    std::vector<double> enq, b2b;
    for (int r = 0; r < 5; ++r) {
        CK(hipStreamSynchronize(st));
        const double t0 = now_us();
        for (int c = 0; c < calls; ++c)
            if (call()) return 1;
        const double t1 = now_us();
        CK(hipStreamSynchronize(st));
        const double t2 = now_us();
        enq.push_back((t1 - t0) / calls);
        b2b.push_back((t2 - t0) / calls);
    }
    // isolated calls: events around one call on an idle stream
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    std::vector<double> iso_ev, iso_wall, floor_ev;
    for (int r = 0; r < 200; ++r) {
        CK(hipStreamSynchronize(st));
        const double t0 = now_us();
        CK(hipEventRecord(e0, st));
        if (call()) return 1;
        CK(hipEventRecord(e1, st));
        CK(hipStreamSynchronize(st));
        iso_wall.push_back(now_us() - t0);
        float ms = 0;
        CK(hipEventElapsedTime(&ms, e0, e1));
        iso_ev.push_back(ms * 1e3);
        CK(hipEventRecord(e0, st));
        hipLaunchKernelGGL(k_empty, dim3(1), dim3(64), 0, st);
        CK(hipEventRecord(e1, st));
        CK(hipStreamSynchronize(st));
        CK(hipEventElapsedTime(&ms, e0, e1));
        floor_ev.push_back(ms * 1e3);
    }
    // check the rotation's CRCs against the host Extend
    std::vector<uint32_t> got(nseg);
    CK(hipMemcpy(got.data(), out, nseg * sizeof(uint32_t), hipMemcpyDeviceToHost));
    std::vector<uint8_t> host(seg);
    int bad = 0;
    for (int k = 0; k < 4; ++k) {
        CK(hipMemcpy(host.data(), arena + (size_t)k * seg, seg, hipMemcpyDeviceToHost));
        if (karma_crc32c_extend_host(0, host.data(), seg) != got[k]) ++bad;
    }
    std::printf("{\"mib\": %zu, \"calls\": %d, \"enqueue_us\": %.2f, \"back_to_back_us\": %.2f, "
                "\"isolated_event_us\": %.2f, \"isolated_event_p10_us\": %.2f, \"isolated_wall_us\": %.2f, "
                "\"launch_floor_us\": %.2f, \"checked\": 4, \"mismatches\": %d}\n",
                mib, calls, median(enq), median(b2b), median(iso_ev),
                [&] { auto v = iso_ev; std::sort(v.begin(), v.end()); return v[v.size() / 10]; }(), median(iso_wall),
                median(floor_ev), bad);
    return bad ? 2 : 0;
}
