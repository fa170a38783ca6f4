// tools/api_cost.cc -- host cost of the HIP calls on the library's enqueue path (one 64 MiB
// segment call enqueues in ~3.3 us from C++, DESIGN.md Appendix B "One segment"): hipGetDeviceCount,
// hipGetDevice, hipStreamIsCapturing, an empty kernel launch, and karma_crc32c_stream itself.
//   hipcc --offload-arch=gfx950 -O2 -o build/api_cost tools/api_cost.cc -Iinclude -Lkarma_amd/lib -lkarma_crc32c \
//         -Wl,-rpath,$PWD/karma_amd/lib && build/api_cost
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>

#include "karma_crc32c.h"

__global__ void k_empty() {}

template <typename F>
double ns_per(F f, int n) {
    for (int i = 0; i < 100; ++i) f();
    const auto t0 = std::chrono::steady_clock::now();
    for (int i = 0; i < n; ++i) f();
    const auto t1 = std::chrono::steady_clock::now();
    return std::chrono::duration<double, std::nano>(t1 - t0).count() / n;
}

int main() {
    hipStream_t s;
    if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) return 1;
    const size_t seg = 64u << 20;
    void* d = nullptr;
    uint32_t* out = nullptr;
    if (hipMalloc(&d, seg) != hipSuccess || hipMalloc(&out, 64) != hipSuccess) return 1;
    if (hipMemset(d, 1, seg) != hipSuccess) return 1;
    int n = 0, dev = 0;
    hipStreamCaptureStatus st;
    std::printf("{\"hipGetDeviceCount_ns\": %.0f", ns_per([&] { (void)hipGetDeviceCount(&n); }, 20000));
    std::printf(", \"hipGetDevice_ns\": %.0f", ns_per([&] { (void)hipGetDevice(&dev); }, 20000));
    std::printf(", \"hipStreamIsCapturing_ns\": %.0f", ns_per([&] { (void)hipStreamIsCapturing(s, &st); }, 20000));
    // launches are enqueued faster than the GPU drains them; synchronise every 256
    int i = 0;
    std::printf(", \"empty_launch_ns\": %.0f", ns_per([&] {
        hipLaunchKernelGGL(k_empty, dim3(256), dim3(1024), 0, s);
        if (++i % 256 == 0) (void)hipStreamSynchronize(s);
    }, 5000));
    (void)hipStreamSynchronize(s);
    i = 0;
    std::printf(", \"karma_crc32c_stream_enqueue_ns\": %.0f", ns_per([&] {
        if (karma_crc32c_stream(0, d, seg, out, s) != 0) std::abort();
        if (++i % 64 == 0) (void)hipStreamSynchronize(s);
    }, 2000));
    (void)hipStreamSynchronize(s);
    std::printf("}\n");
    return 0;
}
