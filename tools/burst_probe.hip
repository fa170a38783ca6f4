// tools/burst_probe.hip -- how fast can one 64 MiB segment come in from HBM as one burst?
// (round-4 VERDICT item 3: k_segment_once's phase stamps show ~14 us from the first chunk load to
// the last workgroup's data for 64 MiB, 4.8 TB/s, against ~7.2 TB/s in steady-state streaming.)
//
// Read-only kernels of k_segment_once's shape (256 workgroups x 16 waves, every lane issuing all of
// its 16 x 16-byte loads at once, xor-reduced so nothing is dead), differing only in which bytes a
// wave reads and in what order:
//   seg      k_segment_once's map: workgroup b owns bytes [256 KiB b, +256 KiB), wave w its 16 KiB
//            [16 KiB w, +16 KiB), group g of 8 lanes 2 KiB of that, lane l 16 B of each 128-B chunk
//   inter    wave-steps interleaved over the workgroups: the 16 KiB of (b, w) at 16 KiB (256 w + b),
//            so the grid's first loads cover 4 MiB of consecutive bytes instead of 256 strided slices
//   rot      seg, each lane issuing its 16 loads starting at chunk (b + w) mod 16
//   flat     every wave instruction 1 KiB of consecutive bytes (lane l: 16 B at 1 KiB q + 16 l of the
//            wave's 16 KiB)
// Each is timed with HIP events, isolated (the GPU idle before every launch) and back to back,
// over 64 distinct segments in rotation (4 GiB, past the 256 MiB Infinity Cache), after a 500 ms
// pre-warm.  One JSON line.
//
//   hipcc --offload-arch=gfx950 -O3 -o tools/bin/burst_probe tools/burst_probe.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) const u32x4 gu32x4;

#define CK(x)                                                                                  \
    do {                                                                                       \
        hipError_t e_ = (x);                                                                   \
        if (e_ != hipSuccess) {                                                                \
            std::printf("HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
            std::exit(1);                                                                      \
        }                                                                                      \
    } while (0)

template <int MODE>
__global__ __launch_bounds__(1024) void k_burst(const uint8_t* __restrict__ seg, uint32_t* out) {
    const uint32_t b = blockIdx.x, w = threadIdx.x >> 6, lane = threadIdx.x & 63u;
    const uint32_t g = lane >> 3, l = lane & 7u;
    uint64_t base;  // the wave's 16 KiB
    if (MODE == 1)
        base = (uint64_t)(w * gridDim.x + b) << 14;
    else
        base = ((uint64_t)b << 18) | ((uint64_t)w << 14);
    u32x4 v[16];
#pragma unroll
    for (int q = 0; q < 16; ++q) {
        uint64_t off;
        if (MODE == 3) {
            off = base + ((uint64_t)q << 10) + 16u * lane;
        } else {
            const uint32_t c = MODE == 2 ? (q + b + w) & 15u : (uint32_t)q;
            off = base + ((uint64_t)g << 11) + ((uint64_t)c << 7) + 16u * l;
        }
        v[q] = __builtin_nontemporal_load((gu32x4*)(seg + off));
    }
    uint32_t x = 0;
#pragma unroll
    for (int q = 0; q < 16; ++q) x ^= v[q].x ^ v[q].y ^ v[q].z ^ v[q].w;
    if (x == 0x9E3779B9u) out[0] = x;
}

namespace {
double now_us() {
    return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
double median(std::vector<double> v) {
    std::sort(v.begin(), v.end());
    return v[v.size() / 2];
}
}  // namespace

int main() {
    const size_t seg = size_t(64) << 20;
    const int nseg = 64, G = 256;
    uint8_t* buf = nullptr;
    uint32_t* out = nullptr;
    CK(hipMalloc(&buf, seg * nseg));
    CK(hipMalloc(&out, 4));
    CK(hipMemset(buf, 0x3C, seg * nseg));
    CK(hipDeviceSynchronize());
    hipStream_t st;
    CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    typedef void (*Kern)(const uint8_t*, uint32_t*);
    const Kern kern[4] = {k_burst<0>, k_burst<1>, k_burst<2>, k_burst<3>};
    const char* name[4] = {"seg", "inter", "rot", "flat"};
    int rot = 0;
    for (double t0 = now_us(); now_us() - t0 < 5e5;) {  // pre-warm
        for (int m = 0; m < 4; ++m) hipLaunchKernelGGL(kern[m], dim3(G), dim3(1024), 0, st, buf + (rot++ % nseg) * seg, out);
        CK(hipStreamSynchronize(st));
    }
    std::printf("{\"segment_mib\": 64, \"workgroups\": %d", G);
    for (int m = 0; m < 4; ++m) {
        std::vector<double> iso, b2b;
        for (int r = 0; r < 100; ++r) {
            CK(hipStreamSynchronize(st));
            CK(hipEventRecord(e0, st));
            hipLaunchKernelGGL(kern[m], dim3(G), dim3(1024), 0, st, buf + (rot++ % nseg) * seg, out);
            CK(hipEventRecord(e1, st));
            CK(hipStreamSynchronize(st));
            float ms = 0;
            CK(hipEventElapsedTime(&ms, e0, e1));
            iso.push_back(ms * 1e3);
        }
        for (int r = 0; r < 10; ++r) {
            CK(hipEventRecord(e0, st));
            for (int k = 0; k < 64; ++k)
                hipLaunchKernelGGL(kern[m], dim3(G), dim3(1024), 0, st, buf + (rot++ % nseg) * seg, out);
            CK(hipEventRecord(e1, st));
            CK(hipStreamSynchronize(st));
            float ms = 0;
            CK(hipEventElapsedTime(&ms, e0, e1));
            b2b.push_back(ms * 1e3 / 64);
        }
        const double i = median(iso), bb = median(b2b);
        std::printf(", \"%s\": {\"isolated_event_us\": %.2f, \"back_to_back_us\": %.2f, \"back_to_back_TBps\": %.2f}", name[m],
                    i, bb, seg / bb / 1e6);
    }
    std::printf("}\n");
    return 0;
}
