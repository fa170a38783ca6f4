// tools/hbm_probe.hip -- read-bandwidth microbenchmark for the roofline "achievable" figure.
//
//   hipcc --offload-arch=gfx950 -O3 -o build/hbm_probe tools/hbm_probe.hip && build/hbm_probe [GiB]
//
// Streams a buffer larger than the 256 MiB Infinity Cache with several load flavours and
// launch shapes, xor-reducing so nothing is dead code.  Reports GB/s (1e9) per variant.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) const u32x4 gu32x4;

#define CK(x)                                                                              \
    do {                                                                                   \
        hipError_t e = (x);                                                                \
        if (e != hipSuccess) {                                                             \
            std::printf("HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); \
            std::exit(1);                                                                  \
        }                                                                                  \
    } while (0)

template <int UNROLL, bool NT>
__global__ void k_read(const uint8_t* __restrict__ src, uint64_t n16, uint32_t* out) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    uint32_t x = 0;
    uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    gu32x4* s = (gu32x4*)src;
    for (; i + (UNROLL - 1) * stride < n16; i += UNROLL * stride) {
        u32x4 v[UNROLL];
#pragma unroll
        for (int u = 0; u < UNROLL; ++u) v[u] = NT ? __builtin_nontemporal_load(s + i + u * stride) : s[i + u * stride];
#pragma unroll
        for (int u = 0; u < UNROLL; ++u) x ^= v[u].x ^ v[u].y ^ v[u].z ^ v[u].w;
    }
    for (; i < n16; i += stride) {
        u32x4 v = s[i];
        x ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    if (x == 0x12345678u) out[0] = x;
}

// Each workgroup streams one contiguous slab (block-contiguous instead of grid-strided).
template <int UNROLL, bool NT>
__global__ void k_read_slab(const uint8_t* __restrict__ src, uint64_t n16, uint32_t* out) {
    const uint64_t per = (n16 + gridDim.x - 1) / gridDim.x;
    const uint64_t lo = per * blockIdx.x, hi = lo + per < n16 ? lo + per : n16;
    gu32x4* s = (gu32x4*)src;
    uint32_t x = 0;
    uint64_t i = lo + threadIdx.x;
    for (; i + (UNROLL - 1) * blockDim.x < hi; i += UNROLL * blockDim.x) {
        u32x4 v[UNROLL];
#pragma unroll
        for (int u = 0; u < UNROLL; ++u)
            v[u] = NT ? __builtin_nontemporal_load(s + i + u * blockDim.x) : s[i + u * blockDim.x];
#pragma unroll
        for (int u = 0; u < UNROLL; ++u) x ^= v[u].x ^ v[u].y ^ v[u].z ^ v[u].w;
    }
    for (; i < hi; i += blockDim.x) {
        u32x4 v = s[i];
        x ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    if (x == 0x12345678u) out[0] = x;
}

// The CRC kernel's load pattern without the arithmetic: a wave owns G records per step,
// G lanes... (64/G lanes per record), each record read as 16-byte windows, PF loads in
// flight per lane, records of REC bytes, waves grid-strided over record batches.
template <int LPR, int PF, int REC>
__global__ void k_read_records(const uint8_t* __restrict__ src, uint64_t nrec, uint32_t* out) {
    const int lane = threadIdx.x & 63;
    const int g = lane / LPR, l = lane % LPR;
    constexpr int RPW = 64 / LPR;          // records per wave step
    constexpr int CH = LPR * 16;           // bytes per record per load step
    constexpr int NCH = REC / CH;
    const uint64_t nw = (uint64_t)gridDim.x * (blockDim.x / 64);
    uint32_t x = 0;
    for (uint64_t wb = (uint64_t)blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6); wb * RPW < nrec; wb += nw) {
        const uint64_t r = wb * RPW + g;
        const uint8_t* p = src + (r < nrec ? r : nrec - 1) * REC + 16 * l;
        for (int c = 0; c < NCH; c += PF) {
            u32x4 v[PF];
#pragma unroll
            for (int q = 0; q < PF; ++q) v[q] = __builtin_nontemporal_load((gu32x4*)(p + (c + q) * CH));
#pragma unroll
            for (int q = 0; q < PF; ++q) x ^= v[q].x ^ v[q].y ^ v[q].z ^ v[q].w;
        }
    }
    if (x == 0x12345678u) out[0] = x;
}

template <typename F>
double time_ms(F f, int iters) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    for (int i = 0; i < 3; ++i) f();
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(a));
    for (int i = 0; i < iters; ++i) f();
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    return ms / iters;
}

int main(int argc, char** argv) {
    const double gib = argc > 1 ? atof(argv[1]) : 4.0;
    const uint64_t bytes = (uint64_t)(gib * (1ull << 30));
    uint8_t* buf;
    uint32_t* out;
    CK(hipMalloc(&buf, bytes));
    CK(hipMalloc(&out, 64));
    CK(hipMemset(buf, 1, bytes));
    int cu = 0;
    CK(hipDeviceGetAttribute(&cu, hipDeviceAttributeMultiprocessorCount, 0));
    const uint64_t n16 = bytes / 16;
    auto rep = [&](const char* name, double ms) {
        std::printf("%-48s %8.3f ms  %7.1f GB/s\n", name, ms, bytes / (ms * 1e-3) / 1e9);
    };
    char nm[128];
    for (int blk : {256, 1024}) {
        for (int per_cu : {1, 2}) {
            if (blk * per_cu > 2048) continue;
            const int grid = cu * per_cu;
            std::snprintf(nm, sizeof nm, "grid-stride u4  blk=%d wg/cu=%d", blk, per_cu);
            rep(nm, time_ms([&] { hipLaunchKernelGGL((k_read<4, false>), grid, blk, 0, 0, buf, n16, out); }, 20));
            std::snprintf(nm, sizeof nm, "grid-stride u8  blk=%d wg/cu=%d", blk, per_cu);
            rep(nm, time_ms([&] { hipLaunchKernelGGL((k_read<8, false>), grid, blk, 0, 0, buf, n16, out); }, 20));
            std::snprintf(nm, sizeof nm, "grid-stride u8 nt blk=%d wg/cu=%d", blk, per_cu);
            rep(nm, time_ms([&] { hipLaunchKernelGGL((k_read<8, true>), grid, blk, 0, 0, buf, n16, out); }, 20));
            std::snprintf(nm, sizeof nm, "slab u8        blk=%d wg/cu=%d", blk, per_cu);
            rep(nm, time_ms([&] { hipLaunchKernelGGL((k_read_slab<8, false>), grid, blk, 0, 0, buf, n16, out); }, 20));
            std::snprintf(nm, sizeof nm, "slab u8 nt     blk=%d wg/cu=%d", blk, per_cu);
            rep(nm, time_ms([&] { hipLaunchKernelGGL((k_read_slab<8, true>), grid, blk, 0, 0, buf, n16, out); }, 20));
        }
    }
    const uint64_t nrec = bytes / 4096;
    for (int blk : {256, 512, 1024}) {
        std::snprintf(nm, sizeof nm, "records 8 lanes/rec PF4 blk=%d", blk);
        rep(nm, time_ms([&] { hipLaunchKernelGGL((k_read_records<8, 4, 4096>), cu, blk, 0, 0, buf, nrec, out); }, 20));
        std::snprintf(nm, sizeof nm, "records 8 lanes/rec PF8 blk=%d", blk);
        rep(nm, time_ms([&] { hipLaunchKernelGGL((k_read_records<8, 8, 4096>), cu, blk, 0, 0, buf, nrec, out); }, 20));
        std::snprintf(nm, sizeof nm, "records 64 lanes/rec PF4 blk=%d", blk);
        rep(nm, time_ms([&] { hipLaunchKernelGGL((k_read_records<64, 4, 4096>), cu, blk, 0, 0, buf, nrec, out); }, 20));
        std::snprintf(nm, sizeof nm, "records 16 lanes/rec PF4 blk=%d", blk);
        rep(nm, time_ms([&] { hipLaunchKernelGGL((k_read_records<16, 4, 4096>), cu, blk, 0, 0, buf, nrec, out); }, 20));
    }
    std::printf("hipMemcpy D2D copy: ");
    uint8_t* dst;
    CK(hipMalloc(&dst, bytes / 2));
    double ms = time_ms([&] { CK(hipMemcpyAsync(dst, buf, bytes / 2, hipMemcpyDeviceToDevice, 0)); }, 10);
    std::printf("%.3f ms  %.1f GB/s (read+write)\n", ms, 2.0 * (bytes / 2) / (ms * 1e-3) / 1e9);
    return 0;
}
