// karma_amd/csrc/crc_util.hip -- synthetic data and the read-bandwidth probe.
#include <hip/hip_runtime.h>

#include "crc_device.h"
#include "engine.h"

namespace karma {
namespace engine {
namespace {

using namespace dev;

__device__ __forceinline__ uint64_t splitmix_word(uint64_t seed, uint64_t i) {
    uint64_t z = seed + (i + 1) * 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

// dst[i] = byte (8*first_word + i) of the little-endian splitmix64 stream.
__global__ __launch_bounds__(256) void k_fill_splitmix(uint8_t* dst, uint64_t n_bytes, uint64_t seed,
                                                      uint64_t first_word) {
    const uint64_t n16 = n_bytes / 16;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += stride) {
        const uint64_t w0 = splitmix_word(seed, first_word + 2 * i);
        const uint64_t w1 = splitmix_word(seed, first_word + 2 * i + 1);
        reinterpret_cast<u32x4*>(dst)[i] = u32x4{(uint32_t)w0, (uint32_t)(w0 >> 32), (uint32_t)w1, (uint32_t)(w1 >> 32)};
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        for (uint64_t b = n16 * 16; b < n_bytes; ++b) {
            const uint64_t w = splitmix_word(seed, first_word + b / 8);
            dst[b] = (uint8_t)(w >> (8 * (b & 7)));
        }
    }
}

// Read-only probe: each workgroup streams one contiguous slab with 8
// non-temporal 16-byte loads per lane in flight (the fastest read shape of
// tools/hbm_probe.hip on MI355X); xor-reduced so nothing is dead code.
__global__ __launch_bounds__(256) void k_stream_probe(const uint8_t* src, uint64_t n_bytes, uint32_t* out) {
    KB_SET_ARENA(src, src + n_bytes);
    const uint64_t n16 = n_bytes / 16;
    const uint64_t per = (n16 + gridDim.x - 1) / gridDim.x;
    const uint64_t lo = per * blockIdx.x, hi = lo + per < n16 ? lo + per : n16;
    uint32_t x = 0;
    uint64_t i = lo + threadIdx.x;
    constexpr int U = 8;
    for (; i + (U - 1) * blockDim.x < hi; i += U * blockDim.x) {
        u32x4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) v[u] = ldg<true>(src + 16 * (i + u * blockDim.x));
#pragma unroll
        for (int u = 0; u < U; ++u) x ^= v[u].x ^ v[u].y ^ v[u].z ^ v[u].w;
    }
    for (; i < hi; i += blockDim.x) {
        const u32x4 a = ldg<true>(src + 16 * i);
        x ^= a.x ^ a.y ^ a.z ^ a.w;
    }
#pragma unroll
    for (int d = 32; d > 0; d >>= 1) x ^= __shfl_xor(x, d, 64);
    if ((threadIdx.x & 63) == 0) atomicXor(out, x);
}

}  // namespace

hipError_t launch_fill_splitmix(uint8_t* dst, uint64_t n_bytes, uint64_t seed, uint64_t first_byte, hipStream_t s) {
    if (n_bytes == 0) return hipSuccess;
    uint64_t blocks = (n_bytes / 16 + 255) / 256;
    if (blocks > 65536) blocks = 65536;
    if (blocks == 0) blocks = 1;
    hipLaunchKernelGGL(k_fill_splitmix, dim3((unsigned)blocks), dim3(256), 0, s, dst, n_bytes, seed, first_byte / 8);
    return hipGetLastError();
}

hipError_t launch_stream_probe(const uint8_t* src, uint64_t n_bytes, uint32_t* out, int grid_blocks, hipStream_t s) {
    hipLaunchKernelGGL(k_stream_probe, dim3(grid_blocks), dim3(256), 0, s, src, n_bytes, out);
    return hipGetLastError();
}

KB_DEFINE_COLLECT(util)

}  // namespace engine
}  // namespace karma
