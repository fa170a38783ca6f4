// tools/fetch_calib.hip -- calibrates rocprofv3's FETCH_SIZE on the WAL walk's access shapes
// (round-4 VERDICT item 2a).  MI355X_MICROARCH.md establishes FETCH_SIZE = half the bytes only for
// wide (16 B/lane) coalesced streaming reads; the header walk reads one 8-byte header per record.
// Four distinct images of 1M x 188-byte records (a 180-B payload + its 8-B header: the replay
// bench's layout, 752 MB together, past the 256 MiB Infinity Cache) are read in rotation by:
//
//   k_stream16   every byte, 16 B per lane, coalesced (the guide's known case)
//   k_header8    one 8-byte load per record at a 188-byte stride, lane i = record i (what the
//                walkers' direct rounds issue: 64 headers per wave load)
//   k_header8_sparse  the same for every 16th record only (isolated lines, no neighbours)
//
// The program prints, per kernel, the bytes it asks for and the distinct 64-B sectors and
// 128-B lines those bytes fall in; rocprofv3 --pmc FETCH_SIZE (KB per dispatch) over the same
// run gives the counter, and tools/fetch_calib_summary.py divides the two.
//
//   hipcc --offload-arch=gfx950 -O3 -o tools/bin/fetch_calib tools/fetch_calib.hip
//   rocprofv3 --pmc FETCH_SIZE -d gpurun_out/calib -o run -- tools/bin/fetch_calib
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <set>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) const u32x4 gu32x4;
typedef __attribute__((address_space(1))) const uint64_t gu64;

#define CK(x)                                                                                  \
    do {                                                                                       \
        hipError_t e_ = (x);                                                                   \
        if (e_ != hipSuccess) {                                                                \
            std::printf("HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
            std::exit(1);                                                                      \
        }                                                                                      \
    } while (0)

__global__ void k_stream16(const uint8_t* __restrict__ src, uint64_t n16, uint32_t* out) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    uint32_t x = 0;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += stride) {
        const u32x4 v = __builtin_nontemporal_load((gu32x4*)src + i);
        x ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    if (x == 0x9E3779B9u) out[0] = x;
}

// record r's 8-byte header at r * rec (rec a multiple of 4, so the load is 4-byte aligned: two
// dwords, as the walkers read a header)
__global__ void k_header8(const uint8_t* __restrict__ src, uint64_t n_rec, uint32_t rec, uint32_t every, uint32_t* out) {
    const uint64_t r = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) * every;
    if (r >= n_rec) return;
    const uint32_t* p = reinterpret_cast<const uint32_t*>(src + r * rec);
    const uint32_t a = *(const __attribute__((address_space(1))) uint32_t*)p;
    const uint32_t b = *(const __attribute__((address_space(1))) uint32_t*)(p + 1);
    if ((a ^ b) == 0x9E3779B9u) out[0] = a;
}

int main() {
    const uint64_t n_rec = 1 << 20;
    const uint32_t rec = 188;
    const uint64_t img = n_rec * rec;
    const int nimg = 4, reps = 8;
    uint8_t* buf = nullptr;
    uint32_t* out = nullptr;
    CK(hipMalloc(&buf, img * nimg));
    CK(hipMalloc(&out, 4));
    CK(hipMemset(buf, 0x5A, img * nimg));
    CK(hipDeviceSynchronize());
    // distinct sectors / lines of the header reads (host)
    auto count = [&](uint32_t every, uint64_t gran) {
        std::set<uint64_t> s;
        for (uint64_t r = 0; r < n_rec; r += every) {
            s.insert(r * rec / gran);
            s.insert((r * rec + 7) / gran);
        }
        return (uint64_t)s.size();
    };
    for (int k = 0; k < reps * nimg; ++k) {
        const uint8_t* b = buf + (uint64_t)(k % nimg) * img;
        hipLaunchKernelGGL(k_stream16, dim3(1024), dim3(256), 0, 0, b, img / 16, out);
    }
    CK(hipDeviceSynchronize());
    for (int k = 0; k < reps * nimg; ++k) {
        const uint8_t* b = buf + (uint64_t)(k % nimg) * img;
        hipLaunchKernelGGL(k_header8, dim3((unsigned)((n_rec + 255) / 256)), dim3(256), 0, 0, b, n_rec, rec, 1u, out);
    }
    CK(hipDeviceSynchronize());
    for (int k = 0; k < reps * nimg; ++k) {
        const uint8_t* b = buf + (uint64_t)(k % nimg) * img;
        hipLaunchKernelGGL(k_header8, dim3((unsigned)((n_rec / 16 + 255) / 256)), dim3(256), 0, 0, b, n_rec, rec, 16u,
                           out);
    }
    CK(hipDeviceSynchronize());
    std::printf("{\"image_bytes\": %llu, \"images\": %d, \"dispatches_per_kernel\": %d,\n",
                (unsigned long long)img, nimg, reps * nimg);
    std::printf(" \"k_stream16\": {\"bytes_asked\": %llu, \"sectors64\": %llu, \"lines128\": %llu},\n",
                (unsigned long long)img, (unsigned long long)(img / 64), (unsigned long long)(img / 128));
    std::printf(" \"k_header8_every1\": {\"bytes_asked\": %llu, \"sectors64\": %llu, \"lines128\": %llu},\n",
                (unsigned long long)(n_rec * 8), (unsigned long long)count(1, 64), (unsigned long long)count(1, 128));
    std::printf(" \"k_header8_every16\": {\"bytes_asked\": %llu, \"sectors64\": %llu, \"lines128\": %llu}}\n",
                (unsigned long long)(n_rec / 16 * 8), (unsigned long long)count(16, 64), (unsigned long long)count(16, 128));
    return 0;
}
