// karma_amd/csrc/crc_ragged.hip -- ragged record batches (offsets + lengths).
//
// Batched form of wal::scan_record's payload check crc32c::Value
// (karma-store/wal.cc:60) and of any Extend over a list of buffers.  Records
// are cut into units of <= unit_bytes (end-aligned to the record's aligned
// body end) so every group of 8 lanes gets at most one unit's worth of work
// regardless of how skewed the record sizes are:
//
//   k_ragged_scan1/2   units per record -> exclusive scan (unit_base)
//   k_ragged_desc      one thread per record: entering register over the
//                      unaligned head (crc32c.cc:323-329 analogue) and one
//                      16-byte descriptor {span start, span length, inj} per unit
//   k_units_ragged     the streaming kernel over the descriptor list
//   k_ragged_finalize  one lane per record: Horner fold of its unit
//                      contributions with Z_unit, unaligned tail bytes, ~R;
//                      records with > 64 units are folded by the whole wave
#include <hip/hip_runtime.h>

#include "crc_device.h"
#include "engine.h"

namespace karma {
namespace engine {
namespace {

using namespace dev;

constexpr int kRaggedPF = 4;
constexpr bool kRaggedNT = true;

__device__ __forceinline__ uint64_t units_of(const Geom& g, uint64_t umax) {
    if (g.is_short) return 1;
    const uint64_t body = (uint64_t)(g.b - g.a);
    return (body + umax - 1) / umax;
}

// Inclusive wave scan of 64-bit values.
__device__ __forceinline__ uint64_t wave_incl_scan(uint64_t x) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint64_t t = __shfl_up(x, d);
        if (lane >= d) x += t;
    }
    return x;
}

// Exclusive block scan (blockDim.x a multiple of 64, <= 1024).
__device__ uint64_t block_excl_scan(uint64_t v, uint64_t* sm, uint64_t& total) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
    const uint64_t inc = wave_incl_scan(v);
    if (lane == 63) sm[wave] = inc;
    __syncthreads();
    if (wave == 0) {
        uint64_t s = lane < nw ? sm[lane] : 0;
        s = wave_incl_scan(s);
        if (lane < nw) sm[lane] = s;
    }
    __syncthreads();
    const uint64_t pre = wave ? sm[wave - 1] : 0;
    total = sm[nw - 1];
    __syncthreads();
    return pre + inc - v;
}

__global__ __launch_bounds__(1024) void k_ragged_scan1(RaggedArgs A) {
    __shared__ uint64_t sm[16];
    const uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint64_t cnt = r < A.n_rec ? units_of(geom(A.arena + A.off[r], A.len[r]), A.unit_bytes) : 0;
    uint64_t total;
    const uint64_t ex = block_excl_scan(cnt, sm, total);
    if (r < A.n_rec) A.unit_base[r] = ex;
    if (threadIdx.x == 0) A.block_sums[blockIdx.x] = total;
}

__global__ __launch_bounds__(1024) void k_ragged_scan2(RaggedArgs A, uint64_t nblocks) {
    __shared__ uint64_t sm[16];
    uint64_t carry = 0;
    for (uint64_t base = 0; base < nblocks; base += blockDim.x) {
        const uint64_t i = base + threadIdx.x;
        const uint64_t v = i < nblocks ? A.block_sums[i] : 0;
        uint64_t total;
        const uint64_t ex = block_excl_scan(v, sm, total);
        if (i < nblocks) A.block_sums[i] = carry + ex;
        carry += total;
    }
    if (threadIdx.x == 0) A.unit_base[A.n_rec] = carry;
}

__global__ __launch_bounds__(256) void k_ragged_desc(RaggedArgs A) {
    __shared__ uint32_t lds[kCombWords];
    load_comb_tables(lds, A.comb_blob);
    __syncthreads();
    const uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= A.n_rec) return;
    const uint64_t base = A.unit_base[r] + A.block_sums[r / 1024];
    A.unit_base[r] = base;
    const uint8_t* p = A.arena + A.off[r];
    const Geom g = geom(p, A.len[r]);
    const uint64_t k = units_of(g, A.unit_bytes);
    if (g.is_short) {
        if (base < A.unit_cap) A.desc[base] = UnitDesc{0, 0, 0};
        return;
    }
    const uint32_t init = A.init ? A.init[r] : A.init_scalar;
    const uint32_t h = head_register(lds, kCombZ4, kCombT8, p, g, init);
    for (uint64_t j = 0; j < k && base + j < A.unit_cap; ++j) {
        const uint8_t* ue = g.b - (int64_t)((k - 1 - j) * A.unit_bytes);
        const uint8_t* us = pmax(ue - (int64_t)A.unit_bytes, g.a);
        A.desc[base + j] = UnitDesc{reinterpret_cast<uint64_t>(us), (uint32_t)(ue - us), j == 0 ? h : 0u};
    }
}

// Descriptor load through address space 1 (global_load_dwordx4, vmcnt only): a
// flat load would also count on lgkmcnt and stall the LDS lookups behind it.
__device__ __forceinline__ UnitDesc load_desc(const UnitDesc* d) {
    const u32x4 v = ld16(reinterpret_cast<const uint8_t*>(d));
    return UnitDesc{v.x | ((uint64_t)v.y << 32), v.z, v.w};
}

__global__ __launch_bounds__(kBlockThreads) void k_units_ragged(RaggedArgs A) {
    __shared__ uint32_t lds[kLdsWords];
    load_stream_tables(lds, A.blob);
    __syncthreads();
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t l = lane & (kGroupLanes - 1);
    const uint32_t grp = lane / kGroupLanes;
    const uint32_t X = lane_const();
    const uint64_t U_all = A.unit_base[A.n_rec];
    const uint64_t U = U_all < A.unit_cap ? U_all : A.unit_cap;  // memory-safe if the caller's bound was low
    const uint64_t nwaves = (uint64_t)gridDim.x * kWavesPerBlock;
    const uint64_t step = nwaves * kGroupsPerWave;
    uint64_t wb = (uint64_t)blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6);
    uint64_t u = wb * kGroupsPerWave + grp;
    UnitDesc d = u < U ? load_desc(A.desc + u) : UnitDesc{0, 0, 0};
    for (; wb * kGroupsPerWave < U; wb += nwaves, u += step) {
        const UnitDesc cur = d;
        const bool valid = u < U;
        // descriptor of this group's next unit, in flight while this one streams
        d = u + step < U ? load_desc(A.desc + u + step) : UnitDesc{0, 0, 0};
        const uint8_t* us = reinterpret_cast<const uint8_t*>(cur.us);
        const uint32_t R = group_unit<kRaggedPF, kRaggedNT>(lds, X, l, us, us + cur.span, us, cur.inj);
        if (valid && l == 0) A.partial[u] = R;
    }
}

__global__ __launch_bounds__(256) void k_ragged_finalize(RaggedArgs A) {
    __shared__ uint32_t lds[kCombWords];
    load_comb_tables(lds, A.comb_blob);
    __syncthreads();
    const uint32_t lane = threadIdx.x & 63u;
    const uint64_t nwaves = (uint64_t)gridDim.x * (blockDim.x >> 6);
    for (uint64_t r0 = ((uint64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6)) * 64; r0 < A.n_rec;
         r0 += nwaves * 64) {
        const uint64_t r = r0 + lane;
        const bool valid = r < A.n_rec;
        uint64_t b0 = 0, k = 0;
        const uint8_t* p = A.arena;
        uint32_t n = 0, init = 0;
        if (valid) {
            b0 = A.unit_base[r];
            k = A.unit_base[r + 1] - b0;
            p = A.arena + A.off[r];
            n = A.len[r];
            init = A.init ? A.init[r] : A.init_scalar;
        }
        const Geom g = geom(p, n);
        const bool ok = valid && b0 + k <= A.unit_cap;
        uint32_t acc = 0, res = 0;
        bool huge = false;
        if (ok && !g.is_short) {
            if (k <= 64) {
                // Horner over the unit contributions, 8 loads in flight at a time
                for (uint64_t j = 0; j < k; j += 8) {
                    uint32_t s[8];
#pragma unroll
                    for (int q = 0; q < 8; ++q) s[q] = j + q < k ? A.partial[b0 + j + q] : 0u;
#pragma unroll
                    for (int q = 0; q < 8; ++q)
                        if (j + q < k) acc = zmap(lds, 0, acc) ^ s[q];
                }
            } else {
                huge = true;
            }
        }
        // records of more than 64 units: the whole wave folds them, one at a time
        uint64_t hm = __ballot(huge);
        while (hm) {
            const int h = __ffsll((long long)hm) - 1;
            hm &= hm - 1;
            const uint64_t hb0 = __shfl(b0, h), hk = __shfl(k, h);
            const uint64_t nb = (hk + 63) / 64;
            const int64_t pad = (int64_t)(nb * 64 - hk);
            uint32_t w = 0;
            for (uint64_t blk = 0; blk < nb; ++blk) {
                const int64_t idx = (int64_t)(blk * 64 + lane) - pad;
                uint32_t v = idx >= 0 ? A.partial[hb0 + idx] : 0u;
                v = wave_tree(lds, v);
                w = zmap(lds, 6 * 1024, w) ^ v;
            }
            w = __shfl(w, 0);
            if ((int)lane == h) acc = w;
        }
        if (ok) {
            if (g.is_short)
                res = short_record(lds, kCombZ4, kCombT8, p, n, init);
            else
                res = ~tail_register(lds, kCombZ4, kCombT8, acc, g);
            A.out[r] = res;
        }
    }
}

}  // namespace

uint64_t ragged_scan_blocks(uint64_t n_rec) { return (n_rec + 1023) / 1024; }

hipError_t launch_ragged_scan(const RaggedArgs& a, hipStream_t s) {
    if (a.n_rec == 0) return hipSuccess;
    const uint64_t nb = ragged_scan_blocks(a.n_rec);
    hipLaunchKernelGGL(k_ragged_scan1, dim3((unsigned)nb), dim3(1024), 0, s, a);
    hipLaunchKernelGGL(k_ragged_scan2, dim3(1), dim3(1024), 0, s, a, nb);
    return hipGetLastError();
}

hipError_t launch_ragged_main(const RaggedArgs& a, int grid_blocks, hipStream_t s) {
    if (a.n_rec == 0) return hipSuccess;
    hipLaunchKernelGGL(k_ragged_desc, dim3((unsigned)((a.n_rec + 255) / 256)), dim3(256), 0, s, a);
    hipLaunchKernelGGL(k_units_ragged, dim3(grid_blocks), dim3(kBlockThreads), 0, s, a);
    uint64_t fblocks = (a.n_rec + 255) / 256;  // 4 waves x 64 records per block
    if (fblocks > 8192) fblocks = 8192;
    hipLaunchKernelGGL(k_ragged_finalize, dim3((unsigned)fblocks), dim3(256), 0, s, a);
    return hipGetLastError();
}

}  // namespace engine
}  // namespace karma
