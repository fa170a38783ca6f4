// karma_amd/csrc/crc_fixed.hip -- fixed-size record batches on MI355X (gfx950).
//
// Batched form of segment_file::append_record's per-record crc32c::Value
// (karma-store/segment_file.cc:22; algorithm karma-util/crc32c.cc:275-376).
// Record r = arena + r*rec_bytes.  Each record body is cut into k units
// (k = 1 for batches large enough to fill the GPU), one unit per
// group of 8 lanes; when k > 1 the unit contributions are folded by
// k_combine_fixed, one level per factor of 64, with maps Z_{D*2^d}.
#include <hip/hip_runtime.h>

#include <cstdlib>

#include "crc_device.h"
#include "engine.h"

namespace karma {
namespace engine {
namespace {

using namespace dev;

template <int PF, bool NT, int MODE = 0>
__global__ __launch_bounds__(kBlockThreads) void k_units_fixed(FixedArgs A) {
    __shared__ __attribute__((aligned(16))) uint32_t lds[kLdsWords];
    load_stream_tables(lds, A.blob);
    __syncthreads();
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t l = lane & (kGroupLanes - 1);
    const uint32_t grp = lane / kGroupLanes;
    const uint32_t X = lane_const();
    const uint64_t k = A.units_per_rec;
    const uint64_t U = A.n_rec * k;
    const uint64_t nwaves = (uint64_t)gridDim.x * kWavesPerBlock;
    for (uint64_t wb = (uint64_t)blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6); wb * kGroupsPerWave < U;
         wb += nwaves) {
        const uint64_t u = wb * kGroupsPerWave + grp;
        const bool valid = u < U;
        uint64_t r = 0, j = 0;
        if (valid) {
            if (k == 1) {
                r = u;
            } else {
                r = u / k;
                j = u - r * k;
            }
        }
        const uint8_t* p = A.arena + r * A.rec_bytes;
        const uint32_t init = valid ? (A.init ? A.init[r] : A.init_scalar) : 0u;
        const Geom g = geom(p, A.rec_bytes);
        // unit j of the body [a, b), end-aligned at b: [b - (k-j)*U, b - (k-1-j)*U) clipped to a
        const uint8_t* us = nullptr;
        const uint8_t* ue = nullptr;
        const uint8_t* inj_at = nullptr;
        uint32_t inj = 0;
        if (valid && !g.is_short) {
            ue = g.b - (int64_t)((k - 1 - j) * A.unit_bytes);
            const uint8_t* us_raw = ue - (int64_t)A.unit_bytes;
            us = pmax(us_raw, g.a);
            if (us > ue) us = ue;
            if (g.a >= us_raw && g.a < ue) {  // this unit holds the body start
                inj_at = g.a;
                inj = head_register(lds, kLZ4, kLT8, p, g, init);
            }
        }
        uint32_t R = group_unit<PF, NT, MODE>(lds, X, l, us, ue, inj_at, inj);
        if (valid && l == 0) {
            if (g.is_short) {
                A.out[r] = short_record(lds, kLZ4, kLT8, p, A.rec_bytes, init);
            } else if (k == 1) {
                A.out[r] = ~tail_register(lds, kLZ4, kLT8, R, g);
            } else {
                A.partial[u] = R;
            }
        }
    }
}

// Fixed records on the absolute 128-byte grid (arena 128-aligned, unit a
// multiple of PF chunks, rec_bytes = k * unit): unit u is simply
// arena + u * unit_bytes, with no head, tail or partial chunk.  Each lane's
// loads form one continuous stream across the wave's units: the first PF
// chunks of the group's next unit are issued before the current unit's
// fold and tree, so no memory bubble opens at unit boundaries.
template <int PF>
__global__ __launch_bounds__(kBlockThreads) void k_units_aligned(FixedArgs A) {
    __shared__ __attribute__((aligned(16))) uint32_t lds[kLdsWords];
    load_stream_tables(lds, A.blob);
    __syncthreads();
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t l = lane & (kGroupLanes - 1);
    const uint32_t grp = lane / kGroupLanes;
    const uint32_t X = lane_const();
    const uint64_t k = A.units_per_rec;
    const uint64_t U = A.n_rec * k;
    const uint64_t C = A.unit_bytes / kChunk;  // chunks per unit, a multiple of PF
    const uint64_t step = (uint64_t)gridDim.x * kWavesPerBlock * kGroupsPerWave;
    const uint8_t* base = A.arena + 16 * l;
    const uint64_t ub = A.unit_bytes;
    auto at = [&](uint64_t uu, uint64_t c) {  // clamped: groups past the end load a valid line
        return base + (uu < U ? uu : U - 1) * ub + c * kChunk;
    };
    uint64_t w0 = ((uint64_t)blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6)) * kGroupsPerWave;
    uint64_t u = w0 + grp;
    u32x4 nb[PF];
#pragma unroll
    for (int q = 0; q < PF; ++q) nb[q] = ldg<true>(at(u, q));
    for (; w0 < U; w0 += step, u += step) {
        const bool valid = u < U;
        uint32_t inj = 0;
        uint64_t r = u;
        if (k != 1) r = u / k;
        if (valid && l == 0 && r * k == u) inj = ~(A.init ? A.init[r] : A.init_scalar);
        uint32_t a0 = 0, a1 = 0, a2 = 0, a3 = 0;
        for (uint64_t c = 0; c < C; c += PF) {
            u32x4 cur[PF];
#pragma unroll
            for (int q = 0; q < PF; ++q) cur[q] = nb[q];
            if (c + PF < C) {
#pragma unroll
                for (int q = 0; q < PF; ++q) nb[q] = ldg<true>(at(u, c + PF + q));
            } else {
#pragma unroll
                for (int q = 0; q < PF; ++q) nb[q] = ldg<true>(at(u + step, q));
            }
            if (c == 0) cur[0].x ^= inj;
#pragma unroll
            for (int q = 0; q < PF; ++q) step4(lds, X, a0, a1, a2, a3, cur[q]);
        }
        // lane fold (crc32c.cc STEP4W order), then the 8-lane tree (lane 7 holds the last window)
        uint32_t c = zmap(lds, kLZ4, a0);
        c = zmap(lds, kLZ4, c ^ a1);
        c = zmap(lds, kLZ4, c ^ a2);
        c = zmap(lds, kLZ4, c ^ a3);
        uint32_t t = __shfl_down(c, 1, kGroupLanes);
        c = zmap(lds, kLZ16, c) ^ t;
        t = __shfl_down(c, 2, kGroupLanes);
        c = zmap(lds, kLZ32, c) ^ t;
        t = __shfl_down(c, 4, kGroupLanes);
        c = zmap(lds, kLZ64, c) ^ t;
        if (valid && l == 0) {
            if (k == 1)
                A.out[u] = ~c;
            else
                A.partial[u] = c;
        }
    }
}

// One combine level: record r's k_in states (end-aligned, D bytes each) ->
// k_out = ceil(k_in / 64) states of 64*D bytes; the last level (k_out == 1)
// adds the record tail and writes the CRC.  One wave per output state.
__global__ __launch_bounds__(256) void k_combine_fixed(FixedArgs A, const uint32_t* in, uint64_t k_in, uint32_t* outs,
                                                      uint64_t k_out, const uint32_t* comb) {
    __shared__ __attribute__((aligned(16))) uint32_t lds[kCombCoreWords];
    load_comb_tables<kCombCoreWords, 256>(lds, comb);
    __syncthreads();
    const uint32_t lane = threadIdx.x & 63u;
    const uint64_t nwaves = (uint64_t)gridDim.x * (blockDim.x >> 6);
    const uint64_t total = A.n_rec * k_out;
    const int64_t pad = (int64_t)(k_out * 64 - k_in);
    for (uint64_t t = (uint64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); t < total; t += nwaves) {
        const uint64_t r = t / k_out;
        const uint64_t o = t - r * k_out;
        const int64_t idx = (int64_t)(o * 64 + lane) - pad;
        uint32_t v = idx >= 0 ? in[r * k_in + idx] : 0u;
        v = wave_tree(lds, v);
        if (lane == 0) {
            if (k_out == 1) {
                const uint8_t* p = A.arena + r * A.rec_bytes;
                A.out[r] = ~tail_register(lds, kCombZ4, kCombT8, v, geom(p, A.rec_bytes));
            } else {
                outs[r * k_out + o] = v;
            }
        }
    }
}

// KARMA_CRC_VARIANT selects an alternative build of the streaming kernel for
// in-process A/B measurements (tools/variant_bench.py); 0 = shipped default.
int fixed_variant() {
    const char* e = getenv("KARMA_CRC_VARIANT");
    return e ? atoi(e) : 0;
}

}  // namespace

bool fixed_aligned_ok(const FixedArgs& a) {
    return (reinterpret_cast<uintptr_t>(a.arena) & (kChunk - 1)) == 0 && a.unit_bytes % (kChunk * 4) == 0 &&
           a.rec_bytes == a.units_per_rec * a.unit_bytes && a.rec_bytes > 0;
}

bool fixed_fast_path_ok(const FixedArgs& a) {
    return (reinterpret_cast<uintptr_t>(a.arena) & 15u) == 0 && a.unit_bytes % kChunk == 0 &&
           a.rec_bytes == a.units_per_rec * a.unit_bytes && a.rec_bytes > 0;
}

hipError_t launch_fixed(const FixedArgs& a, int grid_blocks, hipStream_t s) {
    if (a.n_rec == 0) return hipSuccess;
    const uint64_t units = a.n_rec * a.units_per_rec;
    const uint64_t need = (units + kGroupsPerWave * kWavesPerBlock - 1) / (kGroupsPerWave * kWavesPerBlock);
    const dim3 grid((unsigned)(need < (uint64_t)grid_blocks ? need : (uint64_t)grid_blocks));
    units_timer_begin(s);
    switch (fixed_variant()) {
        case 1: hipLaunchKernelGGL((k_units_fixed<4, false>), grid, dim3(kBlockThreads), 0, s, a); break;
        case 2: hipLaunchKernelGGL((k_units_fixed<2, true>), grid, dim3(kBlockThreads), 0, s, a); break;
        case 3: hipLaunchKernelGGL((k_units_fixed<6, true>), grid, dim3(kBlockThreads), 0, s, a); break;
        case 4: hipLaunchKernelGGL((k_units_fixed<4, true, 1>), grid, dim3(kBlockThreads), 0, s, a); break;
        case 5: hipLaunchKernelGGL((k_units_fixed<4, true, 2>), grid, dim3(kBlockThreads), 0, s, a); break;
        case 6: hipLaunchKernelGGL((k_units_fixed<4, true, 3>), grid, dim3(kBlockThreads), 0, s, a); break;
        case 7:
            if (fixed_aligned_ok(a)) {
                hipLaunchKernelGGL((k_units_aligned<4>), grid, dim3(kBlockThreads), 0, s, a);
                break;
            }
            [[fallthrough]];
        default: hipLaunchKernelGGL((k_units_fixed<4, true>), grid, dim3(kBlockThreads), 0, s, a); break;
    }
    units_timer_end(s);
    return hipGetLastError();
}

hipError_t launch_combine_fixed(const FixedArgs& a, const uint32_t* in_states, uint64_t k_in, uint32_t* out_states,
                                uint64_t k_out, const uint32_t* comb_blob, hipStream_t s) {
    const uint64_t waves = a.n_rec * k_out;
    uint64_t blocks = (waves + 3) / 4;
    if (blocks > 8192) blocks = 8192;
    hipLaunchKernelGGL(k_combine_fixed, dim3((unsigned)blocks), dim3(256), 0, s, a, in_states, k_in, out_states,
                       k_out, comb_blob);
    return hipGetLastError();
}

}  // namespace engine
}  // namespace karma
