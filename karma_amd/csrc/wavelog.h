// karma_amd/csrc/wavelog.h -- per-wave timing log of the units kernels, tools build only.
//
// DESIGN.md §4 asks where the ragged units kernel loses against the fixed one: with
// KARMA_AB, k_units_ragged and k_units_fixed(_v1) write one record per wave -- when it
// started streaming (after the LDS table fill), when it finished, the CU / XCC it ran on,
// and the units and bytes it streamed -- into a buffer set by karma_ab_wave_log() (capi.cc).
// tools/ragged_gap.py reads the spread of the end times and the per-wave work.  The
// shipped build compiles none of it (the macros are empty).
#pragma once
#include <cstdint>

namespace karma::engine {
struct WaveLogRec {
    uint64_t t0, t1;           // wall_clock64() at stream start / end (100 MHz)
    uint32_t hw_id, xcc_id;    // HW_REG_HW_ID, HW_REG_XCC_ID
    uint32_t units;            // units this wave's groups streamed
    uint32_t kib;              // their bytes / 1024
    uint32_t steps, pad;       // wave-steps taken
};
static_assert(sizeof(WaveLogRec) == 40, "40-byte records");
}  // namespace karma::engine

#ifdef KARMA_AB
namespace karma::engine {
namespace {
__device__ WaveLogRec* g_wave_log;  // per translation unit: set by set_wave_log_<tu>()
__device__ uint64_t g_wave_log_cap;
}  // namespace
}  // namespace karma::engine
#define WLOG_DECL uint64_t wlog_t0 = 0, wlog_bytes = 0; uint32_t wlog_units = 0, wlog_steps = 0
#define WLOG_START() (wlog_t0 = wall_clock64())
#define WLOG_UNIT(leader, nbytes)                         \
    do {                                                  \
        if (leader) {                                     \
            wlog_units += 1;                              \
            wlog_bytes += (uint64_t)(nbytes);             \
        }                                                 \
    } while (0)
#define WLOG_STEP() (wlog_steps += 1)
#define WLOG_END(wave_id)                                                                            \
    do {                                                                                             \
        if (::karma::engine::g_wave_log) {                                                           \
            const uint64_t t1 = wall_clock64();                                                      \
            uint64_t b = wlog_bytes;                                                                 \
            uint32_t n = wlog_units;                                                                 \
            for (int d = 32; d >= 1; d >>= 1) {                                                      \
                b += __shfl_xor(b, d);                                                               \
                n += __shfl_xor(n, d);                                                               \
            }                                                                                        \
            const uint64_t w = (wave_id);                                                            \
            if ((threadIdx.x & 63u) == 0 && w < ::karma::engine::g_wave_log_cap) {                   \
                ::karma::engine::WaveLogRec r;                                                       \
                r.t0 = wlog_t0;                                                                      \
                r.t1 = t1;                                                                           \
                r.hw_id = __builtin_amdgcn_s_getreg((31 << 11) | (0 << 6) | 4);                      \
                r.xcc_id = __builtin_amdgcn_s_getreg((15 << 11) | (0 << 6) | 20);                    \
                r.units = n;                                                                         \
                r.kib = (uint32_t)(b >> 10);                                                         \
                r.steps = wlog_steps;                                                                \
                r.pad = 0;                                                                           \
                ::karma::engine::g_wave_log[w] = r;                                                  \
            }                                                                                        \
        }                                                                                            \
    } while (0)
#define WLOG_SETTER(tu)                                                                              \
    hipError_t set_wave_log_##tu(void* p, uint64_t cap) {                                            \
        WaveLogRec* q = static_cast<WaveLogRec*>(p);                                                 \
        hipError_t e = hipMemcpyToSymbol(HIP_SYMBOL(g_wave_log), &q, sizeof(q));                     \
        if (e == hipSuccess) e = hipMemcpyToSymbol(HIP_SYMBOL(g_wave_log_cap), &cap, sizeof(cap));   \
        return e;                                                                                    \
    }
#else
#define WLOG_DECL
#define WLOG_START() ((void)0)
#define WLOG_UNIT(leader, nbytes) ((void)0)
#define WLOG_STEP() ((void)0)
#define WLOG_END(wave_id) ((void)0)
#endif
