// karma_amd/csrc/bounds.h -- the bounds-checked debug build.
//
//   make -C karma_amd/csrc bounds   -> tools/lib/libkarma_crc32c_bounds.so (-DKARMA_BOUNDS)
//   tests/test_gpu_bounds.py        runs the WAL and ragged parity cases against it
//
// In that build every global access of the WAL replay kernels (wal_device.hip: image
// bytes, candidate lists, sub-range reports, spans, gathered lists) and every record-byte
// load of the CRC kernels (crc_device.h's ldg / ld16) is checked against the buffer it
// must stay in.  A violation is counted, the first one is kept (site, index, capacity),
// and the access is redirected to the buffer's first element (reads) or dropped
// (writes), so the run finishes and the test reads the report through
// karma_debug_bounds_report().  In the shipped build every macro is the plain access and
// this header adds nothing.
#pragma once
#include <cstdint>

#ifdef KARMA_BOUNDS
#include <hip/hip_runtime_api.h>

namespace karma::engine {

struct KbReport {
    unsigned long long count;  // violations
    unsigned long long site;   // first violation: its site (KbSite), index and capacity
    unsigned long long index;
    unsigned long long cap;
};

enum KbSite : unsigned {
    kKbImage = 1,        // WAL image byte outside [wal, wal + img_bytes)
    kKbSegment = 2,      // WAL image byte outside the walker's own segment
    kKbCand = 3,         // candidate list slot outside the segment's cand_cap
    kKbCandDropped = 4,  // a list write the walker's cap guard dropped (the list would be short)
    kKbSubMeta = 5,      // sub-range report index
    kKbSpan = 6,         // span index
    kKbMeta = 7,         // segment meta index
    kKbList = 8,         // gathered list index (off / len / stored / crc) >= n_all
    kKbRunSlot = 9,      // a gathered slot outside its sub-range's slots
    kKbArena = 10,       // record byte load outside the arena's allocation
    kKbUnit = 11,        // ragged unit descriptor / partial slot >= unit_cap
};

// Host side: each .hip file's report (KB_DEFINE_COLLECT), read and optionally cleared.
hipError_t kb_collect_fixed(KbReport* out, bool reset);
hipError_t kb_collect_ragged(KbReport* out, bool reset);
hipError_t kb_collect_util(KbReport* out, bool reset);
hipError_t kb_collect_wal(KbReport* out, bool reset);

}  // namespace karma::engine

#ifdef __HIP__  // device side (the .hip files)
#include <hip/hip_runtime.h>

namespace karma::engine {

// The report of the translation unit that includes this header (one per .hip file).
namespace {
__device__ KbReport g_kb;
}

__device__ __forceinline__ bool kb_ok(bool ok, unsigned site, unsigned long long index, unsigned long long cap) {
    if (!ok) {
        if (atomicAdd(&g_kb.count, 1ull) == 0) {
            g_kb.site = site;
            g_kb.index = index;
            g_kb.cap = cap;
        }
    }
    return ok;
}

// The arena range the current kernel's record-byte loads must stay in (set at kernel entry
// with kb_set_arena; one per workgroup).
// [slo, shi) is a second range a kernel may read on purpose: the "safe address" its empty
// units load from (the table blob), else empty.
struct KbRange {
    uintptr_t lo, hi, slo, shi;
};
__device__ __forceinline__ KbRange& kb_arena() {
    __shared__ KbRange r;
    return r;
}
__device__ __forceinline__ void kb_set_arena(uintptr_t lo, uintptr_t hi, uintptr_t slo = 0, uintptr_t shi = 0) {
    if (threadIdx.x == 0) kb_arena() = KbRange{lo, hi, slo, shi};
    __syncthreads();
}
// p checked for n bytes; a violating load reads the arena's first block instead.
__device__ __forceinline__ const uint8_t* kb_bytes(const uint8_t* p, unsigned n) {
    const KbRange r = kb_arena();
    const uintptr_t a = reinterpret_cast<uintptr_t>(p);
    if (a >= r.slo && a + n <= r.shi) return p;
    if (kb_ok(a >= r.lo && a + n <= r.hi, kKbArena, a - r.lo, r.hi - r.lo)) return p;
    return reinterpret_cast<const uint8_t*>(r.lo);
}

}  // namespace karma::engine

#define KB_DEFINE_COLLECT(name)                                                         \
    hipError_t kb_collect_##name(KbReport* out, bool reset) {                           \
        hipError_t e = hipMemcpyFromSymbol(out, HIP_SYMBOL(g_kb), sizeof(KbReport));    \
        if (e == hipSuccess && reset) {                                                 \
            const KbReport z{0, 0, 0, 0};                                               \
            e = hipMemcpyToSymbol(HIP_SYMBOL(g_kb), &z, sizeof(KbReport));              \
        }                                                                               \
        return e;                                                                       \
    }

// idx checked against [0, cap): reads return element 0 of the buffer on a violation,
// writes are dropped.
#define KB_IDX(ok_idx, cap, site) ::karma::engine::kb_ok((uint64_t)(ok_idx) < (uint64_t)(cap), site, (ok_idx), (cap))
#define KB_READ(arr, idx, cap, site) ((arr)[KB_IDX(idx, cap, site) ? (idx) : 0])
#define KB_WRITE(arr, idx, cap, site, v)     \
    do {                                     \
        if (KB_IDX(idx, cap, site)) (arr)[idx] = (v); \
    } while (0)
#define KB_BYTES(p, n) ::karma::engine::kb_bytes((p), (n))
#define KB_SET_ARENA(lo, hi) ::karma::engine::kb_set_arena((uintptr_t)(lo), (uintptr_t)(hi))
#define KB_SET_ARENA_SAFE(lo, hi, slo, shi) \
    ::karma::engine::kb_set_arena((uintptr_t)(lo), (uintptr_t)(hi), (uintptr_t)(slo), (uintptr_t)(shi))
#endif  // __HIP__

#else  // the shipped build: plain accesses

#define KB_READ(arr, idx, cap, site) ((arr)[idx])
#define KB_WRITE(arr, idx, cap, site, v) \
    do {                                 \
        (arr)[idx] = (v);                \
    } while (0)
#define KB_BYTES(p, n) (p)
#define KB_SET_ARENA(lo, hi) \
    do {                     \
    } while (0)
#define KB_SET_ARENA_SAFE(lo, hi, slo, shi) \
    do {                                  \
    } while (0)
#define KB_DEFINE_COLLECT(name)

#endif
