// karma_amd/csrc/wal_device.hip -- WAL replay on the device.
//
// sivir::open's loop over wal::scan_record (sivir.cc:31-41, wal.cc:34-87) over a
// WAL image held in HBM, in three kernels around one ragged CRC batch:
//
//   k_wal_walk     one workgroup per segment: the segment is staged through LDS
//                  in 16 KiB tiles and one lane walks its [crc][len<<8|type]
//                  headers with scan_record's structural checks, writing the
//                  header offset and payload length of every type-0 record
//                  (the candidates) and the segment's stop kind / offset.  The
//                  header chain is serial inside a segment; segments walk in
//                  parallel, replacing the host's per-record pread loop.
//   k_wal_gather   candidates of the segments replay enters, in WAL order,
//                  into contiguous (header offset, length) lists + stored CRCs
//   (ragged batch) payload CRCs: the arena is the image shifted by the 8-byte
//                  header, so the list of header offsets is the offset list
//   k_wal_compare  the first candidate whose payload CRC differs (atomicMin)
//
// The size-0 quirk is kept: read_exact_at returns early for size 0
// (segment_file.cc:8), so the CRC compared is that of the stale 4-byte len/type
// word (wal.cc:50-60); the walk checks it in place.
#include <hip/hip_runtime.h>

#include <cstdlib>

#include "engine.h"
#include "karma_crc32c.h"

namespace karma {
namespace engine {
namespace {

constexpr int kWalkThreads = 256;
constexpr uint32_t kTile = 16384;          // LDS tile of the walk (two buffers)
constexpr uint32_t kTileLoad = kTile + 16;  // + one header's slack (16-byte multiple)
static_assert(kTileLoad % 16 == 0, "tile of whole vectors");

// crc32c::Value of 4 bytes (the stale len/type word of a size-0 record), bitwise.
__device__ __forceinline__ uint32_t crc_word(uint32_t w) {
    uint32_t l = 0xFFFFFFFFu ^ w;
#pragma unroll
    for (int i = 0; i < 32; ++i) l = (l >> 1) ^ (0x82F63B78u & (0u - (l & 1u)));
    return l ^ 0xFFFFFFFFu;
}

// The walker (thread 0) keeps its position in 32 bits (seg_bytes < 2^31) and
// reads each header as three aligned LDS words funnel-shifted into place; the
// common header (type 0, payload that fits) costs one branch.  Its candidates
// go to an LDS list.  While it walks tile t, waves 1-3 write the previous
// tile's list out to global memory (coalesced) and load tile t + 1 into the
// other buffer, so the walker waits neither on tile loads nor on stores; a
// payload that jumps past tile t + 1 costs one synchronous tile load.
__global__ __launch_bounds__(kWalkThreads) void k_wal_walk(WalArgs A) {
    __shared__ __attribute__((aligned(16))) uint32_t tile[2][kTileLoad / 4 + 4];
    __shared__ uint32_t lrec[2][kTile / 8 + 1], llen[2][kTile / 8 + 1];
    __shared__ uint32_t sh_pos, sh_done, sh_n;
    const uint32_t seg = (uint32_t)A.seg_bytes;
    const uint64_t rel = (uint64_t)blockIdx.x * A.seg_bytes;  // segment s0 + blockIdx.x, relative to A.wal
    const uint64_t base = A.base0 + rel;                      // its WAL offset
    const uint8_t* img = A.wal + rel;
    uint32_t* crec = A.cand_rec + blockIdx.x * A.cand_cap;
    uint32_t* clen = A.cand_len + blockIdx.x * A.cand_cap;
    const bool vec = ((reinterpret_cast<uintptr_t>(img)) & 15u) == 0;
    auto load = [&](int b, uint32_t t0, uint32_t tid, uint32_t nthr) {  // [t0, t0 + kTileLoad) clipped to seg
        const uint32_t n = (uint64_t)t0 + kTileLoad < seg ? kTileLoad : seg - t0;
        uint8_t* tb = reinterpret_cast<uint8_t*>(tile[b]);
        uint32_t i0 = 0;
        if (vec) {  // whole 16-byte vectors, then the tail bytes
            const uint32_t nv = n / 16;
            for (uint32_t i = tid; i < nv; i += nthr)
                reinterpret_cast<uint4*>(tb)[i] = reinterpret_cast<const uint4*>(img + t0)[i];
            i0 = nv * 16;
        }
        for (uint32_t i = i0 + tid; i < n; i += nthr) tb[i] = img[t0 + i];
    };
    auto flush = [&](int b, uint32_t nc, uint32_t at, uint32_t tid, uint32_t nthr) {
        for (uint32_t i = tid; i < nc; i += nthr)
            if (at + i < A.cand_cap) {
                crec[at + i] = lrec[b][i];
                clen[at + i] = llen[b][i];
            }
    };
    // uniform: every thread follows the walker through sh_pos
    uint32_t pos = blockIdx.x == 0 ? (uint32_t)A.first_pos : 0u;
    uint32_t count = 0, kind = 0, stop = seg;  // stop: segment-relative (thread 0's)
    uint32_t pend_n = 0, pend_at = 0;          // the list of the previous tile, not yet written out
    int b = 0;
    if ((uint64_t)pos + 8 <= seg) {  // wal.cc:40-45: a shorter rest is skipped (kind 0)
        load(0, pos / kTile * kTile, threadIdx.x, kWalkThreads);
        __syncthreads();
        while (true) {
            const uint32_t t0 = pos / kTile * kTile;
            if (threadIdx.x == 0) {
                const uint32_t* tl = tile[b];
                uint32_t done = 0, nc = 0;
                const uint32_t tend = t0 + kTile, lim = seg - 8;  // a header at pos needs pos <= lim
                while (pos <= lim && pos < tend) {
                    // fast path: type-0 records with a payload that fits, one branch per header
                    uint32_t crc, st, size, npos;
                    while (true) {
                        const uint32_t h = pos - t0, q = h >> 2, sh = h & 3u;
                        const uint32_t w0 = tl[q], w1 = tl[q + 1], w2 = tl[q + 2];
                        crc = __builtin_amdgcn_alignbyte(w1, w0, sh);
                        st = __builtin_amdgcn_alignbyte(w2, w1, sh);
                        size = st >> 8;
                        npos = pos + 8 + size;  // < 2^32: seg_bytes < 2^31, size < 2^24
                        if ((st & 0xffu) != 0 || size == 0 || npos > seg) break;
                        lrec[b][nc] = pos;
                        llen[b][nc] = size;
                        ++nc;
                        pos = npos;
                        if (pos > lim || pos >= tend) break;
                    }
                    if (pos > lim || pos >= tend) break;  // left the segment / tile on the fast path
                    // the header at pos is special (scan_record's other branches)
                    const uint32_t type = st & 0xffu;
                    if (type == 0 && npos <= seg && crc_word(st) == crc) {  // size 0: stale word (wal.cc:50-60)
                        lrec[b][nc] = pos;
                        llen[b][nc] = 0;
                        ++nc;
                        pos = npos;
                        continue;
                    }
                    done = 1;
                    if (type == 0) {  // wal.cc:71-74 (length past the segment), or the stale-word mismatch
                        kind = KARMA_WAL_CORRUPT;
                        stop = pos;
                    } else if (type == 1) {  // padding: skip to the segment end (wal.cc:76-82)
                        pos = seg;
                    } else {
                        kind = KARMA_WAL_BAD_TYPE;
                        stop = pos;
                    }
                    break;
                }
                sh_pos = pos;
                sh_done = done;
                sh_n = nc;
            } else if (threadIdx.x >= 64) {  // waves 1-3: the previous list out, the next tile in
                flush(b ^ 1, pend_n, pend_at, threadIdx.x - 64, kWalkThreads - 64);
                if ((uint64_t)t0 + kTile < seg) load(b ^ 1, t0 + kTile, threadIdx.x - 64, kWalkThreads - 64);
            }
            __syncthreads();
            pos = sh_pos;
            const uint32_t done = sh_done, nc = sh_n;
            pend_n = nc;
            pend_at = count;
            count += nc;
            if (done || (uint64_t)pos + 8 > seg) {
                flush(b, nc, pend_at, threadIdx.x, kWalkThreads);
                break;
            }
            const uint32_t nt0 = pos / kTile * kTile;
            if (nt0 != t0 + kTile) {  // jumped past the prefetched tile
                load(b ^ 1, nt0, threadIdx.x, kWalkThreads);
            }
            __syncthreads();  // sh_* are read by everyone before the walker rewrites them
            b ^= 1;
        }
    }
    if (threadIdx.x == 0) A.meta[blockIdx.x] = WalSegMeta{count, kind, base + (kind ? stop : seg)};
}

// One wave per segment (64 threads, ~8.5 KiB of LDS: many segments walk at
// once).  The segment passes through one 4 KiB LDS tile; every lane holds 64
// bytes of the NEXT tile in registers, loaded while lane 0 walks the current
// one, so dense headers never wait on a load and a payload that jumps past the
// next tile costs one 4 KiB load (instead of streaming the whole segment).
template <uint32_t kWTile>
__global__ __launch_bounds__(64) void k_wal_walk_wave(WalArgs A) {
    constexpr int QV = kWTile / 1024;  // 16-byte vectors per lane per tile
    __shared__ __attribute__((aligned(16))) uint32_t tile[kWTile / 4 + 4];  // + a header's slack
    __shared__ uint32_t lrec[kWTile / 8 + 1], llen[kWTile / 8 + 1];
    const uint32_t lane = threadIdx.x;
    const uint32_t seg = (uint32_t)A.seg_bytes;
    const uint64_t rel = (uint64_t)blockIdx.x * A.seg_bytes;
    const uint64_t base = A.base0 + rel;
    const uint8_t* img = A.wal + rel;
    uint32_t* crec = A.cand_rec + blockIdx.x * A.cand_cap;
    uint32_t* clen = A.cand_len + blockIdx.x * A.cand_cap;
    const bool vec = ((reinterpret_cast<uintptr_t>(img)) & 15u) == 0;
    // this lane's share of the tile at t: vectors lane + 64 q (q < QV) and the slack vector.
    // The fast case is branch-free: a per-lane branch around a load makes the compiler wait
    // for every outstanding load at the join (vmcnt counts in order), and the prefetch
    // would no longer overlap the walk.
    auto fetch = [&](uint32_t t, uint4 (&r)[QV + 1]) {
        if (vec && (uint64_t)t + kWTile + 16 <= seg) {  // uniform: whole vectors
#pragma unroll
            for (int q = 0; q < QV; ++q) r[q] = *reinterpret_cast<const uint4*>(img + t + (lane + 64u * q) * 16u);
            r[QV] = *reinterpret_cast<const uint4*>(img + t + kWTile);  // the slack (every lane, one line)
            return;
        }
        // the segment's last tile, or a misaligned segment: bytes inside the segment, zeros past it
#pragma unroll
        for (int q = 0; q <= QV; ++q) {
            const uint32_t o = q < QV ? (lane + 64u * q) * 16u : kWTile;
            uint32_t w[4] = {0u, 0u, 0u, 0u};
            for (uint32_t b = 0; b < 16; ++b)
                if ((uint64_t)t + o + b < seg) w[b >> 2] |= uint32_t(img[t + o + b]) << (8 * (b & 3));
            r[q] = uint4{w[0], w[1], w[2], w[3]};
        }
    };
    auto store = [&](const uint4 (&r)[QV + 1]) {
#pragma unroll
        for (int q = 0; q < QV; ++q) reinterpret_cast<uint4*>(tile)[lane + 64u * q] = r[q];
        if (lane == 0) reinterpret_cast<uint4*>(tile)[kWTile / 16] = r[QV];
        __syncthreads();  // one wave: orders the tile writes before the walker's reads
    };
    uint32_t pos = blockIdx.x == 0 ? (uint32_t)A.first_pos : 0u;
    uint32_t count = 0, kind = 0, stop = seg;
    if ((uint64_t)pos + 8 <= seg) {  // wal.cc:40-45: a shorter rest is skipped (kind 0)
        uint32_t t0 = pos / kWTile * kWTile;
        uint4 r[QV + 1];  // this lane's share of the next tile
        fetch(t0, r);
        store(r);
        while (true) {
            const bool more = (uint64_t)t0 + kWTile < seg;
            if (more) fetch(t0 + kWTile, r);  // in flight while lane 0 walks
            // Every lane runs the walk on identical values (uniform control flow, so the
            // compiler keeps the header chain in scalar registers); lane 0 writes the list.
            uint32_t done = 0, nc = 0;
            {
                const uint32_t tend = t0 + kWTile, lim = seg - 8;
                while (pos <= lim && pos < tend) {
                    uint32_t crc, st, size, npos;
                    while (true) {  // fast path: type-0 records with a payload that fits
                        const uint32_t h = pos - t0, q = h >> 2, sh = h & 3u;
                        const uint32_t w0 = tile[q], w1 = tile[q + 1], w2 = tile[q + 2];
                        crc = __builtin_amdgcn_readfirstlane(__builtin_amdgcn_alignbyte(w1, w0, sh));
                        st = __builtin_amdgcn_readfirstlane(__builtin_amdgcn_alignbyte(w2, w1, sh));
                        size = st >> 8;
                        npos = pos + 8 + size;
                        if ((st & 0xffu) != 0 || size == 0 || npos > seg) break;
                        if (lane == 0) {
                            lrec[nc] = pos;
                            llen[nc] = size;
                        }
                        ++nc;
                        pos = npos;
                        if (pos > lim || pos >= tend) break;
                    }
                    if (pos > lim || pos >= tend) break;
                    const uint32_t type = st & 0xffu;
                    if (type == 0 && npos <= seg && crc_word(st) == crc) {  // size 0: stale word (wal.cc:50-60)
                        if (lane == 0) {
                            lrec[nc] = pos;
                            llen[nc] = 0;
                        }
                        ++nc;
                        pos = npos;
                        continue;
                    }
                    done = 1;
                    if (type == 0) {
                        kind = KARMA_WAL_CORRUPT;
                        stop = pos;
                    } else if (type == 1) {
                        pos = seg;
                    } else {
                        kind = KARMA_WAL_BAD_TYPE;
                        stop = pos;
                    }
                    break;
                }
            }
            __syncthreads();  // lane 0's list writes before the others read them
            for (uint32_t i = lane; i < nc; i += 64)
                if (count + i < A.cand_cap) {
                    crec[count + i] = lrec[i];
                    clen[count + i] = llen[i];
                }
            count += nc;
            if (done || (uint64_t)pos + 8 > seg) break;
            const uint32_t nt0 = pos / kWTile * kWTile;
            __syncthreads();  // everyone has read the list and the tile
            if (more && nt0 == t0 + kWTile) {
                store(r);  // the prefetched tile
            } else {
                fetch(nt0, r);  // jumped past it
                store(r);
            }
            t0 = nt0;
        }
    }
    if (lane == 0) A.meta[blockIdx.x] = WalSegMeta{count, kind, base + (kind ? stop : seg)};
}

// Candidates of segment s0 + blockIdx.x (one block per segment) into the
// contiguous lists at slot A.cand_base[blockIdx.x]: header offset (relative to
// A.wal), length and the CRC field stored in the header.
__global__ __launch_bounds__(256) void k_wal_gather(WalArgs A) {
    const uint64_t rel = (uint64_t)blockIdx.x * A.seg_bytes;
    const uint32_t count = A.meta[blockIdx.x].count;
    const uint64_t g0 = A.cand_base[blockIdx.x];
    const uint32_t* crec = A.cand_rec + blockIdx.x * A.cand_cap;
    const uint32_t* clen = A.cand_len + blockIdx.x * A.cand_cap;
    for (uint32_t j = threadIdx.x; j < count; j += blockDim.x) {
        const uint64_t rec = rel + crec[j];
        const uint8_t* h = A.wal + rec;
        A.off[g0 + j] = rec;
        A.len[g0 + j] = clen[j];
        A.stored[g0 + j] = uint32_t(h[0]) | uint32_t(h[1]) << 8 | uint32_t(h[2]) << 16 | uint32_t(h[3]) << 24;
    }
}

// The first candidate (in WAL order) whose payload CRC differs from the stored
// one; size-0 records were checked by the walk.
__global__ __launch_bounds__(256) void k_wal_compare(WalArgs A, uint64_t n) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    uint64_t first = ~0ull;
    for (uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; g < n; g += stride)
        if (A.len[g] && A.crc[g] != A.stored[g]) {
            first = g;
            break;  // later g of this thread are larger
        }
    if (first != ~0ull) atomicMin(reinterpret_cast<unsigned long long*>(A.first_bad), (unsigned long long)first);
}

}  // namespace

// Few segments (no more than two per CU): a workgroup per segment, whose helper
// waves keep the walking lane fed (1M x 180 B records in 188 segments: 0.75 ms
// against 0.94 ms for the one-wave walker). Many segments: one wave per segment
// with 4 KiB tiles, many segments per CU (configs[2]'s mix in 4,300 segments:
// 0.44 ms against 1.55 ms; 8 or 16 KiB tiles measured 0.60 and 0.84 ms).
// KARMA_WALK_VARIANT=1 / 2 forces the workgroup / the one-wave walker (tests).
hipError_t launch_wal_walk(const WalArgs& a, uint64_t nseg, int cu, hipStream_t s) {
    if (!nseg) return hipSuccess;
    const char* e = getenv("KARMA_WALK_VARIANT");
    const int v = e && *e ? atoi(e) : (nseg <= 2 * (uint64_t)cu ? 1 : 2);
    if (v == 1)
        hipLaunchKernelGGL(k_wal_walk, dim3((unsigned)nseg), dim3(kWalkThreads), 0, s, a);
    else
        hipLaunchKernelGGL(k_wal_walk_wave<4096>, dim3((unsigned)nseg), dim3(64), 0, s, a);
    return hipGetLastError();
}

hipError_t launch_wal_gather(const WalArgs& a, uint64_t nseg, hipStream_t s) {
    if (!nseg) return hipSuccess;
    hipLaunchKernelGGL(k_wal_gather, dim3((unsigned)nseg), dim3(256), 0, s, a);
    return hipGetLastError();
}

hipError_t launch_wal_compare(const WalArgs& a, uint64_t n, int cu, hipStream_t s) {
    if (!n) return hipSuccess;
    uint64_t blocks = (n + 255) / 256;
    if (blocks > (uint64_t)cu * 8) blocks = (uint64_t)cu * 8;
    hipLaunchKernelGGL(k_wal_compare, dim3((unsigned)blocks), dim3(256), 0, s, a, n);
    return hipGetLastError();
}

}  // namespace engine
}  // namespace karma
