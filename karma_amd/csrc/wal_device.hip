// karma_amd/csrc/wal_device.hip -- WAL replay on the device.
//
// sivir::open's loop over wal::scan_record (sivir.cc:31-41, wal.cc:34-87) over a
// WAL image held in HBM, in a few kernels around one ragged CRC batch:
//
//   k_wal_walk_sub  the header walk: one wave per segment, or (few segments) one
//                   wave per sub-range of a segment, walking the [crc][len<<8|type]
//                   headers with scan_record's structural checks through a 4 KiB
//                   LDS tile, and writing the header offset, payload length and
//                   stored CRC of every type-0 record (the candidates) and the stop
//                   kind / offset.  The header chain is serial; segments and
//                   sub-ranges walk in parallel, replacing the host's pread loop.
//   k_wal_resolve   (sub-ranges) stitches the walkers' lists along the real chain
//   k_wal_walk      the same walk with one workgroup per segment (tools build only)
//   k_wal_gather    candidates of the segments replay enters, in WAL order, into
//                   contiguous (header offset, length, stored CRC) lists
//   (ragged batch)  payload CRCs: the arena is the image shifted by the 8-byte
//                   header, so the list of header offsets is the offset list
//   k_wal_compare   the first candidate whose payload CRC differs (atomicMin)
//
// The size-0 quirk is kept: read_exact_at returns early for size 0
// (segment_file.cc:8), so the CRC compared is that of the stale 4-byte len/type
// word (wal.cc:50-60); the walk checks it in place.  An accepted size-0 record is 12
// bytes long to sivir::open: scan_record appends the 4 stale bytes (wal.cc:66) and the
// loop advances by record.size() (sivir.cc:38), so the next header is read at +12
// (kStaleAdvance); past the segment end the walk reports kWalSpill (engine.h).
#include <hip/hip_runtime.h>

#include <algorithm>

#include "ab.h"
#include "bounds.h"
#include "crc_device.h"
#include "engine.h"
#include "karma_crc32c.h"

namespace karma {
namespace engine {
namespace {
using namespace dev;

// crc32c::Value of the stale len/type word of a size-0 record.  A type-0 record
// of size 0 has the word 0, so the value is a constant: Value("\0\0\0\0").
constexpr uint32_t crc_word_host(uint32_t w) {
    uint32_t l = 0xFFFFFFFFu ^ w;
    for (int i = 0; i < 32; ++i) l = (l >> 1) ^ (0x82F63B78u & (0u - (l & 1u)));
    return l ^ 0xFFFFFFFFu;
}
constexpr uint32_t kStaleZero = crc_word_host(0);
static_assert(kStaleZero == 0x48674BC7u, "crc32c::Value of four zero bytes");
// Inline CRC results (k_wal_walk_crc) in WalSubMeta::pad[0] / WalSegMeta::first_bad.
constexpr uint32_t kNoBad = ~0u;           // no mismatch
constexpr uint32_t kCrcUnknown = ~0u - 1;  // some candidate was not checksummed inline

// sivir::open's advance over an accepted size-0 record: 8 header bytes + the 4 stale bytes
// scan_record appended to it (wal.cc:47-51, :66; sivir.cc:38).
constexpr uint32_t kStaleAdvance = 12;

#ifdef KARMA_AB  // k_wal_walk: the workgroup walker, tools build only (ab.h)
constexpr int kWalkThreads = 256;
constexpr uint32_t kTile = 16384;          // LDS tile of the walk (two buffers)
constexpr uint32_t kTileLoad = kTile + 16;  // + one header's slack (16-byte multiple)
static_assert(kTileLoad % 16 == 0, "tile of whole vectors");

// The walker (thread 0) keeps its position in 32 bits (seg_bytes < 2^31) and
// reads each header as three aligned LDS words funnel-shifted into place; the
// common header (type 0, payload that fits) costs one branch.  Its candidates
// go to an LDS list.  While it walks tile t, waves 1-3 write the previous
// tile's list out to global memory (coalesced) and load tile t + 1 into the
// other buffer, so the walker waits neither on tile loads nor on stores; a
// payload that jumps past tile t + 1 costs one synchronous tile load.
__global__ __launch_bounds__(kWalkThreads) void k_wal_walk(WalArgs A) {
    __shared__ __attribute__((aligned(16))) uint32_t tile[2][kTileLoad / 4 + 4];
    __shared__ uint32_t lrec[2][kTile / 8 + 1], llen[2][kTile / 8 + 1], lcrc[2][kTile / 8 + 1];
    __shared__ uint32_t sh_pos, sh_done, sh_n;
    const uint32_t seg = (uint32_t)A.seg_bytes;
    const uint64_t rel = (uint64_t)blockIdx.x * A.seg_bytes;  // segment s0 + blockIdx.x, relative to A.wal
    const uint64_t base = A.base0 + rel;                      // its WAL offset
    const uint8_t* img = A.wal + rel;
    uint32_t* crec = A.cand_rec + blockIdx.x * A.cand_cap;
    uint32_t* clen = A.cand_len + blockIdx.x * A.cand_cap;
    uint32_t* ccrc = A.cand_crc + blockIdx.x * A.cand_cap;
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
                ccrc[at + i] = lcrc[b][i];
            }
    };
    // uniform: every thread follows the walker through sh_pos
    uint32_t pos = blockIdx.x == 0 ? (uint32_t)A.first_pos : 0u;
    uint32_t count = 0, kind = 0, stop = seg;  // stop: segment-relative (thread 0's)
    uint32_t mx = 0;                            // thread 0's largest payload
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
                        lcrc[b][nc] = crc;
                        mx = size > mx ? size : mx;
                        ++nc;
                        pos = npos;
                        if (pos > lim || pos >= tend) break;
                    }
                    if (pos > lim || pos >= tend) break;  // left the segment / tile on the fast path
                    // the header at pos is special (scan_record's other branches)
                    const uint32_t type = st & 0xffu;
                    if (type == 0 && npos <= seg && crc == kStaleZero) {  // size 0: stale word (wal.cc:50-60)
                        lrec[b][nc] = pos;
                        llen[b][nc] = 0;
                        lcrc[b][nc] = crc;
                        ++nc;
                        pos += kStaleAdvance;  // record.size() = 12 (wal.cc:66, sivir.cc:38)
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
    if (threadIdx.x == 0) {
        if (!kind && pos > seg) {  // a size-0 record's advance left the segment (kWalSpill)
            kind = kWalSpill;
            stop = pos;
        }
        A.meta[blockIdx.x] = WalSegMeta{count, kind, base + (kind ? stop : seg), mx, kCrcUnknown};
        A.span[2 * blockIdx.x] = 0;
        A.span[2 * blockIdx.x + 1] = 0;
    }
}

#endif

// ---- one-wave walkers -------------------------------------------------------
// A wave walks through one 4 KiB LDS tile (4 KiB of LDS: many walkers per CU).  Every lane holds 64 bytes of the NEXT tile in registers,
// loaded while the walk runs on the current one, so dense headers never wait on
// a load and a payload that jumps past the next tile costs one 4 KiB load
// (instead of streaming the whole segment).  The walk runs on every lane with
// identical values (uniform control flow keeps the header chain in scalar
// registers).
constexpr uint32_t kWTile = kWalkTile;
constexpr int kWQV = kWTile / 1024;  // 16-byte vectors per lane per tile
constexpr uint32_t kChainCheck = 4;  // headers a sub-range walker's start must chain through

struct WaveLds {
    uint32_t tile[kWTile / 4 + 4];  // + a header's slack
};

// Orders one walker's LDS tile accesses (its tile writes before its header reads, and the
// reverse).  A walker alone in its workgroup (k_wal_walk_sub, k_wal_resolve): a barrier.
// WG: the fused kernel's workgroup of kFuseWaves independent walkers (k_wal_walk_crc): only
// this wave's LDS accesses are waited for -- a workgroup barrier would tie the walkers together.
template <bool WG>
__device__ __forceinline__ void wave_sync() {
    if constexpr (WG) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0)
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    } else {
        __syncthreads();
    }
}

struct Seg {  // one segment as a walker sees it
    const uint8_t* img;
    uint32_t seg;
    bool vec;  // img 16-byte aligned
#ifdef KARMA_BOUNDS
    const uint8_t* wlo;  // the image (bounds build: every byte read must lie in it)
    const uint8_t* whi;
#endif
};

__device__ __forceinline__ Seg make_seg(const WalArgs& A, uint64_t s) {
    const uint8_t* img = A.wal + s * A.seg_bytes;
#ifdef KARMA_BOUNDS
    return Seg{img, (uint32_t)A.seg_bytes, (reinterpret_cast<uintptr_t>(img) & 15u) == 0, A.wal, A.wal + A.img_bytes};
#else
    return Seg{img, (uint32_t)A.seg_bytes, (reinterpret_cast<uintptr_t>(img) & 15u) == 0};
#endif
}

// S.img + off for an n-byte read (the bounds build checks it against the segment and the image).
__device__ __forceinline__ const uint8_t* seg_at(const Seg& S, uint64_t off, uint32_t n) {
#ifdef KARMA_BOUNDS
    if (!kb_ok(off + n <= S.seg, kKbSegment, off, S.seg)) return S.img;
    const uint8_t* p = S.img + off;
    if (!kb_ok(p >= S.wlo && p + n <= S.whi, kKbImage, (uint64_t)(p - S.wlo), (uint64_t)(S.whi - S.wlo))) return S.wlo;
    return p;
#else
    (void)n;
    return S.img + off;
#endif
}

// This lane's share of the tile at t: vectors lane + 64 q (q < kWQV) and the slack
// vector.  The fast case is branch-free: a per-lane branch around a load makes the
// compiler wait for every outstanding load at the join (vmcnt counts in order), and
// the prefetch would no longer overlap the walk.
__device__ __forceinline__ void wtile_fetch(const Seg& S, uint32_t lane, uint32_t t, uint4 (&r)[kWQV + 1]) {
    if (S.vec && (uint64_t)t + kWTile + 16 <= S.seg) {  // uniform: whole vectors
#pragma unroll
        for (int q = 0; q < kWQV; ++q) r[q] = *reinterpret_cast<const uint4*>(seg_at(S, t + (lane + 64u * q) * 16u, 16));
        r[kWQV] = *reinterpret_cast<const uint4*>(seg_at(S, t + kWTile, 16));  // the slack (every lane, one line)
        return;
    }
    // the segment's last tile, or a misaligned segment: bytes inside the segment, zeros past it
#pragma unroll
    for (int q = 0; q <= kWQV; ++q) {
        const uint32_t o = q < kWQV ? (lane + 64u * q) * 16u : kWTile;
        uint32_t w[4] = {0u, 0u, 0u, 0u};
        for (uint32_t b = 0; b < 16; ++b)
            if ((uint64_t)t + o + b < S.seg) w[b >> 2] |= uint32_t(*seg_at(S, t + o + b, 1)) << (8 * (b & 3));
        r[q] = uint4{w[0], w[1], w[2], w[3]};
    }
}

template <bool WG = false>
__device__ __forceinline__ void wtile_store(WaveLds& W, uint32_t lane, const uint4 (&r)[kWQV + 1]) {
#pragma unroll
    for (int q = 0; q < kWQV; ++q) reinterpret_cast<uint4*>(W.tile)[lane + 64u * q] = r[q];
    if (lane == 0) reinterpret_cast<uint4*>(W.tile)[kWTile / 16] = r[kWQV];
    wave_sync<WG>();  // orders the tile writes before the walker's reads
}

// A 1 KiB window at t (16-byte aligned): one vector per lane + the slack, for a
// walk that jumps (one header per window: a 4 KiB tile and its prefetch would
// read 8 KiB per header).
constexpr uint32_t kWSmall = 1024;
__device__ __forceinline__ void wsmall_fetch(const Seg& S, uint32_t lane, uint32_t t, uint4& v, uint4& slack) {
    if (S.vec && (uint64_t)t + kWSmall + 16 <= S.seg) {
        v = *reinterpret_cast<const uint4*>(seg_at(S, t + lane * 16u, 16));
        slack = *reinterpret_cast<const uint4*>(seg_at(S, t + kWSmall, 16));
        return;
    }
    uint32_t w[8] = {0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u};
    for (uint32_t b = 0; b < 16; ++b) {
        if ((uint64_t)t + lane * 16u + b < S.seg) w[b >> 2] |= uint32_t(*seg_at(S, t + lane * 16u + b, 1)) << (8 * (b & 3));
        if ((uint64_t)t + kWSmall + b < S.seg) w[4 + (b >> 2)] |= uint32_t(*seg_at(S, t + kWSmall + b, 1)) << (8 * (b & 3));
    }
    v = uint4{w[0], w[1], w[2], w[3]};
    slack = uint4{w[4], w[5], w[6], w[7]};
}

template <bool WG = false>
__device__ __forceinline__ void wsmall_store(WaveLds& W, uint32_t lane, const uint4& v, const uint4& slack) {
    reinterpret_cast<uint4*>(W.tile)[lane] = v;
    if (lane == 0) reinterpret_cast<uint4*>(W.tile)[kWSmall / 16] = slack;
    wave_sync<WG>();
}

// The header at segment offset c, read from the tile at t0 (c - t0 < kWTile).
__device__ __forceinline__ void tile_header(const WaveLds& W, uint32_t c, uint32_t t0, uint32_t& crc, uint32_t& st) {
    const uint32_t h = c - t0, q = h >> 2, sh = h & 3u;
    const uint32_t w0 = W.tile[q], w1 = W.tile[q + 1], w2 = W.tile[q + 2];
    crc = __builtin_amdgcn_alignbyte(w1, w0, sh);
    st = __builtin_amdgcn_alignbyte(w2, w1, sh);
}

// The fused walker's inline CRCs (k_wal_walk_crc): the LDS image (16-copy stride tables of the
// quad blob, small tables at kSmallBase), its lane constant and the safe address of empty units.
struct CrcCtx {
    const uint32_t* lds;
    uint32_t X;
    const uint8_t* safe;
};
constexpr uint32_t kCrcInlineMax = 1024;  // payloads the walker checksums itself (4-lane groups)

struct WalkEnd {
    uint32_t count;  // candidates written
    uint32_t max_len;  // their largest payload
    uint32_t kind;   // KARMA_WAL_CORRUPT / _BAD_TYPE, or 0
    uint32_t stop;   // where kind was found
    uint32_t pos;    // where the walk left off (seg after a type-1 padding record; up to seg + 4
                     // after a size-0 record at the segment end: kWalSpill)
};

// The fused kernel's second phase: the walker's own list [slot0, slot0 + count), 64 entries at
// a time (read back from the slots it just wrote), checksummed by groups of 4 lanes
// (direct_batch, the small-record kernel's body, through the 16-copy tables) and compared with
// the stored CRCs.  Returns the first mismatching entry (kNoBad: none), or kCrcUnknown when a
// payload is over kCrcInlineMax (the replay then takes the unit plan).
__device__ uint32_t crc_list(const CrcCtx& C, const Seg& S, const WalArgs& A, uint32_t lane, uint64_t slot0,
                             uint32_t count, uint32_t max_len) {
    if (!count) return kNoBad;
    if (max_len > kCrcInlineMax) return kCrcUnknown;
    const uint64_t total = A.nwork * A.cand_cap;
    (void)total;
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");  // the list writes before their reads
    __builtin_amdgcn_s_waitcnt(0);
    for (uint32_t i0 = 0; i0 < count; i0 += 64) {
        const uint32_t i = i0 + lane;
        const bool v = i < count;
        uint32_t rec = 0, n = 0, st = 0;
        if (v) {
            rec = KB_READ(A.cand_rec, slot0 + i, total, kKbCand);
            n = KB_READ(A.cand_len, slot0 + i, total, kKbCand);
            st = KB_READ(A.cand_crc, slot0 + i, total, kKbCand);
        }
        const uint8_t* p = v ? S.img + rec + 8 : C.safe;
        const uint32_t res = direct_batch<4, 4, true, 24>(C.lds, C.X, C.safe, p, n, 0u, v);
        const uint64_t bm = __ballot(v && n != 0 && res != st);  // size 0: checked by the walk
        if (bm) return i0 + (uint32_t)__builtin_ctzll(bm);
    }
    return kNoBad;
}

// Walk the header chain from pos while pos < hi, with scan_record's checks (wal.cc:34-87):
// a rest shorter than a header ends the segment, type 0 with a payload that fits
// is a candidate, a size-0 record compares the stored CRC with Value of the stale
// len/type word (wal.cc:50-60), type 1 skips to the segment end, anything else
// stops the walk.  Candidates go to crec / clen (cap slots).
// resident: the tile start W already holds (find_start's tile), or ~0u.
template <bool WG = false>
__device__ WalkEnd walk_range(WaveLds& W, const Seg& S, uint32_t lane, uint32_t pos, uint32_t hi, const WalArgs& A,
                              uint64_t slot0, uint64_t cap, uint32_t resident = ~0u) {
    const uint64_t total = A.nwork * A.cand_cap;  // every list slot (bounds build)
    (void)total;
    auto put = [&](uint64_t i, uint32_t rec, uint32_t n, uint32_t c) {  // list entry i (< cap: else dropped)
#ifdef KARMA_BOUNDS
        kb_ok(i < cap, kKbCandDropped, i, cap);
#endif
        if (i < cap) {
            KB_WRITE(A.cand_rec, slot0 + i, total, kKbCand, rec);
            KB_WRITE(A.cand_len, slot0 + i, total, kKbCand, n);
            KB_WRITE(A.cand_crc, slot0 + i, total, kKbCand, c);
        }
    };
    const uint32_t seg = S.seg;
    WalkEnd E{0u, 0u, 0u, seg, pos};
    if ((uint64_t)pos + 8 > seg || pos >= hi) return E;  // wal.cc:40-45: a shorter rest is skipped
    // The list is built in registers, entry i of each run of 64 in lane i, and written
    // out 64 entries at a time (coalesced): no LDS traffic besides the header reads.
    uint32_t myrec = 0, mylen = 0, mycrc = 0, k = 0, vmax = 0;  // vmax: per lane, reduced at the end
    // Append entries 0..na-1 (entry j in lane j of rec_j / len_j / crc_j) to the run: run
    // lane (k + j) mod 64 takes entry j, the run is written out when it fills.
    // (Round 5 measured each round's entries written straight to their list slots instead, no
    // rotation into run registers: 0.1154 vs 0.1123 ms per rotated call, profiles/r05_replay_walk_put_ab.txt.)
    auto push_many = [&](uint32_t rec_j, uint32_t len_j, uint32_t crc_j, uint32_t na) {
        const uint32_t src = (lane - k) & 63u;
        const uint32_t r = __shfl(rec_j, (int)src), n = __shfl(len_j, (int)src), c = __shfl(crc_j, (int)src);
        const bool take = src < na;
        if (take && lane >= k) {
            myrec = r;
            mylen = n;
            mycrc = c;
            vmax = n > vmax ? n : vmax;
        }
        if (k + na >= 64) {
            put(E.count + lane, myrec, mylen, mycrc);
            E.count += 64;
            if (take && lane < k) {  // the entries that wrapped into the next run
                myrec = r;
                mylen = n;
                mycrc = c;
                vmax = n > vmax ? n : vmax;
            }
            k = k + na - 64;
        } else {
            k += na;
        }
    };
    auto push = [&](uint32_t p, uint32_t n, uint32_t c) { push_many(p, n, c, 1u); };  // uniform values
    uint32_t g = 0;  // the guessed header stride: 8 + the last record's size
    uint32_t streak = 0;  // headers the last fast round took (direct rounds from A.direct_streak on)
    const uint32_t tlim = hi < seg ? hi : seg;  // tiles from here on hold no header before hi
    // Sequential headers go through 4 KiB tiles with the next one prefetched; after a
    // jump past the prefetched tile the walk reads a 1 KiB window at the header, and
    // goes back to tiles when it leaves a window for the next one.
    uint32_t t0 = pos / kWTile * kWTile, tsz = kWTile;
    uint4 r[kWQV + 1];
    if (t0 != resident) {  // else find_start left this tile in W: no second load of it
        wtile_fetch(S, lane, t0, r);
        wtile_store<WG>(W, lane, r);
    }
    while (true) {
        const bool more = tsz == kWTile && (uint64_t)t0 + kWTile < tlim;
        if (more) wtile_fetch(S, lane, t0 + kWTile, r);  // in flight while the walk runs
        uint32_t done = 0;
        // Direct rounds: while the records repeat their size (the last fast round took at least
        // A.direct_streak headers), lane j reads the header at pos + j*g straight from global
        // memory -- 64 headers per memory latency instead of a 4 KiB tile per latency, and the
        // payload bytes between the headers are not read by the walk at all.  A size change keeps
        // them going while rounds stay long; a header the fast path does not take (size 0,
        // padding, a bad type or length, the sub-range end) hands pos back to the tile path.
        // (a round the tile cut short counts as long: records of more than kWTile / direct_streak
        // bytes never put direct_streak headers in one tile)
        if (A.direct_streak && g >= 8 && (streak >= A.direct_streak || (streak >= 2 && g * (streak + 1) > kWTile))) {
            const uint32_t dend = hi < seg - 7 ? hi : seg - 7;  // a header at pos needs pos + 8 <= seg
            // lane j's header of the round at base b: (crc, size/type), its position and window
            // (Round 5 measured three aligned dword loads funnel-shifted into the header instead of
            // the eight byte loads: 0.1170 vs 0.1148 ms per rotated call, profiles/r05_replay_hdr_ab.txt.)
            auto hdr = [&](uint32_t b, uint32_t& c, uint32_t& st, uint32_t& pj, bool& inwin) {
                pj = b + lane * g;  // < 2^32: b < 2^31 + 2^30, 63 g < 2^30
                inwin = pj < dend;
                const uint8_t* h = seg_at(S, inwin ? pj : pos, 8);
                c = uint32_t(h[0]) | uint32_t(h[1]) << 8 | uint32_t(h[2]) << 16 | uint32_t(h[3]) << 24;
                st = uint32_t(h[4]) | uint32_t(h[5]) << 8 | uint32_t(h[6]) << 16 | uint32_t(h[7]) << 24;
            };
            uint32_t c_, s_, pj;
            bool inwin;
            hdr(pos, c_, s_, pj, inwin);
            while (pos < dend) {
                // the next round's headers, assuming this one chains all 64 lanes at stride g
                uint32_t c2, s2, pj2;
                bool inwin2;
                hdr(pos + 64 * g, c2, s2, pj2, inwin2);
                const uint32_t hp = inwin ? pj : pos;
                const uint32_t nx = hp + 8 + (s_ >> 8);
                const bool ok = inwin && (s_ & 0xffu) == 0 && s_ >= 256u && nx <= seg;
                const uint64_t brk = __ballot(!(ok && nx == pj + g));
                const uint32_t f = brk ? (uint32_t)__builtin_ctzll(brk) : 64u;
                const uint32_t okf = f < 64 ? __builtin_amdgcn_readlane((uint32_t)ok, f) : 0u;
                const uint32_t na = f + okf;
                if (na) push_many(hp, s_ >> 8, c_, na);
                streak = na;
                if (f == 64) {  // pos + 64 g: the round already in flight is the next one
                    pos = __builtin_amdgcn_readlane(nx, 63);
                    c_ = c2;
                    s_ = s2;
                    pj = pj2;
                    inwin = inwin2;
                    continue;
                }
                if (!okf) {  // lane f's header: the tile path takes it (or the sub-range ends there)
                    pos += f * g;
                    streak = 0;
                    break;
                }
                pos = __builtin_amdgcn_readlane(nx, f);  // a size change: the round at the new stride
                g = __builtin_amdgcn_readlane(s_ >> 8, f) + 8;
                if (streak < (g * (streak + 1) > kWTile ? 2u : A.direct_streak) || pos >= dend) break;
                hdr(pos, c_, s_, pj, inwin);
            }
        }
        {
            const uint32_t tend = t0 + tsz < hi ? t0 + tsz : hi, lim = seg - 8;
            const uint32_t fend = lim + 1 < tend ? lim + 1 : tend;  // a header at pos needs pos < fend
            while (pos < fend) {
                uint32_t crc, st, npos;
                // Fast path: type-0 records with a payload that fits.  Lane j reads the header
                // at pos + j*g, g the last record's stride: when the records repeat their size
                // (the common case: a log of one record type), one round of header reads
                // accepts every header of the tile up to the first size change -- the chain is
                // confirmed lane by lane (lane j's next header is at lane j+1's position).  With
                // sizes that change every record it is one header a round, as a plain walk.
                // Only the round's outcome crosses to scalar registers (the scalar unit is
                // shared by the CU's 4 SIMDs and bounded an all-scalar walk).
                bool special = false;
                while (true) {
                    const uint32_t pj = pos + lane * g;  // < 2^32: pos < 2^31, 63 g < 2^30
                    const bool inwin = pj < fend;
                    const uint32_t hp = inwin ? pj : pos;
                    uint32_t c_, s_;
                    tile_header(W, hp, t0, c_, s_);
                    const uint32_t nx = hp + 8 + (s_ >> 8);  // < 2^32: seg < 2^31, size < 2^24
                    const bool ok = inwin && (s_ & 0xffu) == 0 && s_ >= 256u && nx <= seg;
                    const uint64_t brk = __ballot(!(ok && nx == pj + g));
                    const uint32_t f = brk ? (uint32_t)__builtin_ctzll(brk) : 64u;  // lanes < f chain on
                    const uint32_t okf = f < 64 ? __builtin_amdgcn_readlane((uint32_t)ok, f) : 0u;
                    const uint32_t na = f + okf;  // lane f's header is real too (lanes < f led to it)
                    if (na) push_many(hp, s_ >> 8, c_, na);
                    streak = na;
                    if (f == 64) {
                        pos = __builtin_amdgcn_readlane(nx, 63);
                    } else if (okf) {
                        pos = __builtin_amdgcn_readlane(nx, f);
                        g = __builtin_amdgcn_readlane(s_ >> 8, f) + 8;
                    } else {  // lane f's position holds a header the fast path does not take
                        pos += f * g;
                        if (pos < fend) {
                            crc = __builtin_amdgcn_readlane(c_, f);
                            st = __builtin_amdgcn_readlane(s_, f);
                            special = true;
                        }
                        break;
                    }
                    if (pos >= fend) break;
                }
                if (!special) break;
                npos = pos + 8 + (st >> 8);
                const uint32_t type = st & 0xffu;
                if (type == 0 && npos <= seg && crc == kStaleZero) {  // size 0: the stale word
                    push(pos, 0u, crc);
                    pos += kStaleAdvance;  // record.size() = 12 (wal.cc:66, sivir.cc:38); may pass seg
                    continue;
                }
                done = 1;
                if (type == 0) {  // wal.cc:71-74 (length past the segment), or the stale-word mismatch
                    E.kind = KARMA_WAL_CORRUPT;
                    E.stop = pos;
                } else if (type == 1) {  // padding: skip to the segment end (wal.cc:76-82)
                    pos = seg;
                } else {
                    E.kind = KARMA_WAL_BAD_TYPE;
                    E.stop = pos;
                }
                break;
            }
        }
        if (done || (uint64_t)pos + 8 > seg || pos >= hi) break;
        const uint32_t nt0 = pos / kWTile * kWTile;
        wave_sync<WG>();  // the walk's tile reads are done before the next tile is stored
        if (more && nt0 == t0 + kWTile) {  // the prefetched tile
            wtile_store<WG>(W, lane, r);
            t0 = nt0;
        } else if (pos - t0 < 2 * tsz) {  // just past a window (or a tile at the segment end): tiles again
            wtile_fetch(S, lane, nt0, r);
            wtile_store<WG>(W, lane, r);
            t0 = nt0;
            tsz = kWTile;
        } else {  // a jump: the window at the header
            uint4 v, sl;
            t0 = pos & ~15u;
            wsmall_fetch(S, lane, t0, v, sl);
            wsmall_store<WG>(W, lane, v, sl);
            tsz = kWSmall;
        }
    }
    if (lane < k) put(E.count + lane, myrec, mylen, mycrc);  // the last, partial run
    E.count += k;
    E.pos = pos;
    E.max_len = wave_max32(vmax);  // (DPP)
    return E;
}

// Is the header (crc, st) at c one scan_record accepts?  Type 0 with a payload that
// fits, size 0 with the stale-word CRC, or a padding record (CRC field 0,
// segment_file.cc:33-49).  *next: the following header.
__device__ __forceinline__ bool header_ok(uint32_t crc, uint32_t st, uint32_t c, uint32_t seg, uint32_t* next,
                                          bool* last) {
    const uint32_t type = st & 0xffu, size = st >> 8;
    *last = false;
    *next = c + (size ? 8 + size : kStaleAdvance);
    if (type == 1) {
        *last = true;
        return crc == 0;
    }
    if (type != 0 || (uint64_t)c + 8 + size > seg) return false;
    return size != 0 || crc == kStaleZero;
}

// The first offset c in [lo, lo + 4 KiB) where a chain of kChainCheck headers
// scan_record accepts starts (ending early at padding or at the segment's short
// rest also counts), or hi.  64 candidates per step, one per lane, from the tile;
// the rare lanes whose first header passes follow the chain in global memory.
// One tile is enough: where headers are further apart, k_wal_resolve walks the
// sub-range itself in a few steps.  A wrong start only costs time: k_wal_resolve
// accepts a walker's list only where the authoritative chain meets it.
template <bool WG = false>
__device__ uint32_t find_start(WaveLds& W, const Seg& S, uint32_t lane, uint32_t lo, uint32_t hi) {
    const uint32_t seg = S.seg;
    uint4 r[kWQV + 1];
    for (uint32_t t0 = lo; t0 < hi && t0 < lo + kWTile; t0 += kWTile) {  // lo is tile-aligned
        wtile_fetch(S, lane, t0, r);
        wtile_store<WG>(W, lane, r);
        const uint32_t tend = t0 + kWTile < hi ? t0 + kWTile : hi;
        for (uint32_t c0 = t0; c0 < tend; c0 += 64) {
            const uint32_t c = c0 + lane;
            bool ok = false;
            if (c < tend && (uint64_t)c + 8 <= seg) {
                uint32_t crc, st, next;
                bool last;
                tile_header(W, c, t0, crc, st);
                // The first hop must stay close: a random "header" whose size happens to land
                // exactly on a real header far ahead would pass the chain check.  Starts with
                // longer records are left to k_wal_resolve (few headers there).
                ok = header_ok(crc, st, c, seg, &next, &last) && (last || next < t0 + 2 * kWTile);
                for (uint32_t k = 1; ok && !last && k < kChainCheck && (uint64_t)next + 8 <= seg; ++k) {
                    if (next < t0 + kWTile) {  // still in the tile (+ its slack): from LDS
                        tile_header(W, next, t0, crc, st);
                    } else {
                        const uint8_t* h = seg_at(S, next, 8);
                        crc = uint32_t(h[0]) | uint32_t(h[1]) << 8 | uint32_t(h[2]) << 16 | uint32_t(h[3]) << 24;
                        st = uint32_t(h[4]) | uint32_t(h[5]) << 8 | uint32_t(h[6]) << 16 | uint32_t(h[7]) << 24;
                    }
                    const uint32_t at = next;
                    ok = header_ok(crc, st, at, seg, &next, &last);
                }
            }
            const uint64_t m = __ballot(ok);
            if (m) return c0 + (uint32_t)(__ffsll((long long)m) - 1);
        }
        wave_sync<WG>();  // everyone is done with the tile before the next store
    }
    return hi;
}

// One wave per (segment, sub-range): segment s0 + blockIdx.x / nsub, sub-range
// j = blockIdx.x % nsub, [j sub_bytes, min(seg, (j + 1) sub_bytes)).  The walker
// of the sub-range holding replay's start walks from the start; later ones find
// a start (find_start); earlier ones have nothing to do.  Each walks until it
// leaves its sub-range and reports to A.sub; with one sub-range per segment the
// walk is the whole segment's and goes straight to A.meta / A.span.
__global__ __launch_bounds__(64) void k_wal_walk_sub(WalArgs A) {
    __shared__ __attribute__((aligned(16))) WaveLds W;
    const uint32_t lane = threadIdx.x;
    const uint64_t P = A.nsub, s = blockIdx.x / P, j = blockIdx.x % P;
    const uint64_t rel = s * A.seg_bytes;
    const Seg S = make_seg(A, s);
    const uint32_t lo = (uint32_t)(j * A.sub_bytes);
    const uint32_t hi = (uint64_t)lo + A.sub_bytes < S.seg ? lo + (uint32_t)A.sub_bytes : S.seg;
    const uint32_t start = s == 0 ? (uint32_t)A.first_pos : 0u;
    uint32_t first;
    if (start >= hi)
        first = hi;  // before replay's start
    else if (start >= lo)
        first = start;
    else
        first = find_start(W, S, lane, lo, hi);
    const uint64_t slot = s * A.cand_cap + j * A.sub_cap;
    // find_start leaves the sub-range's first tile in W
    const WalkEnd E = walk_range(W, S, lane, first, hi, A, slot, A.sub_cap, start < lo && first < hi ? lo : ~0u);
    if (lane != 0) return;
    if (P == 1) {
        const bool spill = !E.kind && E.pos > S.seg;  // a size-0 record's advance left the segment
        const uint32_t kind = spill ? kWalSpill : E.kind, stop = spill ? E.pos : E.stop;
        KB_WRITE(A.meta, s, A.nwork, kKbMeta,
                 (WalSegMeta{E.count, kind, A.base0 + rel + (kind ? stop : S.seg), E.max_len, kCrcUnknown}));
        KB_WRITE(A.span, 2 * s, 2 * A.nwork, kKbSpan, 0u);
        KB_WRITE(A.span, 2 * s + 1, 2 * A.nwork, kKbSpan, 0u);
    } else {
        KB_WRITE(A.sub, blockIdx.x, A.nwork * P, kKbSubMeta,
                 (WalSubMeta{first, E.count, E.kind, E.stop, E.pos, E.max_len, {kCrcUnknown, 0u}}));
    }
}

// The walk with the CRCs in the same kernel (the device-planned replay of small records):
// kFuseWaves walkers per workgroup, each exactly k_wal_walk_sub's walker (its own sub-range,
// its own 4 KiB tile, no workgroup barriers between them), sharing one LDS image of the quad
// blob's tables (16 copies).  After its walk each walker checksums its own list (crc_list):
// the payloads it just read through its tiles (L2 / Infinity Cache hits), no gathered lists,
// no separate gather and CRC launches.  Reports per walker the first
// mismatching list entry (kNoBad: none) or kCrcUnknown.
constexpr int kFuseWaves = kWalFuseWaves;
static_assert(kRep16Words + kFuseWaves * (int)(sizeof(WaveLds) / 4) <= kSmallBase, "the walkers' tiles fit");
__global__ __launch_bounds__(kFuseWaves * 64) void k_wal_walk_crc(WalArgs A) {
    KB_SET_ARENA_SAFE(A.kb_lo, A.kb_hi, A.crc_blob, A.crc_blob + kBlobWords);
    __shared__ __attribute__((aligned(16))) uint32_t lds[kLdsWords];  // 16-copy image | tiles | small tables
    load_stream_tables16<kFuseWaves * 64>(lds, A.crc_blob);
    __syncthreads();
    const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
    const uint64_t P = A.nsub, w = (uint64_t)blockIdx.x * kFuseWaves + wave;
    if (w >= A.nwork * P) return;
    WaveLds& W = reinterpret_cast<WaveLds*>(lds + kRep16Words)[wave];
    const CrcCtx C{lds, lane_const16(), reinterpret_cast<const uint8_t*>(A.crc_blob)};
    const uint64_t s = w / P, j = w % P;
    const uint64_t rel = s * A.seg_bytes;
    const Seg S = make_seg(A, s);
    const uint32_t lo = (uint32_t)(j * A.sub_bytes);
    const uint32_t hi = (uint64_t)lo + A.sub_bytes < S.seg ? lo + (uint32_t)A.sub_bytes : S.seg;
    const uint32_t start = s == 0 ? (uint32_t)A.first_pos : 0u;
    uint32_t first;
    if (start >= hi)
        first = hi;
    else if (start >= lo)
        first = start;
    else
        first = find_start<true>(W, S, lane, lo, hi);
    const uint64_t slot = s * A.cand_cap + j * A.sub_cap;
    const WalkEnd E = walk_range<true>(W, S, lane, first, hi, A, slot, A.sub_cap, start < lo && first < hi ? lo : ~0u);
    const uint32_t fb = crc_list(C, S, A, lane, slot, E.count < A.sub_cap ? E.count : (uint32_t)A.sub_cap, E.max_len);
    if (lane != 0) return;
    if (P == 1) {
        const bool spill = !E.kind && E.pos > S.seg;
        const uint32_t kind = spill ? kWalSpill : E.kind, stop = spill ? E.pos : E.stop;
        KB_WRITE(A.meta, s, A.nwork, kKbMeta, (WalSegMeta{E.count, kind, A.base0 + rel + (kind ? stop : S.seg), E.max_len, fb}));
        KB_WRITE(A.span, 2 * s, 2 * A.nwork, kKbSpan, 0u);
        KB_WRITE(A.span, 2 * s + 1, 2 * A.nwork, kKbSpan, 0u);
    } else {
        KB_WRITE(A.sub, w, A.nwork * P, kKbSubMeta, (WalSubMeta{first, E.count, E.kind, E.stop, E.pos, E.max_len, {fb, 0u}}));
    }
}

// The walkers' lists checksummed after the walk (plan kernel 3: k_wal_walk_sub, then this,
// then k_wal_resolve): the same per-walker report as k_wal_walk_crc's crc_list (the first
// mismatching entry of the walker's own list, kNoBad, or kCrcUnknown over kCrcInlineMax), but
// computed by the small-record kernel staged through LDS (crc_device.h: stg_prefix, lane_record):
// a wave takes a walker, and each step the longest run of its next 64 entries whose bytes fit
// the wave's stage is copied in with whole-wave loads and checksummed one record per lane.
// The walk keeps its occupancy (no CRC state in the walker) and the CRC pass its own.
__global__ __launch_bounds__(kStgWaves * 64) void k_wal_list_crc(WalArgs A) {
    KB_SET_ARENA(A.kb_lo, A.kb_hi);
    __shared__ __attribute__((aligned(16))) uint32_t lds[kStgLdsWords];
    load_stg_tables<kStgWaves * 64>(lds, A.crc_blob);  // the lane blob
    __syncthreads();
    const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
    const uint32_t X = lane_const16();
    uint8_t* stage = reinterpret_cast<uint8_t*>(lds + kStgBuf) + wave * kStgBytes;
    const uint64_t P = A.nsub, nw = A.nwork * P, total = A.nwork * A.cand_cap;
    (void)total;
    for (uint64_t w = (uint64_t)blockIdx.x * kStgWaves + wave; w < nw; w += (uint64_t)gridDim.x * kStgWaves) {
        const uint64_t s = w / P, j = w % P;
        const Seg S = make_seg(A, s);
        uint32_t count, max_len;
        if (P == 1) {
            const WalSegMeta M = KB_READ(A.meta, s, A.nwork, kKbMeta);
            count = M.count;
            max_len = M.max_len;
        } else {
            const WalSubMeta M = KB_READ(A.sub, w, nw, kKbSubMeta);
            count = M.count;
            max_len = M.max_len;
        }
        if (count > A.sub_cap) count = (uint32_t)A.sub_cap;
        const uint64_t slot0 = s * A.cand_cap + j * A.sub_cap;
        uint32_t fb = kNoBad;
        if (max_len > kCrcInlineMax) {
            fb = kCrcUnknown;
        } else {
            for (uint32_t i0 = 0; i0 < count;) {
                const uint32_t i = i0 + lane;
                const bool v = i < count;
                uint32_t rec = 0, n = 0, st = 0;
                if (v) {
                    rec = KB_READ(A.cand_rec, slot0 + i, total, kKbCand);
                    n = KB_READ(A.cand_len, slot0 + i, total, kKbCand);
                    st = KB_READ(A.cand_crc, slot0 + i, total, kKbCand);
                }
                const uintptr_t p = reinterpret_cast<uintptr_t>(S.img) + rec + 8;
                const StgSpan SP = stg_prefix(p, n, v && n, lane);
                const bool staged = SP.hi != 0;
                if (staged) {
                    stg_copy(SP.lo, SP.hi, lane, stage);
                    wave_lds_sync();
                }
                uint32_t res = 0;
                const bool mine = v && n && lane < SP.cnt;  // size 0: checked by the walk
                if (mine) {
                    if (staged)
                        res = lane_record(lds, X, kStgZ4, kStgT8, p, n, 0u, [&](uintptr_t a) {
                            return *reinterpret_cast<const u32x4*>(stage + (uint32_t)(a - SP.lo));
                        });
                    else
                        res = lane_record(lds, X, kStgZ4, kStgT8, p, n, 0u,
                                          [&](uintptr_t a) { return ld16(reinterpret_cast<const uint8_t*>(a)); });
                }
                const uint64_t bm = __ballot(mine && res != st);
                if (bm) {
                    fb = i0 + (uint32_t)__builtin_ctzll(bm);
                    break;
                }
                i0 += SP.cnt;
                wave_lds_sync();  // this step's reads before the next step's stores
            }
        }
        if (lane == 0) {
#ifdef KARMA_BOUNDS
            if (!KB_IDX(P == 1 ? s : w, P == 1 ? A.nwork : nw, P == 1 ? kKbMeta : kKbSubMeta)) continue;
#endif
            if (P == 1)
                A.meta[s].first_bad = fb;
            else
                A.sub[w].pad[0] = fb;
        }
    }
}

// One wave per segment: follow the authoritative chain through the sub-ranges.
// Entering sub-range j at pos, the chain continues exactly as walker j's list
// from the entry equal to pos on (the walk is a function of the position), so
// that run is accepted; when pos is not in the list (walker j started on a wrong
// header, or none), this wave walks the sub-range itself from pos, into the same
// slots.  Writes the segment's count / stop and the accepted run per sub-range.
// The resolver's body for segment s, run by one wave (lane = its lane): WG as walk_range's (a
// wave alone in its workgroup: false; one wave of a larger workgroup: true).  lspan: the
// segment's runs also into LDS (the fused resolve + gather), else nullptr.  Returns the meta.
template <bool WG>
__device__ __forceinline__ WalSegMeta resolve_segment(const WalArgs& A, WaveLds& W, uint64_t s, uint32_t lane,
                                                      uint2* lspan) {
    const uint64_t P = A.nsub;
    const uint64_t rel = s * A.seg_bytes;
    const Seg S = make_seg(A, s);
    const uint32_t seg = S.seg;
    const uint64_t c0 = s * A.cand_cap, total = A.nwork * A.cand_cap;  // the segment's first list slot
    (void)total;
    uint32_t pos = s == 0 ? (uint32_t)A.first_pos : 0u;
    uint32_t count = 0, kind = 0, stop = seg, mx = 0;
    // the walkers' inline CRCs (k_wal_walk_crc; WalSubMeta::pad[0]): the segment's first
    // mismatching candidate (ordinal among its accepted ones), or kCrcUnknown when a run the
    // chain accepts was not checksummed whole (a walker with a long payload, a run taken from
    // past a mismatch in the walker's own rejected prefix, or a sub-range walked here)
    uint32_t sfb = kNoBad;
    bool sunk = false;
    // Fast pass, 64 sub-ranges at a time (lane l: sub-range j0 + l): when every walker started
    // exactly where the one before it left off (the usual case: find_start lands on the real
    // chain), each run is accepted whole, and the spans are a prefix sum.  Lane l takes the
    // previous lane's exit as its entry and checks the serial loop's conditions for it; from
    // the first lane that fails, the serial loop below takes over.
    uint64_t j = 0;
    while (j < P) {
        const uint64_t jj = j + lane;
        const bool in = jj < P;
        WalSubMeta m{};
        if (in) m = KB_READ(A.sub, s * P + jj, A.nwork * P, kKbSubMeta);
        const uint32_t lo = (uint32_t)(jj * A.sub_bytes);
        const uint32_t hi = (uint64_t)lo + A.sub_bytes < seg ? lo + (uint32_t)A.sub_bytes : seg;
        uint32_t pj = __shfl_up(m.exit, 1);
        if (lane == 0) pj = pos;
        const uint64_t km = __ballot(in && m.kind != 0);
        const bool kbefore = kind != 0 || (km & ((1ull << lane) - 1ull)) != 0;  // replay stopped before
        const bool acc = in && !kbefore && pj < hi && (uint64_t)pj + 8 <= seg && m.first == pj;
        const uint64_t bad = __ballot(!(!in || kbefore || acc));
        const uint32_t f = bad ? (uint32_t)__builtin_ctzll(bad) : 64u;  // lanes < f follow the serial loop
        const bool take = lane < f && acc;
        const uint32_t n = take ? m.count : 0u;
        const uint32_t pre = wave_incl_scan32(n);  // inclusive prefix of n (DPP)
        if (in && lane < f) {
            KB_WRITE(A.span, 2 * (s * P + jj), 2 * A.nwork * P, kKbSpan, (uint32_t)(jj * A.sub_cap));
            KB_WRITE(A.span, 2 * (s * P + jj) + 1, 2 * A.nwork * P, kKbSpan, count + pre - n);
            if (lspan) lspan[jj] = uint2{(uint32_t)(jj * A.sub_cap), count + pre - n};
        }
        {  // (count: the candidates before this batch of runs)
            const uint32_t f0 = m.pad[0];
            const bool unk = take && n != 0 && f0 == kCrcUnknown;
            const uint32_t ord = wave_min32(take && f0 < kCrcUnknown ? count + pre - n + f0 : kNoBad);
            if (__ballot(unk)) sunk = true;
            sfb = ord < sfb ? ord : sfb;
        }
        count += (uint32_t)__builtin_amdgcn_readlane((int)pre, 63);
        const uint32_t vmx = wave_max32(take ? m.max_len : 0u);
        mx = vmx > mx ? vmx : mx;
        const uint64_t kt = __ballot(take && m.kind != 0);
        if (kt) {
            const int l = __builtin_ctzll(kt);
            kind = __builtin_amdgcn_readlane(m.kind, l);
            stop = __builtin_amdgcn_readlane(m.stop, l);
        }
        const uint64_t tm = __ballot(take);
        if (tm) pos = __builtin_amdgcn_readlane(m.exit, 63 - __builtin_clzll(tm));
        pos = __builtin_amdgcn_readfirstlane(pos);
        count = __builtin_amdgcn_readfirstlane(count);
        mx = __builtin_amdgcn_readfirstlane(mx);
        if (f < 64) {
            j += f;
            break;
        }
        j += 64;
    }
    WalSubMeta mine{};  // lane l holds walker (j & ~63) + l's report: 64 loads at once, not one per step
    for (const uint64_t j1 = j; j < P; ++j) {
        if ((j % 64 == 0 || j == j1) && (j & ~63ull) + lane < P)
            mine = KB_READ(A.sub, s * P + (j & ~63ull) + lane, A.nwork * P, kKbSubMeta);
        const uint32_t lo = (uint32_t)(j * A.sub_bytes);
        const uint32_t hi = (uint64_t)lo + A.sub_bytes < seg ? lo + (uint32_t)A.sub_bytes : seg;
        uint32_t st = (uint32_t)(j * A.sub_cap), n = 0;
        if (!kind && pos < hi && (uint64_t)pos + 8 <= seg) {
            const int src = (int)(j % 64);
            WalSubMeta m;
            m.first = __builtin_amdgcn_readlane(mine.first, src);  // uniform lane: v_readlane, no LDS
            m.count = __builtin_amdgcn_readlane(mine.count, src);
            m.kind = __builtin_amdgcn_readlane(mine.kind, src);
            m.stop = __builtin_amdgcn_readlane(mine.stop, src);
            m.exit = __builtin_amdgcn_readlane(mine.exit, src);
            m.max_len = __builtin_amdgcn_readlane(mine.max_len, src);
            m.pad[0] = __builtin_amdgcn_readlane(mine.pad[0], src);
            int64_t idx = -1;
            if (m.first == pos) {
                idx = 0;
            } else if (m.first < pos && m.count > 1) {  // pos among the list's later entries?
                uint32_t a = 1, b = m.count;             // search [a, b)
                auto rec_at = [&](uint32_t i) {  // entry i of walker j's list (bounds build: in its slots)
#ifdef KARMA_BOUNDS
                    kb_ok(i < A.sub_cap, kKbRunSlot, i, A.sub_cap);
#endif
                    return KB_READ(A.cand_rec, c0 + st + i, total, kKbCand);
                };
                while (a < b) {
                    const uint32_t mid = (a + b) / 2;
                    if (rec_at(mid) < pos) a = mid + 1;
                    else b = mid;
                }
                if (a < m.count && rec_at(a) == pos) idx = a;
            }
            if (idx >= 0) {
                st += (uint32_t)idx;
                n = m.count - (uint32_t)idx;
                if (n && (m.pad[0] == kCrcUnknown || (m.pad[0] != kNoBad && m.pad[0] < (uint32_t)idx))) sunk = true;
                else if (m.pad[0] < kCrcUnknown && count + (m.pad[0] - (uint32_t)idx) < sfb)
                    sfb = count + (m.pad[0] - (uint32_t)idx);
                pos = m.exit;
                mx = m.max_len > mx ? m.max_len : mx;  // of the walker's whole list: an upper bound
                if (m.kind) {
                    kind = m.kind;
                    stop = m.stop;
                }
            } else {
                const WalkEnd E = walk_range<WG>(W, S, lane, pos, hi, A, c0 + st, A.sub_cap);
                n = E.count;
                if (n) sunk = true;  // no inline CRCs for this run
                pos = E.pos;
                mx = E.max_len > mx ? E.max_len : mx;
                if (E.kind) {
                    kind = E.kind;
                    stop = E.stop;
                }
            }
        }
        if (lane == 0) {
            KB_WRITE(A.span, 2 * (s * P + j), 2 * A.nwork * P, kKbSpan, st);
            KB_WRITE(A.span, 2 * (s * P + j) + 1, 2 * A.nwork * P, kKbSpan, count);  // candidates before the run
            if (lspan) lspan[j] = uint2{st, count};
        }
        count += n;
    }
    if (!kind && pos > seg) {  // a size-0 record's advance left the segment
        kind = kWalSpill;
        stop = pos;
    }
    const WalSegMeta out{count, kind, A.base0 + rel + (kind ? stop : seg), mx, sunk ? kCrcUnknown : sfb};
    if (lane == 0) KB_WRITE(A.meta, s, A.nwork, kKbMeta, out);
    return out;
}

__global__ __launch_bounds__(64) void k_wal_resolve(WalArgs A) {
    __shared__ __attribute__((aligned(16))) WaveLds W;
    (void)resolve_segment<false>(A, W, blockIdx.x, threadIdx.x, nullptr);
}

// The replay plan on the device (one block): replay enters segment s + 1 only when segment s
// ended cleanly, so it reads segments [0, w1) with w1 = the first segment whose walk did not end
// (+ 1); their candidates are gathered at cand_base[w] = the exclusive prefix of the counts.
// Writes A.sum (first_bad reset) so no host round trip is needed before the gather.
__global__ __launch_bounds__(1024) void k_wal_plan(WalArgs A) {
    __shared__ uint32_t s_w1, s_max;
    __shared__ unsigned long long s_wsum[16];
    const uint32_t tid = threadIdx.x, lane = tid & 63u, wave = tid >> 6;
    const uint64_t nw = A.nwork;
    if (tid == 0) {
        s_w1 = (uint32_t)nw;
        s_max = 0;
    }
    __syncthreads();
    for (uint64_t w = tid; w < nw; w += blockDim.x)
        if (A.meta[w].kind != KARMA_WAL_END) atomicMin(&s_w1, (uint32_t)(w + 1));
    __syncthreads();
    const uint32_t w1 = s_w1;
    uint64_t carry = 0;
    uint32_t mx = 0;
    for (uint64_t b = 0; b < w1; b += blockDim.x) {  // exclusive prefix of the counts, 1024 at a time
        const uint64_t w = b + tid;
        const uint64_t c = w < w1 ? A.meta[w].count : 0;
        if (w < w1) mx = A.meta[w].max_len > mx ? A.meta[w].max_len : mx;
        uint64_t x = c;  // inclusive wave scan
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const uint64_t t = __shfl_up(x, d);
            if ((int)lane >= d) x += t;
        }
        if (lane == 63) s_wsum[wave] = x;
        __syncthreads();
        uint64_t pre = 0, tot = 0;
        for (uint32_t v = 0; v < blockDim.x / 64; ++v) {
            if (v < wave) pre += s_wsum[v];
            tot += s_wsum[v];
        }
        if (w < w1) A.cand_base[w] = carry + pre + x - c;
        carry += tot;
        __syncthreads();  // s_wsum is rewritten by the next chunk
    }
    atomicMax(&s_max, mx);
    // the inline CRCs' first mismatch in WAL order (k_wal_walk_crc): min over the segments replay
    // enters of list offset + the segment's ordinal, packed with the segment; or unknown
    __shared__ unsigned long long s_bad;
    __shared__ uint32_t s_unk;
    if (tid == 0) {
        s_bad = ~0ull;
        s_unk = 0;
    }
    __syncthreads();
    for (uint64_t w = tid; w < w1; w += blockDim.x) {
        const uint32_t fb = A.meta[w].first_bad;
        if (fb == kCrcUnknown) s_unk = 1;
        else if (fb != kNoBad) atomicMin(&s_bad, ((A.cand_base[w] + fb) << 24) | w);  // < 2^40 candidates, < 2^24 segments
    }
    __syncthreads();
    if (tid == 0) {
        WalSummary S{carry, A.wal_end, w1, KARMA_WAL_END, s_max, s_unk, ~0ull, 0ull};
        if (w1 > 0 && A.meta[w1 - 1].kind != KARMA_WAL_END) {
            S.status = A.meta[w1 - 1].kind;
            S.end = A.meta[w1 - 1].stop;
        }
        if (!s_unk && s_bad != ~0ull) {  // its header offset: the segment's run holding the ordinal
            const uint64_t g = s_bad >> 24, w = s_bad & 0xffffffu, o = g - A.cand_base[w];
            const uint32_t* sp = A.span + 2 * w * A.nsub;
            uint32_t a = 0, b = (uint32_t)A.nsub;  // the last run whose prefix is <= o
            while (b - a > 1) {
                const uint32_t mid = (a + b) / 2;
                if (sp[2 * mid + 1] <= o) a = mid;
                else b = mid;
            }
            const uint64_t slot = sp[2 * a] + (o - sp[2 * a + 1]);
            S.first_bad = g;
            S.bad_off = w * A.seg_bytes + KB_READ(A.cand_rec, w * A.cand_cap + slot, A.nwork * A.cand_cap, kKbCand);
        }
        *A.sum = S;
    }
}

// Candidates of segment s0 + blockIdx.x (one block per segment) into the
// contiguous lists at slot A.cand_base[blockIdx.x]: header offset (relative to
// A.wal), length and the CRC field stored in the header (the walk kept it).  The segment's list is
// its accepted runs in order (A.span: first slot, candidates before the run);
// candidate i finds its run by a binary search over the runs staged in LDS.
// FUSED_PLAN (at most 1024 segments, the device-planned path): there is no k_wal_plan
// launch; every block reduces the metas itself (w1, its own list offset) and block 0 writes
// the summary.
template <bool FUSED_PLAN>
__global__ __launch_bounds__(1024) void k_wal_gather(WalArgs A) {
    __shared__ uint2 spans[kMaxSub];
    __shared__ uint32_t s_count;
    // the segment's spans first: their load is in flight with the metas' (one latency, not two)
    const uint32_t P = (uint32_t)A.nsub;
    const uint2* sp = reinterpret_cast<const uint2*>(A.span) + blockIdx.x * A.nsub;
    for (uint32_t j = threadIdx.x; j < P; j += blockDim.x)
        spans[j] = KB_READ(sp, j, (A.nwork - blockIdx.x) * A.nsub, kKbSpan);
    uint64_t g0;
    if constexpr (FUSED_PLAN) {
        __shared__ uint32_t s_w1, s_max;
        __shared__ unsigned long long s_pre[16], s_all[16];
        const uint32_t tid = threadIdx.x, lane = tid & 63u, wave = tid >> 6;
        const uint32_t nw = (uint32_t)A.nwork;  // <= blockDim.x
        if (tid == 0) {
            s_w1 = nw;
            s_max = 0;
        }
        __syncthreads();
        WalSegMeta m{0u, KARMA_WAL_END, 0u, 0u, 0u};
        if (tid < nw) m = A.meta[tid];
        if (tid < nw && m.kind != KARMA_WAL_END) atomicMin(&s_w1, tid + 1);
        if (tid == blockIdx.x) s_count = m.count;
        __syncthreads();
        const uint32_t w1 = s_w1;
        if (blockIdx.x >= w1 && blockIdx.x != 0) return;  // replay does not enter this segment
        // (32-bit sums through DPP: the device-planned path has images <= kDevicePlanMax, and a
        // candidate takes at least 8 image bytes, so the counts fit in 32 bits)
        static_assert(kDevicePlanMax / 8 < (1ull << 32), "fused-plan candidate sums are 32-bit");
        const unsigned long long pre = (uint32_t)__builtin_amdgcn_readlane((int)wave_incl_scan32(tid < blockIdx.x ? m.count : 0u), 63);
        const unsigned long long all = (uint32_t)__builtin_amdgcn_readlane((int)wave_incl_scan32(tid < w1 ? m.count : 0u), 63);
        if (lane == 0) {
            s_pre[wave] = pre;
            s_all[wave] = all;
        }
        if (tid < w1) atomicMax(&s_max, m.max_len);
        __syncthreads();
        g0 = 0;
        uint64_t n_all = 0;
        for (uint32_t v = 0; v < blockDim.x / 64; ++v) {
            g0 += s_pre[v];
            n_all += s_all[v];
        }
        if (blockIdx.x == 0 && blockIdx.y == 0 && tid == 0) {
            WalSummary S{n_all, A.wal_end, w1, KARMA_WAL_END, s_max, 1u, ~0ull, 0ull};
            if (A.meta[w1 - 1].kind != KARMA_WAL_END) {
                S.status = A.meta[w1 - 1].kind;
                S.end = A.meta[w1 - 1].stop;
            }
            *A.sum = S;
        }
        if (blockIdx.x >= w1) return;
    } else {
        if (blockIdx.x >= A.sum->w1) return;  // replay does not enter this segment
        g0 = A.cand_base[blockIdx.x];
        if (threadIdx.x == 0) s_count = A.meta[blockIdx.x].count;
    }
    const uint64_t rel = (uint64_t)blockIdx.x * A.seg_bytes;
    const uint32_t* crec = A.cand_rec + blockIdx.x * A.cand_cap;
    const uint32_t* clen = A.cand_len + blockIdx.x * A.cand_cap;
    const uint32_t* ccrc = A.cand_crc + blockIdx.x * A.cand_cap;
    __syncthreads();
    // gridDim.y blocks per segment (few segments would leave CUs idle), each a contiguous part
    const uint32_t per = (s_count + gridDim.y - 1) / gridDim.y, i_lo = blockIdx.y * per;
    const uint32_t count = min(s_count, i_lo + per);
    // kGatherU candidates per thread per trip, every load issued before the first store: one
    // memory latency per trip instead of one per candidate (a segment of 1 MiB holds ~5600
    // candidates of 180 B: one trip of 1024 threads)
    constexpr int kGatherU = 8;
    for (uint32_t i0 = i_lo + threadIdx.x; i0 < count; i0 += kGatherU * blockDim.x) {
        uint32_t vr[kGatherU], vn[kGatherU], vc[kGatherU];
#pragma unroll
        for (int u = 0; u < kGatherU; ++u) {
            const uint32_t i = i0 + u * blockDim.x;
            if (i >= count) break;
            uint32_t a = 0, b = P;  // the last run whose prefix is <= i: [a, b)
            while (b - a > 1) {
                const uint32_t mid = (a + b) / 2;
                if (spans[mid].y <= i) a = mid;
                else b = mid;
            }
            const uint32_t slot = spans[a].x + (i - spans[a].y);
#ifdef KARMA_BOUNDS
            kb_ok(slot >= a * A.sub_cap && slot < (a + 1) * A.sub_cap, kKbRunSlot, slot, A.sub_cap);
#endif
            vr[u] = KB_READ(crec, slot, A.cand_cap, kKbCand);
            vn[u] = KB_READ(clen, slot, A.cand_cap, kKbCand);
            vc[u] = KB_READ(ccrc, slot, A.cand_cap, kKbCand);
        }
#pragma unroll
        for (int u = 0; u < kGatherU; ++u) {
            const uint32_t i = i0 + u * blockDim.x;
            if (i >= count) break;
            KB_WRITE(A.off, g0 + i, A.n_all, kKbList, rel + vr[u]);
            KB_WRITE(A.len, g0 + i, A.n_all, kKbList, vn[u]);
            KB_WRITE(A.stored, g0 + i, A.n_all, kKbList, vc[u]);
        }
    }
}

// Resolve and gather in one launch (round 6; the device-planned replay with sub-range walkers and
// at most 1024 segments).  Block s: wave 0 resolves segment s (resolve_segment, its runs also into
// LDS) and publishes two tagged words -- the segment's candidate count with a flag for "did not end
// cleanly", and its largest payload; meanwhile wave 1 sums the words of segments [0, s) (each lane a
// stride of them, loads issued together, a word not yet tagged with this call's tag waited for):
// the block's list offset, whether replay stops before segment s (replay enters s only if every
// earlier segment ended cleanly), and the largest payload so far.  Every block it waits on has a lower index, so it
// was dispatched earlier and publishes before waiting on anything: the waits end.  The segment
// replay stops in (or the last one) writes the summary, as k_wal_gather<true>'s block 0 does; the
// other blocks gather their candidates exactly as k_wal_gather does.  Replaces k_wal_resolve's
// launch and k_wal_gather<true>'s re-reduction of every segment's meta in every block.
constexpr uint64_t kRgTagShift = 48, kRgStop = 1ull << 47, kRgValue = (1ull << 47) - 1;
__global__ __launch_bounds__(1024) void k_wal_resolve_gather(WalArgs A) {
    __shared__ __attribute__((aligned(16))) WaveLds W;
    __shared__ uint2 spans[kMaxSub];
    __shared__ unsigned long long s_pre;
    __shared__ uint32_t s_count, s_stop_before, s_mx, s_mx_pred, s_kind;
    __shared__ uint64_t s_stop_off;
    const uint32_t tid = threadIdx.x, lane = tid & 63u, wave = tid >> 6;
    const uint64_t s = blockIdx.x;
    const unsigned long long tag = (unsigned long long)A.rg_tag << kRgTagShift;
    if (wave == 0) {  // the segment's resolve, then its words
        const WalSegMeta m = resolve_segment<true>(A, W, s, lane, spans);
        if (lane == 0) {
            __hip_atomic_store(A.rg_words + 2 * s, tag | (m.kind != KARMA_WAL_END ? kRgStop : 0ull) | m.count,
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(A.rg_words + 2 * s + 1, tag | m.max_len, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            s_count = m.count;
            s_kind = m.kind;
            s_stop_off = m.stop;
            s_mx = m.max_len;
        }
    } else if (wave == 1) {  // meanwhile, the earlier segments' words (they publish before waiting)
        uint32_t cnt = 0, stop = 0, mx = 0;  // (counts: < 2^25 candidates in an image of <= 256 MiB)
        constexpr int kQ = 16;               // 16 x 64 = 1024 segments, every load out at once
        unsigned long long wc[kQ], wm[kQ];
#pragma unroll
        for (int q = 0; q < kQ; ++q) {
            const uint64_t i = lane + 64ull * q;
            wc[q] = wm[q] = tag;  // (segments at or past s: nothing)
            if (i < s) {
                wc[q] = __hip_atomic_load(A.rg_words + 2 * i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                wm[q] = __hip_atomic_load(A.rg_words + 2 * i + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
        }
#pragma unroll
        for (int q = 0; q < kQ; ++q) {
            const uint64_t i = lane + 64ull * q;
            if (i < s) {
                while ((wc[q] >> kRgTagShift) != A.rg_tag) {  // not published yet
                    __builtin_amdgcn_s_sleep(1);
                    wc[q] = __hip_atomic_load(A.rg_words + 2 * i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                }
                while ((wm[q] >> kRgTagShift) != A.rg_tag) {
                    __builtin_amdgcn_s_sleep(1);
                    wm[q] = __hip_atomic_load(A.rg_words + 2 * i + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                }
                cnt += (uint32_t)(wc[q] & kRgValue);
                stop |= (wc[q] & kRgStop) ? 1u : 0u;
                mx = (uint32_t)wm[q] > mx ? (uint32_t)wm[q] : mx;
            }
        }
        cnt = (uint32_t)__builtin_amdgcn_readlane((int)wave_incl_scan32(cnt), 63);
        stop = wave_or32(stop);
        mx = wave_max32(mx);
        if (lane == 0) {
            s_pre = cnt;
            s_stop_before = stop;
            s_mx_pred = mx;
        }
    }
    __syncthreads();
    // the segment replay stops in, or the last one: the summary (k_wal_gather<true>'s)
    if (tid == 0 && !s_stop_before && (s_kind != KARMA_WAL_END || s + 1 == A.nwork)) {
        const uint32_t mx = s_mx > s_mx_pred ? s_mx : s_mx_pred;
        WalSummary S{(uint64_t)s_pre + s_count, A.wal_end, (uint32_t)(s + 1), KARMA_WAL_END, mx, 1u, ~0ull, 0ull};
        if (s_kind != KARMA_WAL_END) {
            S.status = s_kind;
            S.end = s_stop_off;
        }
        *A.sum = S;
    }
    if (s_stop_before) return;  // replay does not enter this segment
    const uint64_t g0 = s_pre;
    const uint32_t P = (uint32_t)A.nsub, count = s_count;
    const uint64_t rel = s * A.seg_bytes;
    const uint32_t* crec = A.cand_rec + s * A.cand_cap;
    const uint32_t* clen = A.cand_len + s * A.cand_cap;
    const uint32_t* ccrc = A.cand_crc + s * A.cand_cap;
    constexpr int kGatherU = 8;  // (as k_wal_gather)
    for (uint32_t i0 = tid; i0 < count; i0 += kGatherU * blockDim.x) {
        uint32_t vr[kGatherU], vn[kGatherU], vc[kGatherU];
#pragma unroll
        for (int u = 0; u < kGatherU; ++u) {
            const uint32_t i = i0 + u * blockDim.x;
            if (i >= count) break;
            uint32_t a = 0, b = P;  // the last run whose prefix is <= i: [a, b)
            while (b - a > 1) {
                const uint32_t mid = (a + b) / 2;
                if (spans[mid].y <= i) a = mid;
                else b = mid;
            }
            const uint32_t slot = spans[a].x + (i - spans[a].y);
#ifdef KARMA_BOUNDS
            kb_ok(slot >= a * A.sub_cap && slot < (a + 1) * A.sub_cap, kKbRunSlot, slot, A.sub_cap);
#endif
            vr[u] = KB_READ(crec, slot, A.cand_cap, kKbCand);
            vn[u] = KB_READ(clen, slot, A.cand_cap, kKbCand);
            vc[u] = KB_READ(ccrc, slot, A.cand_cap, kKbCand);
        }
#pragma unroll
        for (int u = 0; u < kGatherU; ++u) {
            const uint32_t i = i0 + u * blockDim.x;
            if (i >= count) break;
            KB_WRITE(A.off, g0 + i, A.n_all, kKbList, rel + vr[u]);
            KB_WRITE(A.len, g0 + i, A.n_all, kKbList, vn[u]);
            KB_WRITE(A.stored, g0 + i, A.n_all, kKbList, vc[u]);
        }
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

hipError_t launch_wal_walk(const WalArgs& a, uint64_t nseg, const WalWalkPlan& plan, hipStream_t s, bool resolve) {
    if (!nseg) return hipSuccess;
#ifdef KARMA_AB
    if (plan.kernel == 1) {
        hipLaunchKernelGGL(k_wal_walk, dim3((unsigned)nseg), dim3(kWalkThreads), 0, s, a);
        return hipGetLastError();
    }
#endif
    if (plan.kernel == 2) {
        if (!a.crc_blob) return hipErrorInvalidValue;
        const uint64_t walkers = nseg * plan.nsub;
        hipLaunchKernelGGL(k_wal_walk_crc, dim3((unsigned)((walkers + kFuseWaves - 1) / kFuseWaves)),
                           dim3(kFuseWaves * 64), 0, s, a);
    } else {
        hipLaunchKernelGGL(k_wal_walk_sub, dim3((unsigned)(nseg * plan.nsub)), dim3(64), 0, s, a);
    }
    if (plan.kernel == 3) {  // the walkers' lists checksummed after the walk (the lane blob)
        if (!a.crc_blob) return hipErrorInvalidValue;
        const uint64_t walkers = nseg * plan.nsub;
        uint64_t blocks = (walkers + kStgWaves - 1) / kStgWaves;
        if (blocks > (uint64_t)plan.cu) blocks = (uint64_t)plan.cu;
        hipLaunchKernelGGL(k_wal_list_crc, dim3((unsigned)blocks), dim3(kStgWaves * 64), 0, s, a);
    }
    if (plan.nsub > 1 && resolve) hipLaunchKernelGGL(k_wal_resolve, dim3((unsigned)nseg), dim3(64), 0, s, a);
    return hipGetLastError();
}

hipError_t launch_wal_plan(const WalArgs& a, uint64_t nseg, hipStream_t s) {
    (void)nseg;
    hipLaunchKernelGGL(k_wal_plan, dim3(1), dim3(1024), 0, s, a);
    return hipGetLastError();
}

hipError_t launch_wal_gather(const WalArgs& a, uint64_t nseg, bool fused_plan, int cu, hipStream_t s) {
    if (!nseg) return hipSuccess;
    // One block per segment.  (Splitting a segment's candidates over ~2 blocks per CU in all --
    // 3 blocks per segment for the bench image's 188 segments -- made the gather 16.3 us instead
    // of 12 and the rotated replay call 4 us slower, profiles/r04_replay_ab.txt: every block reads
    // all the metas and the segment's spans.  The tools build keeps KARMA_GATHER_PARTS for A/B.)
    (void)cu;
    uint64_t parts = 1;
    if (const long p = KARMA_AB_KNOB("KARMA_GATHER_PARTS", 0); p > 0) parts = (uint64_t)std::min(p, 64l);
    const dim3 grid((unsigned)nseg, (unsigned)parts);
    if (fused_plan) {
        if (nseg > 1024) return hipErrorInvalidValue;
        hipLaunchKernelGGL(k_wal_gather<true>, grid, dim3(1024), 0, s, a);
    } else {
        hipLaunchKernelGGL(k_wal_gather<false>, grid, dim3(1024), 0, s, a);
    }
    return hipGetLastError();
}

namespace {
// One wave: word i of the summary to the host copy (system scope: written through to host memory).
__global__ __launch_bounds__(64) void k_wal_publish(const WalSummary* src, WalSummary* dst) {
    constexpr uint32_t kWords = sizeof(WalSummary) / 4;
    static_assert(sizeof(WalSummary) % 4 == 0 && kWords <= 64, "one word per lane");
    const uint32_t i = threadIdx.x;
    if (i < kWords) {
        const uint32_t w = reinterpret_cast<const uint32_t*>(src)[i];
        __hip_atomic_store(reinterpret_cast<uint32_t*>(dst) + i, w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}
}  // namespace

hipError_t launch_wal_publish(const WalSummary* src, WalSummary* dst_host, hipStream_t s) {
    hipLaunchKernelGGL(k_wal_publish, dim3(1), dim3(64), 0, s, src, dst_host);
    return hipGetLastError();
}

hipError_t launch_wal_resolve_gather(const WalArgs& a, uint64_t nseg, hipStream_t s) {
    if (!nseg) return hipSuccess;
    if (nseg > 1024 || a.nsub > kMaxSub || !a.rg_words || !a.rg_tag || a.rg_tag >= (1u << 16)) return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_wal_resolve_gather, dim3((unsigned)nseg), dim3(1024), 0, s, a);
    return hipGetLastError();
}

hipError_t launch_wal_compare(const WalArgs& a, uint64_t n, int cu, hipStream_t s) {
    if (!n) return hipSuccess;
    uint64_t blocks = (n + 255) / 256;
    if (blocks > (uint64_t)cu * 8) blocks = (uint64_t)cu * 8;
    hipLaunchKernelGGL(k_wal_compare, dim3((unsigned)blocks), dim3(256), 0, s, a, n);
    return hipGetLastError();
}

KB_DEFINE_COLLECT(wal)

}  // namespace engine
}  // namespace karma
