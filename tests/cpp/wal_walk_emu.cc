// tests/cpp/wal_walk_emu.cc -- CPU emulation of the device WAL replay, with bounds checks
// (test infrastructure; built under ASan/UBSan by `make -C karma_amd/csrc san`, driven by
// tests/test_sanitizers.py).
//
// Restates, wave by wave and lane by lane, the control flow and the address arithmetic of
//   karma_amd/csrc/wal_device.hip  wal_walk_plan, k_wal_walk_sub (find_start, walk_range with
//                                  its speculative header rounds, wtile_fetch / wsmall_fetch,
//                                  tile_header), k_wal_resolve,
//                                  k_wal_gather, k_wal_compare
//   karma_amd/csrc/wal.cc          replay_core's planning around them
//   k_wal_walk_crc / k_wal_resolve / k_wal_plan's inline CRCs: each walker's first mismatching
//                                  list entry, the resolver's per-segment ordinal, the plan's
//                                  minimum -- which must equal the gathered batch's first
//                                  mismatch whenever every accepted run was checksummed
//   karma_amd/csrc/crc_ragged.hip  the 16-byte blocks k_ragged_direct reads per record
// and checks, on every access:
//   * each global read of a walker lies inside its own segment ([0, seg) of segment s);
//   * each LDS tile read lies inside the part of the tile the last fetch filled;
//   * each list slot written or read lies inside its sub-range's capacity, and no list
//     write is ever dropped by the kernels' capacity guards;
//   * each CRC-batch read lies inside the 16-byte blocks of the image.
// A violation aborts (non-zero exit).  The result (records accepted, stop, status) is
// printed so the test can compare it with tests/wal_model.py (wal::scan_record,
// karma-store/wal.cc:34-87).
//
// usage: wal_walk_emu <image file> <seg_bytes> <start> <sub_bytes (0 = planned)> <cu>
#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

namespace {

constexpr uint32_t kWTile = 4096, kWQV = kWTile / 1024, kChainCheck = 4, kMaxSub = 4096, kWSmall = 1024;
constexpr uint32_t kStaleZero = 0x48674BC7u;  // crc32c::Value("\0\0\0\0")
constexpr uint32_t kStaleAdvance = 12;         // an accepted size-0 record: 8 + 4 stale bytes (sivir.cc:38)
enum { END = 0, CORRUPT = 1, BAD_TYPE = 2, SPILL = 16 };

uint64_t g_reads = 0, g_slots = 0, g_inline_known = 0, g_inline_unknown = 0;

[[noreturn]] void die(const char* what, uint64_t a, uint64_t b) {
    std::fprintf(stderr, "VIOLATION: %s (%llu, %llu)\n", what, (unsigned long long)a, (unsigned long long)b);
    std::abort();
}

uint32_t crc32c(const uint8_t* p, size_t n) {  // bitwise CRC-32C (karma-util/crc32c.cc semantics)
    uint32_t l = 0xFFFFFFFFu;
    for (size_t i = 0; i < n; ++i) {
        l ^= p[i];
        for (int k = 0; k < 8; ++k) l = (l >> 1) ^ (0x82F63B78u & (0u - (l & 1u)));
    }
    return l ^ 0xFFFFFFFFu;
}

struct Seg {  // one segment as a walker sees it: its bytes are img[0, seg)
    const uint8_t* img;
    uint32_t seg;
    bool vec;
};

uint8_t rd(const Seg& S, uint64_t off) {  // a global byte read of a walker
    if (off >= S.seg) die("walker read outside its segment", off, S.seg);
    ++g_reads;
    return S.img[off];
}

struct Tile {  // WaveLds: the tile bytes and how many of them the last fetch filled
    uint8_t b[kWTile + 16];
    uint32_t valid = 0;
};

// wtile_fetch + wtile_store: vectors lane + 64 q (q < kWQV) and the slack vector
void tile_fetch(Tile& W, const Seg& S, uint32_t t) {
    std::memset(W.b, 0xAB, sizeof W.b);
    if (S.vec && (uint64_t)t + kWTile + 16 <= S.seg) {
        for (uint32_t q = 0; q < kWQV; ++q)
            for (uint32_t lane = 0; lane < 64; ++lane)
                for (uint32_t i = 0; i < 16; ++i) W.b[(lane + 64 * q) * 16 + i] = rd(S, t + (lane + 64 * q) * 16 + i);
        for (uint32_t i = 0; i < 16; ++i) W.b[kWTile + i] = rd(S, t + kWTile + i);
    } else {
        for (uint32_t q = 0; q <= kWQV; ++q)
            for (uint32_t lane = 0; lane < (q < kWQV ? 64u : 1u); ++lane) {
                const uint32_t o = q < kWQV ? (lane + 64 * q) * 16 : kWTile;
                for (uint32_t i = 0; i < 16; ++i)
                    W.b[o + i] = (uint64_t)t + o + i < S.seg ? rd(S, t + o + i) : 0;
            }
    }
    W.valid = kWTile + 16;
}

// wsmall_fetch + wsmall_store: one vector per lane + the slack
void window_fetch(Tile& W, const Seg& S, uint32_t t) {
    std::memset(W.b, 0xAB, sizeof W.b);
    const bool fast = S.vec && (uint64_t)t + kWSmall + 16 <= S.seg;
    for (uint32_t lane = 0; lane < 64; ++lane)
        for (uint32_t i = 0; i < 16; ++i)
            W.b[lane * 16 + i] = fast || (uint64_t)t + lane * 16 + i < S.seg ? rd(S, t + lane * 16 + i) : 0;
    for (uint32_t i = 0; i < 16; ++i) W.b[kWSmall + i] = fast || (uint64_t)t + kWSmall + i < S.seg ? rd(S, t + kWSmall + i) : 0;
    W.valid = kWSmall + 16;
}

// tile_header: three aligned LDS words at (c - t0) >> 2, funnel-shifted
void tile_header(const Tile& W, uint32_t c, uint32_t t0, uint32_t& crc, uint32_t& st) {
    const uint32_t h = c - t0, q = h >> 2;
    if (c < t0 || 4 * q + 12 > W.valid) die("LDS tile read outside the fetched tile", h, W.valid);
    uint8_t x[8];
    std::memcpy(x, W.b + h, 8);
    crc = uint32_t(x[0]) | uint32_t(x[1]) << 8 | uint32_t(x[2]) << 16 | uint32_t(x[3]) << 24;
    st = uint32_t(x[4]) | uint32_t(x[5]) << 8 | uint32_t(x[6]) << 16 | uint32_t(x[7]) << 24;
}

struct List {  // one sub-range's candidate slots
    std::vector<uint32_t>* rec;
    std::vector<uint32_t>* len;
    std::vector<uint32_t>* crc;
    uint64_t base, cap;
    void put(uint64_t i, uint32_t r, uint32_t n, uint32_t c) const {
        if (i >= cap) die("list write dropped by the capacity guard", i, cap);
        if (base + i >= rec->size()) die("list slot outside the table", base + i, rec->size());
        ++g_slots;
        (*rec)[base + i] = r;
        (*len)[base + i] = n;
        (*crc)[base + i] = c;
    }
};

struct WalkEnd {
    uint32_t count = 0, max_len = 0, kind = 0, stop = 0, pos = 0;
};

// walk_range (wal_device.hip): the 64-entry runs are flushed lane by lane.  The fast path
// reads a round of 64 headers, lane j at pos + j * g (g: the last record's stride), and takes
// the lanes up to the first one whose next header is not the next lane's position.
constexpr uint32_t kDirectStreak = 8;  // wal.cc: direct header rounds after a fast round this long

WalkEnd walk_range(Tile& W, const Seg& S, uint32_t pos, uint32_t hi, const List& out) {
    const uint32_t seg = S.seg;
    WalkEnd E;
    E.stop = seg;
    E.pos = pos;
    if ((uint64_t)pos + 8 > seg || pos >= hi) return E;
    uint32_t run[64][3], k = 0, g = 0, streak = 0;
    auto push = [&](uint32_t p, uint32_t n, uint32_t c) {
        E.max_len = std::max(E.max_len, n);
        run[k][0] = p, run[k][1] = n, run[k][2] = c;
        if (++k == 64) {
            for (uint32_t lane = 0; lane < 64; ++lane) out.put(E.count + lane, run[lane][0], run[lane][1], run[lane][2]);
            E.count += 64;
            k = 0;
        }
    };
    const uint32_t tlim = hi < seg ? hi : seg;
    uint32_t t0 = pos / kWTile * kWTile, tsz = kWTile;
    tile_fetch(W, S, t0);
    Tile next;
    while (true) {
        const bool more = tsz == kWTile && (uint64_t)t0 + kWTile < tlim;
        if (more) tile_fetch(next, S, t0 + kWTile);
        uint32_t done = 0;
        {  // direct rounds (kDirectStreak, wal.cc): 64 headers read from the segment, not the tile
            const uint32_t dend = hi < seg - 7 ? hi : seg - 7;
            while (g >= 8 && (streak >= kDirectStreak || (streak >= 2 && g * (streak + 1) > kWTile)) && pos < dend) {
                uint32_t hc[64], hs[64], hn[64];
                bool ok[64], chain[64];
                for (uint32_t lane = 0; lane < 64; ++lane) {
                    const uint32_t pj = pos + lane * g;
                    const bool inwin = pj < dend;
                    const uint32_t hp = inwin ? pj : pos;
                    uint8_t h[8];
                    for (uint32_t b = 0; b < 8; ++b) h[b] = rd(S, hp + b);  // checked: inside the segment
                    hc[lane] = uint32_t(h[0]) | uint32_t(h[1]) << 8 | uint32_t(h[2]) << 16 | uint32_t(h[3]) << 24;
                    hs[lane] = uint32_t(h[4]) | uint32_t(h[5]) << 8 | uint32_t(h[6]) << 16 | uint32_t(h[7]) << 24;
                    hn[lane] = hp + 8 + (hs[lane] >> 8);
                    ok[lane] = inwin && (hs[lane] & 0xffu) == 0 && hs[lane] >= 256u && hn[lane] <= seg;
                    chain[lane] = ok[lane] && hn[lane] == pj + g;
                }
                uint32_t f = 64;
                for (uint32_t lane = 0; lane < 64; ++lane)
                    if (!chain[lane]) {
                        f = lane;
                        break;
                    }
                for (uint32_t lane = 0; lane < 64; ++lane) {  // the next round, read speculatively
                    const uint32_t pj2 = pos + (64 + lane) * g;
                    const uint32_t hp2 = pj2 < dend ? pj2 : pos;
                    for (uint32_t b = 0; b < 8; ++b) (void)rd(S, hp2 + b);
                }
                const bool okf = f < 64 && ok[f];
                const uint32_t na = f + (okf ? 1 : 0);
                for (uint32_t j = 0; j < na; ++j) push(pos + j * g, hs[j] >> 8, hc[j]);
                streak = na;
                if (f == 64) {
                    pos = hn[63];
                } else if (okf) {
                    pos = hn[f];
                    g = (hs[f] >> 8) + 8;
                    if (streak < (g * (streak + 1) > kWTile ? 2u : kDirectStreak)) break;
                } else {
                    pos += f * g;
                    streak = 0;
                    break;
                }
            }
        }
        {
            const uint32_t tend = t0 + tsz < hi ? t0 + tsz : hi, lim = seg - 8;
            const uint32_t fend = lim + 1 < tend ? lim + 1 : tend;
            while (pos < fend) {
                uint32_t crc = 0, st = 0, npos;
                bool special = false;
                while (true) {  // one round: every lane reads its header, then the ballot
                    uint32_t hc[64], hs[64], hn[64];
                    bool ok[64], chain[64];
                    for (uint32_t lane = 0; lane < 64; ++lane) {
                        const uint32_t pj = pos + lane * g;
                        const bool inwin = pj < fend;
                        const uint32_t hp = inwin ? pj : pos;
                        tile_header(W, hp, t0, hc[lane], hs[lane]);
                        hn[lane] = hp + 8 + (hs[lane] >> 8);
                        ok[lane] = inwin && (hs[lane] & 0xffu) == 0 && hs[lane] >= 256u && hn[lane] <= seg;
                        chain[lane] = ok[lane] && hn[lane] == pj + g;
                    }
                    uint32_t f = 64;
                    for (uint32_t lane = 0; lane < 64; ++lane)
                        if (!chain[lane]) {
                            f = lane;
                            break;
                        }
                    const bool okf = f < 64 && ok[f];
                    const uint32_t na = f + (okf ? 1 : 0);
                    for (uint32_t j = 0; j < na; ++j) push(pos + j * g, hs[j] >> 8, hc[j]);
                    streak = na;
                    if (f == 64) {
                        pos = hn[63];
                    } else if (okf) {
                        pos = hn[f];
                        g = (hs[f] >> 8) + 8;
                    } else {
                        pos += f * g;
                        if (pos < fend) {
                            crc = hc[f];
                            st = hs[f];
                            special = true;
                        }
                        break;
                    }
                    if (pos >= fend) break;
                }
                if (!special) break;
                npos = pos + 8 + (st >> 8);
                const uint32_t type = st & 0xffu;
                if (type == 0 && npos <= seg && crc == kStaleZero) {
                    push(pos, 0u, crc);
                    pos += kStaleAdvance;
                    continue;
                }
                done = 1;
                if (type == 0) {
                    E.kind = CORRUPT;
                    E.stop = pos;
                } else if (type == 1) {
                    pos = seg;
                } else {
                    E.kind = BAD_TYPE;
                    E.stop = pos;
                }
                break;
            }
        }
        if (done || (uint64_t)pos + 8 > seg || pos >= hi) break;
        const uint32_t nt0 = pos / kWTile * kWTile;
        if (more && nt0 == t0 + kWTile) {
            W = next;
            t0 = nt0;
        } else if (pos - t0 < 2 * tsz) {
            tile_fetch(W, S, nt0);
            t0 = nt0;
            tsz = kWTile;
        } else {
            t0 = pos & ~15u;
            window_fetch(W, S, t0);
            tsz = kWSmall;
        }
    }
    for (uint32_t lane = 0; lane < k; ++lane) out.put(E.count + lane, run[lane][0], run[lane][1], run[lane][2]);
    E.count += k;
    E.pos = pos;
    return E;
}

bool header_ok(uint32_t crc, uint32_t st, uint32_t c, uint32_t seg, uint32_t* next, bool* last) {
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

// find_start: 64 candidates per step, one per lane; ballot -> the lowest lane that passes
uint32_t find_start(Tile& W, const Seg& S, uint32_t lo, uint32_t hi) {
    const uint32_t seg = S.seg;
    for (uint32_t t0 = lo; t0 < hi && t0 < lo + kWTile; t0 += kWTile) {
        tile_fetch(W, S, t0);
        const uint32_t tend = t0 + kWTile < hi ? t0 + kWTile : hi;
        for (uint32_t c0 = t0; c0 < tend; c0 += 64) {
            for (uint32_t lane = 0; lane < 64; ++lane) {
                const uint32_t c = c0 + lane;
                bool ok = false;
                if (c < tend && (uint64_t)c + 8 <= seg) {
                    uint32_t crc, st, next;
                    bool last;
                    tile_header(W, c, t0, crc, st);
                    ok = header_ok(crc, st, c, seg, &next, &last) && (last || next < t0 + 2 * kWTile);
                    for (uint32_t k = 1; ok && !last && k < kChainCheck && (uint64_t)next + 8 <= seg; ++k) {
                        if (next < t0 + kWTile) {
                            tile_header(W, next, t0, crc, st);
                        } else {
                            uint8_t h[8];
                            for (int i = 0; i < 8; ++i) h[i] = rd(S, (uint64_t)next + i);
                            crc = uint32_t(h[0]) | uint32_t(h[1]) << 8 | uint32_t(h[2]) << 16 | uint32_t(h[3]) << 24;
                            st = uint32_t(h[4]) | uint32_t(h[5]) << 8 | uint32_t(h[6]) << 16 | uint32_t(h[7]) << 24;
                        }
                        const uint32_t at = next;
                        ok = header_ok(crc, st, at, seg, &next, &last);
                    }
                }
                if (ok) return c;  // the ballot's lowest set lane
            }
        }
    }
    return hi;
}

struct Plan {
    uint64_t nsub, sub_bytes, sub_cap, cand_cap;
};

// wal_walk_plan (no forced workgroup kernel: the shipped build)
Plan walk_plan(uint64_t seg_bytes, uint64_t nseg, int cu, uint64_t sub_bytes) {
    const uint64_t tiles = (seg_bytes + kWTile - 1) / kWTile;
    uint64_t sub_tiles = tiles;
    if (sub_bytes) {
        sub_tiles = std::max<uint64_t>(1, sub_bytes / kWTile);
    } else {
        // the default replay plan walks with the CRCs in the same kernel: 15 walkers per CU
        // (k_wal_walk_crc, kFuseWaves; the walk itself is k_wal_walk_sub's, restated here)
        const uint64_t want = 15 * (uint64_t)(cu > 0 ? cu : 1);
        if (nseg > 0 && nseg < want) {
            const uint64_t per = (want + nseg - 1) / nseg;
            sub_tiles = std::max<uint64_t>(4, (tiles + per - 1) / per);
        }
    }
    sub_tiles = std::min(sub_tiles, tiles);
    sub_tiles = std::max(sub_tiles, (tiles + kMaxSub - 1) / kMaxSub);
    Plan p;
    p.sub_bytes = sub_tiles * kWTile;
    p.nsub = (seg_bytes + p.sub_bytes - 1) / p.sub_bytes;
    if (p.nsub == 1) p.sub_bytes = seg_bytes;
    p.sub_cap = p.sub_bytes / 8 + 1;
    p.cand_cap = p.nsub * p.sub_cap;
    if (p.nsub > kMaxSub) die("more sub-ranges than k_wal_gather stages", p.nsub, kMaxSub);
    return p;
}

struct SubMeta {
    uint32_t first, count, kind, stop, exit, max_len, fb;  // fb: the walker's inline-CRC result
};
struct SegMeta {
    uint32_t count, kind;
    uint64_t stop;
    uint32_t max_len, first_bad;  // first_bad: the segment's inline-CRC ordinal / unknown
};
constexpr uint32_t kNoBad = ~0u, kCrcUnknown = ~0u - 1, kCrcInlineMax = 1024;

// replay_pass (wal.cc): one device pass from start; appends the accepted offsets to recs
void replay_pass(const std::vector<uint8_t>& file, uint64_t seg_bytes, uint64_t start, uint64_t force_sub, int cu,
                 std::vector<uint64_t>& recs, uint64_t& end_out, int& status_out) {
    const uint64_t wal_bytes = file.size();
    const uint64_t nseg = wal_bytes / seg_bytes, s0 = std::min<uint64_t>(start / seg_bytes, nseg), nwork = nseg - s0;
    if (!nwork) {
        end_out = start;
        status_out = END;
        return;
    }
    const uint64_t base0 = s0 * seg_bytes, first_pos = start - base0;
    // the image as the kernels see it: A.wal = a 256-byte aligned copy of segments s0.. (the
    // staged copy, or the caller's device image + base0)
    const uint64_t img_bytes = nwork * seg_bytes;
    std::vector<uint8_t> store(img_bytes + 256 + 64);
    uint8_t* wal = store.data() + ((256 - (reinterpret_cast<uintptr_t>(store.data()) & 255)) & 255);
    std::memcpy(wal, file.data() + base0, img_bytes);
    const Plan plan = walk_plan(seg_bytes, nwork, cu, force_sub);
    std::vector<uint32_t> crec(nwork * plan.cand_cap), clen(crec.size()), ccrc(crec.size());
    std::vector<SegMeta> meta(nwork);
    std::vector<SubMeta> sub(nwork * plan.nsub);
    std::vector<uint32_t> span(nwork * plan.nsub * 2, 0xFFFFFFFFu);
    Tile W;
    // k_wal_walk_sub: one wave per (segment, sub-range)
    for (uint64_t s = 0; s < nwork; ++s)
        for (uint64_t j = 0; j < plan.nsub; ++j) {
            const uint64_t rel = s * seg_bytes;
            const Seg S{wal + rel, (uint32_t)seg_bytes, ((reinterpret_cast<uintptr_t>(wal + rel)) & 15u) == 0};
            const uint32_t lo = (uint32_t)(j * plan.sub_bytes);
            const uint32_t hi = (uint64_t)lo + plan.sub_bytes < S.seg ? lo + (uint32_t)plan.sub_bytes : S.seg;
            const uint32_t st0 = s == 0 ? (uint32_t)first_pos : 0u;
            uint32_t first;
            if (st0 >= hi) first = hi;
            else if (st0 >= lo) first = st0;
            else first = find_start(W, S, lo, hi);
            const List L{&crec, &clen, &ccrc, s * plan.cand_cap + j * plan.sub_cap, plan.sub_cap};
            const WalkEnd E = walk_range(W, S, first, hi, L);
            if (E.count > plan.sub_cap) die("walker list longer than its capacity", E.count, plan.sub_cap);
            // k_wal_walk_crc's crc_list: the walker's own list, the first entry whose payload CRC
            // differs (size 0: checked by the walk), or unknown when a payload is over 1 KiB
            uint32_t fb = kNoBad;
            if (E.count && E.max_len > kCrcInlineMax) {
                fb = kCrcUnknown;
            } else {
                for (uint32_t i = 0; i < E.count; ++i) {
                    const uint64_t slot = L.base + i;
                    if (clen[slot] && crc32c(S.img + crec[slot] + 8, clen[slot]) != ccrc[slot]) {
                        fb = i;
                        break;
                    }
                }
            }
            if (plan.nsub == 1) {
                const bool spill = !E.kind && E.pos > S.seg;
                const uint32_t kind = spill ? (uint32_t)SPILL : E.kind, stop = spill ? E.pos : E.stop;
                meta[s] = SegMeta{E.count, kind, base0 + rel + (kind ? stop : S.seg), E.max_len, fb};
                span[2 * s] = 0;
                span[2 * s + 1] = 0;
            } else {
                sub[s * plan.nsub + j] = SubMeta{first, E.count, E.kind, E.stop, E.pos, E.max_len, fb};
            }
        }
    // k_wal_resolve: one wave per segment, along the real chain
    if (plan.nsub > 1)
        for (uint64_t s = 0; s < nwork; ++s) {
            const uint64_t P = plan.nsub, rel = s * seg_bytes;
            const Seg S{wal + rel, (uint32_t)seg_bytes, ((reinterpret_cast<uintptr_t>(wal + rel)) & 15u) == 0};
            const uint32_t seg = S.seg;
            uint32_t pos = s == 0 ? (uint32_t)first_pos : 0u, count = 0, kind = 0, stop = seg, mx = 0;
            uint32_t sfb = kNoBad;  // k_wal_resolve's inline-CRC ordinal of the segment
            bool sunk = false;
            for (uint64_t j = 0; j < P; ++j) {
                const uint32_t lo = (uint32_t)(j * plan.sub_bytes);
                const uint32_t hi = (uint64_t)lo + plan.sub_bytes < seg ? lo + (uint32_t)plan.sub_bytes : seg;
                uint32_t st = (uint32_t)(j * plan.sub_cap), n = 0;
                if (!kind && pos < hi && (uint64_t)pos + 8 <= seg) {
                    const SubMeta m = sub[s * P + j];
                    const uint64_t cbase = s * plan.cand_cap;
                    auto rec_at = [&](uint32_t i) {
                        if (i >= plan.sub_cap || i >= m.count) die("resolver list read outside the run", i, m.count);
                        return crec[cbase + st + i];
                    };
                    int64_t idx = -1;
                    if (m.first == pos) {
                        idx = 0;
                    } else if (m.first < pos && m.count > 1) {
                        uint32_t a = 1, b = m.count;
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
                        if (n && (m.fb == kCrcUnknown || (m.fb != kNoBad && m.fb < (uint32_t)idx))) sunk = true;
                        else if (m.fb < kCrcUnknown) sfb = std::min(sfb, count + (m.fb - (uint32_t)idx));
                        pos = m.exit;
                        mx = std::max(mx, m.max_len);
                        if (m.kind) {
                            kind = m.kind;
                            stop = m.stop;
                        }
                    } else {
                        const List L{&crec, &clen, &ccrc, cbase + st, plan.sub_cap};
                        const WalkEnd E = walk_range(W, S, pos, hi, L);
                        n = E.count;
                        if (n) sunk = true;  // walked by the resolver: no inline CRCs
                        pos = E.pos;
                        mx = std::max(mx, E.max_len);
                        if (E.kind) {
                            kind = E.kind;
                            stop = E.stop;
                        }
                    }
                }
                span[2 * (s * P + j)] = st;
                span[2 * (s * P + j) + 1] = count;
                count += n;
            }
            if (!kind && pos > seg) {
                kind = SPILL;
                stop = pos;
            }
            meta[s] = SegMeta{count, kind, base0 + rel + (kind ? stop : seg), mx, sunk ? kCrcUnknown : sfb};
        }
    // replay_core: replay enters segment s + 1 only if segment s ended cleanly
    int status = END;
    uint64_t end = wal_bytes, w1 = nwork;
    for (uint64_t w = 0; w < nwork; ++w)
        if (meta[w].kind != END) {
            status = (int)meta[w].kind;
            end = meta[w].stop;
            w1 = w + 1;
            break;
        }
    std::vector<uint64_t> cb(w1);
    uint64_t n_all = 0;
    for (uint64_t w = 0; w < w1; ++w) {
        cb[w] = n_all;
        n_all += meta[w].count;
    }
    // k_wal_gather: candidate i of segment w finds its run by a binary search over the spans
    std::vector<uint64_t> off(n_all);
    std::vector<uint32_t> len(n_all), stored(n_all);
    for (uint64_t w = 0; w < w1; ++w) {
        const uint32_t P = (uint32_t)plan.nsub;
        const uint32_t* sp = span.data() + 2 * w * plan.nsub;
        for (uint32_t j = 0; j < P; ++j)
            if (sp[2 * j] == 0xFFFFFFFFu) die("span never written", w, j);
        for (uint32_t i = 0; i < meta[w].count; ++i) {
            uint32_t a = 0, b = P;
            while (b - a > 1) {
                const uint32_t mid = (a + b) / 2;
                if (sp[2 * mid + 1] <= i) a = mid;
                else b = mid;
            }
            const uint64_t slot = sp[2 * a] + (uint64_t)(i - sp[2 * a + 1]);
            if (slot >= plan.cand_cap) die("gather slot outside the segment's table", slot, plan.cand_cap);
            if (cb[w] + i >= n_all) die("gather index outside the lists", cb[w] + i, n_all);
            ++g_slots;
            off[cb[w] + i] = w * seg_bytes + crec[w * plan.cand_cap + slot];
            len[cb[w] + i] = clen[w * plan.cand_cap + slot];
            stored[cb[w] + i] = ccrc[w * plan.cand_cap + slot];
        }
    }
    // the CRC batch over arena = A.wal + 8 (k_ragged_direct / the unit plan read whole 16-byte
    // blocks of each record: its head block, the aligned body and its tail block) + k_wal_compare
    const uint64_t lim16 = (img_bytes + 15) / 16 * 16;
    uint64_t first_bad = n_all;
    for (uint64_t g = 0; g < n_all; ++g) {
        const uint64_t p = off[g] + 8, e = p + len[g];
        if (len[g] && (p / 16 * 16 >= lim16 || (e + 15) / 16 * 16 > lim16)) die("CRC read outside the image", p, e);
        if (len[g] && crc32c(wal + p, len[g]) != stored[g]) {
            first_bad = g;
            break;
        }
    }
    // k_wal_plan with the inline CRCs: the first mismatch = min over the segments entered of
    // list offset + ordinal, unless some segment is unknown (the replay then runs the batch
    // above); when known it must be the batch's answer
    bool unknown = false;
    uint64_t inline_bad = ~0ull;
    for (uint64_t w = 0; w < w1; ++w) {
        if (meta[w].first_bad == kCrcUnknown) unknown = true;
        else if (meta[w].first_bad != kNoBad) inline_bad = std::min<uint64_t>(inline_bad, cb[w] + meta[w].first_bad);
    }
    if (!unknown) {
        const uint64_t want = first_bad < n_all ? first_bad : ~0ull;
        if (inline_bad != want) die("inline CRC first mismatch differs from the batch's", inline_bad, want);
        ++g_inline_known;
    } else {
        ++g_inline_unknown;
    }
    uint64_t accepted = n_all;
    if (first_bad < n_all) {
        accepted = first_bad;
        status = CORRUPT;
        end = base0 + off[first_bad];
    }
    for (uint64_t g = 0; g < accepted; ++g) recs.push_back(off[g] + base0);
    end_out = end;
    status_out = status;
    std::fprintf(stderr,
                 "pass from %llu: plan nsub=%llu sub_bytes=%llu; checked %llu walker reads, %llu list slots; inline "
                 "CRCs %s\n",
                 (unsigned long long)start, (unsigned long long)plan.nsub, (unsigned long long)plan.sub_bytes,
                 (unsigned long long)g_reads, (unsigned long long)g_slots, unknown ? "unknown (batch)" : "known");
}

}  // namespace

int main(int argc, char** argv) {
    if (argc != 6) {
        std::fprintf(stderr, "usage: %s image seg_bytes start sub_bytes cu\n", argv[0]);
        return 2;
    }
    FILE* f = std::fopen(argv[1], "rb");
    if (!f) return 2;
    std::vector<uint8_t> file;
    uint8_t buf[1 << 16];
    size_t got;
    while ((got = std::fread(buf, 1, sizeof buf, f)) > 0) file.insert(file.end(), buf, buf + got);
    std::fclose(f);
    const uint64_t wal_bytes = file.size(), seg_bytes = std::strtoull(argv[2], nullptr, 10);
    uint64_t start = std::strtoull(argv[3], nullptr, 10);
    const uint64_t force_sub = std::strtoull(argv[4], nullptr, 10);
    const int cu = std::atoi(argv[5]);
    if (!seg_bytes || wal_bytes % seg_bytes || start > wal_bytes || seg_bytes >= (1ull << 31)) return 2;
    // replay_core (wal.cc): passes until the chain no longer spills past a segment end
    std::vector<uint64_t> recs;
    uint64_t end = 0;
    int status = END;
    while (true) {
        replay_pass(file, seg_bytes, start, force_sub, cu, recs, end, status);
        if (status != SPILL) break;
        if (end <= start) die("spill pass made no progress", start, end);
        start = end;
        if (start >= wal_bytes) {
            status = END;
            break;
        }
    }
    std::printf("%llu %llu %d\n", (unsigned long long)recs.size(), (unsigned long long)end, status);
    for (uint64_t r : recs) std::printf("%llu\n", (unsigned long long)r);
    return 0;
}
