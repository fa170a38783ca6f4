// tests/cpp/host_logic_test.cc -- the library's host-side logic under AddressSanitizer and
// UBSan (test infrastructure; built by `make -C karma_amd/csrc san`, run by
// tests/test_sanitizers.py).  Linked against the sanitized host objects of the library.
//
//   1. crc32c::Extend / karma_crc32c_extend_host / _portable / _combine against a bitwise
//      CRC-32C (karma-util/crc32c.cc:275-376 semantics) at every alignment;
//   2. WalPlacer (the writer's placement, sivir.cc:276-317, segment_file.cc:21-49, 74-77)
//      against its invariants and a direct restatement of the writer's loop;
//   3. kfp_walk (connection::read_frame's parse loop, frame.cc:62-130) on valid, truncated,
//      corrupted and random buffers;
//   4. wal_walk_plan's sub-range split for many segment sizes, counts and CU counts;
//   5. without a device: every C ABI entry point with real arguments runs its host part
//      (validation, placement, directory scan, structural walks) and refuses cleanly;
//   6. the grouped point-to-point gather (gather_p2p.h, karma_crc32c_gather_u32 without
//      ncclGather) through a recording stub of the RCCL calls: every rank's shard lands at
//      recv + p * count on the root, the root's own by its copy, each slot written once;
//   7. the per-stream state's lifetime (stream_state.h, karma_crc32c_release_stream / _trim /
//      _graph_hold) through a recording allocator: 1,000 streams created, used with every kind
//      of growth, released; captured streams keep outgrown buffers until a trim with no graph
//      hold; exited threads' state is freed by the next trim; nothing leaks or is freed twice
//      (ASan would also report either);
//   8. the multi-device host batches' split and merge (multi_dev.h) through stubs of the
//      one-device calls: ranges cover the batch once in order, byte-balanced cuts, the shares'
//      CRCs land in record order, a failing share fails the call with its detail, and replay
//      shares merge as one sequential replay would (clean ends, a stop inside a range, a spill
//      past a range's end handed back).
#include <hip/hip_runtime_api.h>
#include <unistd.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <thread>
#include <random>
#include <string>
#include <vector>

#include "engine.h"
#include "gather_p2p.h"
#include "stream_state.h"
#include "multi_dev.h"
#include "karma-util/crc32c.h"
#include "karma_crc32c.h"
#include "wal_place.h"

using namespace karma::engine;

namespace {

int g_fail = 0;
#define CHECK(c)                                                                     \
    do {                                                                             \
        if (!(c)) {                                                                  \
            std::fprintf(stderr, "%s:%d: CHECK failed: %s\n", __FILE__, __LINE__, #c); \
            if (++g_fail > 20) std::exit(1);                                         \
        }                                                                            \
    } while (0)

uint32_t crc_bitwise(uint32_t init, const uint8_t* p, size_t n) {
    uint32_t l = init ^ 0xFFFFFFFFu;
    for (size_t i = 0; i < n; ++i) {
        l ^= p[i];
        for (int k = 0; k < 8; ++k) l = (l >> 1) ^ (0x82F63B78u & (0u - (l & 1u)));
    }
    return l ^ 0xFFFFFFFFu;
}

void test_host_crc(std::mt19937_64& rng) {
    std::vector<uint8_t> buf(70000 + 64);
    for (auto& b : buf) b = uint8_t(rng());
    for (size_t n = 0; n <= 600; ++n)
        for (size_t a = 0; a < 16; ++a) {
            const uint32_t init = uint32_t(rng());
            const uint8_t* p = buf.data() + a;
            const uint32_t want = crc_bitwise(init, p, n);
            CHECK(karma_crc32c_extend_host(init, p, n) == want);
            CHECK(karma_crc32c_extend_host_portable(init, p, n) == want);
            CHECK(crc32c::Extend(init, reinterpret_cast<const char*>(p), n) == want);
        }
    for (size_t n : {4095, 4096, 4097, 65535, 65536, 65543, 70000}) {
        const uint32_t want = crc_bitwise(0, buf.data() + 3, n);
        CHECK(karma_crc32c_extend_host(0, buf.data() + 3, n) == want);
        CHECK(karma_crc32c_extend_host_portable(0, buf.data() + 3, n) == want);
        for (size_t cut : {size_t(0), size_t(1), n / 3, n - 1, n}) {  // Value(A||B) = Combine(Value(A), Value(B), |B|)
            const uint32_t a = crc_bitwise(0, buf.data() + 3, cut), b = crc_bitwise(0, buf.data() + 3 + cut, n - cut);
            CHECK(karma_crc32c_combine(a, b, n - cut) == want);
        }
    }
    CHECK(crc32c::Value("123456789", 9) == 0xE3069283u);
    CHECK(crc32c::Mask(0xE3069283u) == 0xC78AB0E5u && crc32c::Unmask(crc32c::Mask(0x12345678u)) == 0x12345678u);
}

// The writer's loop restated (wal_model.append): returns the cursor; fills at / footers.
uint64_t place_model(const std::vector<uint64_t>& len, uint64_t seg, uint64_t wal, uint64_t cursor,
                     std::vector<uint64_t>* at, std::vector<std::pair<uint64_t, uint64_t>>* footers) {
    for (uint64_t n : len) {
        if (n + 8 > seg || (n >> 24)) break;
        const uint64_t seg_end = (cursor / seg + 1) * seg;
        if (cursor + 8 + n > seg_end) {
            footers->emplace_back(cursor, seg_end);
            cursor = seg_end;
        }
        if (cursor + 8 + n > wal) break;
        at->push_back(cursor);
        cursor += 8 + n;
    }
    return cursor;
}

void test_placement(std::mt19937_64& rng) {
    for (int it = 0; it < 3000; ++it) {
        const uint64_t seg = std::vector<uint64_t>{8, 9, 16, 100, 4096, 4100, 65536, 1 << 20}[rng() % 8];
        const uint64_t nseg = 1 + rng() % 6, wal = nseg * seg;
        const uint64_t cursor = (rng() % 4 == 0) ? rng() % wal : 0;
        std::vector<uint64_t> len(rng() % 200);
        for (auto& l : len) {
            const int k = int(rng() % 10);
            l = k == 0 ? 0 : k == 1 ? seg - 8 : k == 2 ? seg - 7 : k == 3 ? (1u << 24) : rng() % (seg / 2 + 1);
        }
        std::vector<uint64_t> at_m;
        std::vector<std::pair<uint64_t, uint64_t>> ft_m;
        const uint64_t cur_m = place_model(len, seg, wal, cursor, &at_m, &ft_m);
        WalPlacer P(seg, wal, cursor);
        std::vector<uint64_t> at;
        std::vector<std::pair<uint64_t, uint64_t>> ft;
        for (uint64_t L : len) {
            uint64_t a = 0, f0, f1;
            const bool ok = P.place(L, &a, &f0, &f1);
            if (f1 > f0) ft.emplace_back(f0, f1);
            if (!ok) break;
            CHECK(a / seg == (a + 8 + L - 1) / seg);  // a record never straddles a segment end
            CHECK(a + 8 + L <= wal);
            at.push_back(a);
        }
        CHECK(at == at_m);
        CHECK(ft == ft_m);
        CHECK(P.cur == cur_m);
        // the run form of the parallel writer (wal_append.cc): same records, footers and cursor
        size_t n_valid = 0;
        while (n_valid < len.size() && len[n_valid] + 8 <= seg && !(len[n_valid] >> 24)) ++n_valid;
        std::vector<uint64_t> V(n_valid + 1, 0);
        for (size_t i = 0; i < n_valid; ++i) V[i + 1] = V[i] + len[i] + 8;
        std::vector<WalRun> runs;
        std::vector<WalFooter> rft;
        uint64_t rcur = cursor;
        const size_t placed = place_runs(seg, wal, &rcur, n_valid, [&](size_t i) { return V[i]; },
                                         [&](size_t i) { return len[i]; }, &runs, &rft);
        std::vector<uint64_t> rat;
        for (const auto& r : runs)
            for (size_t i = r.i0; i < r.i1; ++i) rat.push_back(r.base + V[i]);
        std::vector<std::pair<uint64_t, uint64_t>> rftp;
        for (const auto& f : rft) rftp.emplace_back(f.f0, f.f1);
        CHECK(placed == at.size());
        CHECK(rat == at);
        CHECK(rftp == ft);
        CHECK(rcur == P.cur);
        for (const auto& f : ft) CHECK(f.second % seg == 0 && f.second > f.first && f.second - f.first < seg);
    }
}

void put32(std::vector<uint8_t>& b, size_t at, uint32_t v) { std::memcpy(b.data() + at, &v, 4); }

void test_kfp_walk(std::mt19937_64& rng) {
    for (int it = 0; it < 2000; ++it) {
        std::vector<uint8_t> b;
        std::vector<uint64_t> frames;
        const int nf = int(rng() % 20);
        for (int f = 0; f < nf; ++f) {
            const uint32_t hl = uint32_t(rng() % 70), pl = uint32_t(rng() % 300), fl = 16 + hl + pl + 4;
            frames.push_back(b.size());
            const size_t o = b.size();
            b.resize(o + fl);
            for (size_t i = o; i < o + fl; ++i) b[i] = uint8_t(rng());
            put32(b, o, fl);
            b[o + 4] = KARMA_KFP_MAGIC;
            put32(b, o + 12, hl);
        }
        KfpWalk W;
        CHECK(kfp_walk(b.data(), b.size(), 1 << 20, &W) == KARMA_KFP_OK);
        CHECK(W.frame == frames && W.consumed == b.size());
        if (!b.empty()) {  // truncated: the last frame is incomplete
            KfpWalk T;
            CHECK(kfp_walk(b.data(), b.size() - 1, 1 << 20, &T) == KARMA_KFP_OK);
            CHECK(T.frame.size() + 1 == frames.size());
            std::vector<uint8_t> c = b;  // one corrupted field
            const size_t f = frames[rng() % frames.size()];
            const int what = int(rng() % 4);
            int want;
            if (what == 0) {
                put32(c, f, KARMA_KFP_MAX_FRAME + 1), want = KARMA_KFP_BAD_SIZE;
            } else if (what == 1) {
                c[f + 4] ^= 1, want = KARMA_KFP_BAD_MAGIC;
            } else if (what == 2) {
                uint32_t fl;
                std::memcpy(&fl, c.data() + f, 4);
                put32(c, f + 12, fl - 19), want = KARMA_KFP_BAD_HEADER_LEN;
            } else {
                put32(c, f, 19), want = KARMA_KFP_BAD_LENGTH;
            }
            KfpWalk X;
            CHECK(kfp_walk(c.data(), c.size(), 1 << 20, &X) == want);
            CHECK(X.consumed == f);
        }
    }
    std::vector<uint8_t> junk(1 << 16);  // random bytes: whatever the verdict, every read in bounds
    for (int it = 0; it < 4000; ++it) {
        const size_t n = rng() % junk.size();
        for (size_t i = 0; i < n; ++i) junk[i] = uint8_t(rng() % 5 == 0 ? KARMA_KFP_MAGIC : rng());
        if (n >= 4 && rng() % 2) put32(junk, 0, uint32_t(20 + rng() % 64));
        KfpWalk W;
        (void)kfp_walk(junk.data(), n, 1 + rng() % 64, &W);
        CHECK(W.consumed <= n);
    }
}

void test_walk_plan() {
    for (uint64_t seg : {8ull, 100ull, 4096ull, 4100ull, 16388ull, 65536ull, 262148ull, 1ull << 20, 32ull << 20,
                         (1ull << 31) - 8})
        for (uint64_t nseg : {1ull, 2ull, 7ull, 188ull, 4096ull, 100000ull})
            for (int cu : {1, 80, 256})
                for (uint64_t sub : {0ull, 4096ull, 16384ull, 1ull << 30}) {
                    const WalWalkPlan p = wal_walk_plan(seg, nseg, cu, sub);
                    CHECK(p.nsub >= 1 && p.nsub <= kMaxSub);
                    CHECK(p.nsub * p.sub_bytes >= seg && (p.nsub - 1) * p.sub_bytes < seg);
                    CHECK(p.nsub == 1 ? p.sub_bytes == seg : p.sub_bytes % kWalkTile == 0);
                    CHECK(p.sub_cap == p.sub_bytes / 8 + 1 && p.cand_cap == p.nsub * p.sub_cap);
                }
}

void test_abi_without_device() {
    int n = 0;
    if (hipGetDeviceCount(&n) == hipSuccess && n > 0) {
        std::printf("(a device is visible: the no-device checks are skipped)\n");
        return;
    }
    std::vector<uint8_t> src(1 << 16, 0x5A), wal(8 * 4096);
    std::vector<uint64_t> off(100);
    std::vector<uint32_t> len(100, 300), out(100);
    for (size_t i = 0; i < off.size(); ++i) off[i] = i * 300;
    uint64_t cursor = 0, recoff[100];
    size_t nf = 0;
    CHECK(karma_wal_append_batch(src.data(), off.data(), len.data(), 100, wal.data(), wal.size(), 4096, &cursor, recoff,
                                 &nf, 0) == KARMA_E_NO_DEVICE);
    CHECK(karma_wal_append_batch(src.data(), off.data(), len.data(), 100, wal.data(), wal.size() - 1, 4096, &cursor,
                                 recoff, &nf, 0) == KARMA_E_INVALID);
    uint64_t nrec, stop, base;
    int status;
    CHECK(karma_wal_replay(wal.data(), nullptr, wal.size(), 4096, 0, &nrec, &stop, &status, recoff, 100, 0) ==
          KARMA_E_NO_DEVICE);
    karma_wal_tuning t{4096, KARMA_WAL_CRC_DIRECT, 0};
    CHECK(karma_wal_replay_tuned(wal.data(), nullptr, wal.size(), 4096, 0, &nrec, &stop, &status, recoff, 100, 0,
                                 &t) == KARMA_E_NO_DEVICE);
    t.crc_batch = 7;
    CHECK(karma_wal_replay_tuned(wal.data(), nullptr, wal.size(), 4096, 0, &nrec, &stop, &status, recoff, 100, 0,
                                 &t) == KARMA_E_INVALID);
    CHECK(karma_wal_replay(wal.data(), nullptr, wal.size(), 4096, wal.size(), &nrec, &stop, &status, recoff, 100,
                           0) == 0 &&
          nrec == 0 && stop == wal.size() && status == KARMA_WAL_END);
    // a segment directory: scanned, opened, then the device is needed
    char dir[] = "/tmp/karma_san_XXXXXX";
    CHECK(mkdtemp(dir) != nullptr);
    for (int i = 0; i < 3; ++i) {
        const std::string p = std::string(dir) + "/" + std::to_string(8192 + i * 4096);
        FILE* f = std::fopen(p.c_str(), "wb");
        std::fwrite(wal.data(), 1, 4096, f);
        std::fclose(f);
    }
    FILE* f = std::fopen((std::string(dir) + "/LOCK").c_str(), "wb");
    std::fclose(f);
    CHECK(karma_wal_replay_dir(dir, 0, 8192, &base, &nrec, &stop, &status, recoff, 100, 0) == KARMA_E_NO_DEVICE);
    CHECK(karma_wal_replay_dir(dir, 0, 0, &base, &nrec, &stop, &status, recoff, 100, 0) == KARMA_E_INVALID);
    const int devs[2] = {0, 1};
    CHECK(karma_crc32c_batch_fixed_host_multi(src.data(), 300, 100, 0, out.data(), devs, 2) == KARMA_E_NO_DEVICE);
    CHECK(karma_crc32c_batch_fixed_host_multi(src.data(), 300, 100, 0, out.data(), devs, 0) == KARMA_E_INVALID);
    CHECK(karma_wal_replay_multi(wal.data(), wal.size(), 4096, 0, &nrec, &stop, &status, recoff, 100, devs, 2) ==
          KARMA_E_NO_DEVICE);
    for (int i = 0; i < 3; ++i) unlink((std::string(dir) + "/" + std::to_string(8192 + i * 4096)).c_str());
    unlink((std::string(dir) + "/LOCK").c_str());
    rmdir(dir);
    CHECK(karma_wal_replay_dir("/nonexistent/karma", 0, 0, &base, &nrec, &stop, &status, recoff, 100, 0) ==
          KARMA_E_IO);
    // batches
    CHECK(karma_crc32c_batch_ragged_host(src.data(), src.size(), off.data(), len.data(), 100, 0, out.data(), 0) ==
          KARMA_E_NO_DEVICE);
    off[99] = src.size();
    CHECK(karma_crc32c_batch_ragged_host(src.data(), src.size(), off.data(), len.data(), 100, 0, out.data(), 0) ==
          KARMA_E_INVALID);
    CHECK(karma_crc32c_batch_fixed_host(src.data(), 512, 64, 0, out.data(), 0) == KARMA_E_NO_DEVICE);
    CHECK(karma_crc32c_batch_fixed(src.data(), 512, 64, nullptr, 0, out.data(), nullptr) == KARMA_E_NO_DEVICE);
    CHECK(karma_crc32c_batch_ragged_bounded(src.data(), off.data(), len.data(), 100, 0, 300, nullptr, 0, out.data(),
                                            nullptr) == KARMA_E_NO_DEVICE);
    // KFP: encode refuses at the CRC batch; parse walks the frames, then refuses
    std::vector<uint8_t> frames(4096);
    size_t ne = 0;
    uint64_t bytes = 0;
    std::vector<int16_t> op(4, 1);
    std::vector<uint8_t> flag(4, 0);
    std::vector<uint32_t> seq(4, 7), hl(4, 10), pl(4, 20);
    std::vector<uint64_t> ho(4, 0), po(4, 100);
    CHECK(karma_kfp_encode_batch(src.data(), ho.data(), hl.data(), src.data(), po.data(), pl.data(), op.data(),
                                 flag.data(), seq.data(), 4, frames.data(), frames.size(), nullptr, &ne, &bytes,
                                 0) == KARMA_E_NO_DEVICE);
    size_t nfr = 0;
    uint64_t used = 0;
    CHECK(karma_kfp_parse_batch(frames.data(), nullptr, 0, 16, nullptr, &nfr, &used, &status, 0) == 0 && nfr == 0);
}

}  // namespace

// A stub of the RCCL calls gather_p2p makes: records them (rank, op, buffer, count, peer).
struct P2POp {
    int rank;
    char op;  // 'S' send, 'R' recv, 'C' root's copy, '[' / ']' group
    const uint32_t* src;
    uint32_t* dst;
    size_t count;
    int peer;
};
struct StubOps {
    int rank;
    std::vector<P2POp>* log;
    int fail_at = -1;  // make the n-th operation of this rank fail (error paths)
    int n = 0;
    int rec(P2POp o) {
        log->push_back(o);
        return n++ == fail_at ? KARMA_E_RCCL : 0;
    }
    int group_start() { return rec({rank, '[', nullptr, nullptr, 0, -1}); }
    int group_end() { return rec({rank, ']', nullptr, nullptr, 0, -1}); }
    int send(const uint32_t* b, size_t c, int peer) { return rec({rank, 'S', b, nullptr, c, peer}); }
    int recv(uint32_t* b, size_t c, int peer) { return rec({rank, 'R', nullptr, b, c, peer}); }
    int copy(uint32_t* d, const uint32_t* s, size_t c) { return rec({rank, 'C', s, d, c, rank}); }
};

void test_gather_p2p() {
    for (int nranks = 1; nranks <= 8; ++nranks)
        for (int root = 0; root < nranks; ++root)
            for (size_t count : {size_t(0), size_t(1), size_t(5), size_t(1000)}) {
                std::vector<std::vector<uint32_t>> shard(nranks);
                for (int p = 0; p < nranks; ++p)
                    for (size_t i = 0; i < count; ++i) shard[p].push_back(uint32_t(p) << 24 | uint32_t(i));
                std::vector<uint32_t> out(nranks * count + 1, 0xDEADBEEFu);  // + a guard word
                std::vector<P2POp> log;
                for (int p = 0; p < nranks; ++p) {
                    StubOps ops{p, &log};
                    CHECK(gather_p2p(ops, p, nranks, root, shard[p].data(), count,
                                     p == root ? out.data() : nullptr) == 0);
                }
                // match the root's receives with the senders' sends, then apply them and the copy
                std::vector<int> written(nranks * count, 0);
                int sends = 0, recvs = 0, copies = 0;
                for (const P2POp& o : log) {
                    if (o.op == 'S') {
                        ++sends;
                        CHECK(o.rank != root && o.peer == root && o.count == count && o.src == shard[o.rank].data());
                    } else if (o.op == 'R' || o.op == 'C') {
                        CHECK(o.rank == root);
                        const int from = o.op == 'R' ? o.peer : root;
                        CHECK(o.count == count && from >= 0 && from < nranks);
                        CHECK(o.dst == out.data() + (size_t)from * count);  // slot p * count
                        if (o.op == 'R') {
                            ++recvs;
                            CHECK(from != root);
                        } else {
                            ++copies;
                            CHECK(o.src == shard[root].data());
                        }
                        for (size_t i = 0; i < o.count; ++i) {
                            const size_t slot = (size_t)(o.dst - out.data()) + i;
                            CHECK(slot < (size_t)nranks * count);
                            ++written[slot];
                            out[slot] = shard[from][i];
                        }
                    }
                }
                CHECK(sends == nranks - 1 && recvs == nranks - 1 && copies == (count ? 1 : 0));
                for (size_t i = 0; i < (size_t)nranks * count; ++i) CHECK(written[i] == 1);
                for (int p = 0; p < nranks; ++p)
                    for (size_t i = 0; i < count; ++i) CHECK(out[(size_t)p * count + i] == shard[p][i]);
                CHECK(out.back() == 0xDEADBEEFu);
                // the root's ops sit inside one group, the copy after it
                int depth = 0;
                for (const P2POp& o : log)
                    if (o.rank == root) {
                        if (o.op == '[') ++depth;
                        if (o.op == ']') --depth;
                        if (o.op == 'R') CHECK(depth == 1);
                        if (o.op == 'C') CHECK(depth == 0);
                    }
            }
    // a failing receive: the group is still closed, the error returned, no copy made
    for (int fail = 0; fail < 3; ++fail) {
        std::vector<uint32_t> a(4, 1), out(16, 0);
        std::vector<P2POp> log;
        StubOps ops{0, &log, fail};
        CHECK(gather_p2p(ops, 0, 4, 0, a.data(), 4, out.data()) == KARMA_E_RCCL);
        CHECK(!log.empty() && (fail == 0 || log.back().op == ']'));
        for (const P2POp& o : log) CHECK(o.op != 'C');
    }
    std::printf("gather_p2p: slots checked for 1..8 ranks, every root\n");
}

// ---- 7. stream state lifetime ------------------------------------------------------------
struct FakeOps {
    struct World {
        std::map<void*, size_t> live;  // allocation -> bytes
        std::map<void*, int> pending;  // stream -> work not yet drained
        std::map<void*, bool> capturing;
        std::vector<void*> freed_while_pending;  // buffers freed while their stream had work
        std::map<void*, void*> owner;            // allocation -> stream that used it last
        size_t allocs = 0, frees = 0, syncs = 0, device_syncs = 0;
    };
    World* w;
    int alloc(void** p, size_t bytes) {
        *p = std::malloc(bytes ? bytes : 1);
        w->live[*p] = bytes;
        ++w->allocs;
        return 0;
    }
    void free(void* p) {
        CHECK(w->live.count(p) == 1);  // never freed twice, never a foreign pointer
        auto o = w->owner.find(p);
        if (o != w->owner.end() && w->pending[o->second] > 0) w->freed_while_pending.push_back(p);
        w->live.erase(p);
        ++w->frees;
        std::free(p);
    }
    int zero(void* p, size_t bytes, void* s) {
        std::memset(p, 0, bytes);
        w->owner[p] = s;
        ++w->pending[s];
        return 0;
    }
    int sync_stream(void* s) {
        w->pending[s] = 0;
        ++w->syncs;
        return 0;
    }
    int sync_device(int) {
        for (auto& kv : w->pending) kv.second = 0;
        ++w->device_syncs;
        return 0;
    }
    bool capturing(void* s) { return w->capturing.count(s) && w->capturing[s]; }
};

void test_stream_state_lifetime(std::mt19937_64& rng) {
    using namespace karma::engine;
    FakeOps::World world;
    StreamStates<FakeOps> S(FakeOps{&world});
    auto use = [&](int dev, uintptr_t key, void* s, size_t ws, size_t lb, bool fused) {
        auto& st = S.get(dev, key, s);
        CHECK(S.grow(st, st.ws, ws, ws + ws / 4, false) == 0);
        world.owner[st.ws.p] = s;
        ++world.pending[s];  // a kernel on s uses the workspace
        if (lb) CHECK(S.grow(st, st.lb, lb, lb, true) == 0);
        if (fused) CHECK(S.grow(st, st.fused, 4096, 4096, true) == 0);
    };
    // 1,000 streams, each used with growing batches, then released: everything is freed, and no
    // buffer is freed while its stream still had work queued
    for (int i = 0; i < 1000; ++i) {
        void* s = reinterpret_cast<void*>(uintptr_t(0x10000 + 16 * i));
        for (int k = 0; k < 4; ++k) use(0, (uintptr_t)s, s, 1000 + (rng() % 100000), (k + 1) * 2048, k == 2);
        CHECK(S.release(0, (uintptr_t)s) == 0);
    }
    CHECK(S.states() == 0 && world.live.empty());
    CHECK(world.freed_while_pending.empty());
    CHECK(world.allocs == world.frees);
    // a captured stream keeps what it outgrows until a trim without a graph hold
    void* cs = reinterpret_cast<void*>(uintptr_t(0x900000));
    use(1, (uintptr_t)cs, cs, 1000, 0, false);
    world.capturing[cs] = true;
    use(1, (uintptr_t)cs, cs, 1000, 0, false);  // (the capture is noticed)
    world.capturing[cs] = false;
    const size_t before = world.live.size();
    use(1, (uintptr_t)cs, cs, 50000, 0, false);  // outgrown: kept
    CHECK(world.live.size() == before + 1);
    CHECK(S.hold(1, +1) == 1);
    CHECK(S.trim(1) == 0);
    CHECK(world.live.size() == before + 1);  // held
    CHECK(S.hold(1, -1) == 0);
    CHECK(S.trim(1) == 0);
    CHECK(world.live.size() == before);  // freed
    CHECK(S.hold(1, -5) == 0);            // never below zero
    // a per-thread key orphaned at thread exit: freed by the next trim on its device only
    const uintptr_t tkey = 0x13;
    use(2, tkey, nullptr, 777, 4096, true);
    use(3, tkey, nullptr, 999, 0, false);
    S.orphan(tkey);
    CHECK(S.zombies() == 2);
    CHECK(S.trim(2) == 0);
    CHECK(S.zombies() == 1);
    CHECK(S.trim(3) == 0);
    CHECK(S.zombies() == 0);
    // ... unless it saw a capture and a graph hold is active: a graph captured on the exited
    // thread's hipStreamPerThread may still be replayed
    const uintptr_t gkey = 0x15;
    void* ps = reinterpret_cast<void*>(uintptr_t(2));  // hipStreamPerThread
    use(2, gkey, ps, 555, 2048, false);
    world.capturing[ps] = true;
    use(2, gkey, ps, 555, 2048, false);
    world.capturing[ps] = false;
    S.orphan(gkey);
    CHECK(S.hold(2, +1) == 1);
    const size_t live_held = world.live.size();
    CHECK(S.trim(2) == 0);
    CHECK(S.zombies() == 1 && world.live.size() == live_held);  // kept under the hold
    CHECK(S.hold(2, -1) == 0);
    CHECK(S.trim(2) == 0);
    CHECK(S.zombies() == 0 && world.live.size() < live_held);  // freed once the hold is gone
    CHECK(S.release(1, (uintptr_t)cs) == 0);
    CHECK(S.release(1, 12345) == 0);  // unknown: nothing to do
    CHECK(world.live.empty() && world.allocs == world.frees);
}

// ---- 8. multi-device split and merge -------------------------------------------------------
void test_multi_device_split(std::mt19937_64& rng) {
    using namespace karma::engine;
    // contiguous equal-count ranges
    for (size_t n : {0ul, 1ul, 7ul, 8ul, 1000ul, 1000003ul})
        for (int parts = 1; parts <= 9; ++parts) {
            size_t prev = 0;
            for (int k = 0; k < parts; ++k) {
                const size_t lo = share_lo(n, parts, k), hi = share_lo(n, parts, k + 1);
                CHECK(lo == prev && hi >= lo && hi - lo <= n / parts + 1);
                prev = hi;
            }
            CHECK(prev == n);
        }
    // byte-balanced cuts: non-decreasing, cover [0, n), each share within one record of total/parts
    for (int trial = 0; trial < 200; ++trial) {
        const size_t n = rng() % 3000;
        std::vector<uint32_t> len(n);
        uint64_t total = 0;
        for (auto& l : len) total += (l = (uint32_t)(rng() % 2 ? rng() % 100 : rng() % 70000));
        uint32_t mx = 0;
        for (uint32_t l : len) mx = std::max(mx, l);
        const int parts = 1 + (int)(rng() % 8);
        const auto cuts = byte_balanced_cuts(len.data(), n, parts);
        CHECK(cuts.size() == (size_t)parts + 1 && cuts[0] == 0 && cuts[parts] == n);
        for (int k = 0; k < parts; ++k) {
            CHECK(cuts[k] <= cuts[k + 1]);
            uint64_t b = 0;
            for (size_t r = cuts[k]; r < cuts[k + 1]; ++r) b += len[r];
            CHECK(b <= total / parts + mx + 1);
        }
    }
    // the shares' results land in record order; a failing share fails with its own detail
    std::vector<uint32_t> out(10007, 0);
    const int parts = 5;
    std::string what;
    int rc = run_shares(
        parts,
        [&](int k) {
            for (size_t r = share_lo(out.size(), parts, k); r < share_lo(out.size(), parts, k + 1); ++r) out[r] = (uint32_t)r * 3u;
            return 0;
        },
        [] { return std::string("none"); }, &what);
    CHECK(rc == 0);
    for (size_t r = 0; r < out.size(); ++r) CHECK(out[r] == r * 3u);
    // (the detail is read on the failing share's own thread, right after its call)
    std::vector<std::thread::id> ids(parts);
    std::vector<std::string> tag(parts);
    std::mutex mu;
    rc = run_shares(
        parts,
        [&](int k) {
            std::lock_guard<std::mutex> g(mu);
            ids[k] = std::this_thread::get_id();
            tag[k] = "share-" + std::to_string(k);
            return k == 3 || k == 4 ? -3 - k : 0;
        },
        [&] {
            std::lock_guard<std::mutex> g(mu);
            for (int k = 0; k < parts; ++k)
                if (ids[k] == std::this_thread::get_id()) return tag[k];
            return std::string("?");
        },
        &what);
    CHECK(rc == -6 && what == "device share 3: share-3");
    // replay shares: whole segments from start's segment, contiguous, start kept in share 0
    const uint64_t seg = 4096;
    for (uint64_t nseg : {1ull, 2ull, 5ull, 64ull})
        for (uint64_t start : {0ull, 100ull, 4096ull * 1 + 17})
            for (int p : {1, 2, 3, 8}) {
                if (start >= nseg * seg) continue;
                auto sh = replay_shares(nseg * seg, seg, start, p);
                CHECK(!sh.empty() && sh[0].start == start && sh[0].lo == start / seg * seg && sh.back().hi == nseg * seg);
                for (size_t k = 0; k < sh.size(); ++k) {
                    CHECK(sh[k].hi > sh[k].lo && sh[k].lo % seg == 0 && sh[k].hi % seg == 0);
                    if (k) CHECK(sh[k].lo == sh[k - 1].hi && sh[k].start == sh[k].lo);
                }
            }
    // merge: clean ends chain the shares; a stop inside a range ends replay there; a stop past a
    // range's end is handed back (-1)
    auto mk = [](uint64_t lo, uint64_t hi, uint64_t n, uint64_t stop, int st) {
        ReplayShare s;
        s.lo = lo;
        s.hi = hi;
        s.n = n;
        s.stop = stop;
        s.status = st;
        for (uint64_t i = 0; i < n; ++i) s.rec.push_back(lo + 16 * i);
        return s;
    };
    uint64_t n = 0, stop = 0, rec[64];
    int st = 0, redo_rc = 0;
    int redos = 0;
    auto no_redo = [&](int, uint64_t) {
        ++redos;
        return 0;
    };
    std::vector<ReplayShare> sh = {mk(0, 100, 3, 100, 0), mk(100, 200, 2, 200, 0), mk(200, 300, 4, 300, 0)};
    CHECK(merge_replays(sh, &n, &stop, &st, rec, 64, 0, no_redo, &redo_rc) == 2 && n == 9 && stop == 300 && st == 0);
    CHECK(rec[0] == 0 && rec[3] == 100 && rec[5] == 200 && rec[8] == 248 && redos == 0);
    sh = {mk(0, 100, 3, 100, 0), mk(100, 200, 2, 150, 1), mk(200, 300, 4, 300, 0)};
    CHECK(merge_replays(sh, &n, &stop, &st, rec, 4, 0, no_redo, &redo_rc) == 1 && n == 5 && stop == 150 && st == 1);
    CHECK(redos == 0);
    // a spill past every share boundary: each costs one replay of the next share alone (a stub
    // counting the one-device calls), never the rest of the image on one device
    for (int parts : {2, 3, 8}) {
        sh.clear();
        for (int k = 0; k < parts; ++k) sh.push_back(mk(100 * k, 100 * (k + 1), 2, 100 * (k + 1) + 2, 0));
        std::vector<int> calls(parts, 0);
        auto redo = [&](int k, uint64_t from) {
            ++calls[k];
            CHECK(from == sh[k].lo + 2);
            sh[k] = mk(sh[k].lo, sh[k].hi, 3, k + 1 == parts ? sh[k].hi : sh[k].hi + 2, 0);  // spills on
            sh[k].rec.assign({from, from + 40, from + 80});
            return 0;
        };
        CHECK(merge_replays(sh, &n, &stop, &st, rec, 64, 0, redo, &redo_rc) == parts - 1);
        CHECK(n == 2 + 3 * (uint64_t)(parts - 1) && stop == 100ull * parts && st == 0 && redo_rc == 0);
        for (int k = 0; k < parts; ++k) CHECK(calls[k] == (k ? 1 : 0));
        CHECK(rec[2] == 102 && rec[3] == 142);
    }
    // a redone share that ends cleanly at its own hi: the later shares' first results stand
    sh = {mk(0, 100, 3, 102, 0), mk(100, 200, 2, 200, 0), mk(200, 300, 4, 300, 0)};
    int later = 0;
    auto redo1 = [&](int k, uint64_t from) {
        if (k != 1) ++later;
        sh[k] = mk(sh[k].lo, sh[k].hi, 1, 200, 0);
        sh[k].rec.assign({from});
        return 0;
    };
    CHECK(merge_replays(sh, &n, &stop, &st, rec, 64, 0, redo1, &redo_rc) == 2 && n == 8 && stop == 300 && later == 0);
    // a failing redo is reported
    sh = {mk(0, 100, 3, 102, 0), mk(100, 200, 2, 200, 0)};
    CHECK(merge_replays(sh, &n, &stop, &st, nullptr, 0, 0, [](int, uint64_t) { return -3; }, &redo_rc) == -1);
    CHECK(redo_rc == -3 && n == 3 && stop == 102);
}

int main() {
    std::mt19937_64 rng(20260131);
    test_host_crc(rng);
    test_placement(rng);
    test_kfp_walk(rng);
    test_walk_plan();
    test_abi_without_device();
    test_gather_p2p();
    test_stream_state_lifetime(rng);
    test_multi_device_split(rng);
    if (g_fail) {
        std::printf("host_logic_test: %d failures\n", g_fail);
        return 1;
    }
    std::printf("host_logic_test: ok\n");
    return 0;
}
