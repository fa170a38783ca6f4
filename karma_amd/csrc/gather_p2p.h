// karma_amd/csrc/gather_p2p.h -- the gather of per-record CRCs to the root as grouped
// point-to-point operations, for an RCCL without ncclGather.
//
// Rank p's `count` CRCs land at recv + p * count on the root, in rank order, so the gathered
// array is the whole batch's CRCs in record order (ranks hold contiguous record ranges,
// karma_amd/shard.py).  Inside one group the root posts a receive from every other rank and
// every other rank one send to the root; after the group the root copies its own shard into
// its slot (a device-to-device copy on the same stream).
//
// The operations go through `Ops` so the slot arithmetic is testable without RCCL or a device
// (tests/cpp/host_logic_test.cc drives it with a recording stub):
//   int group_start(); int group_end();
//   int send(const uint32_t* buf, size_t count, int peer);
//   int recv(uint32_t* buf, size_t count, int peer);
//   int copy(uint32_t* dst, const uint32_t* src, size_t count);     // the root's own shard
// Each returns 0 on success; the first failure is returned (group_end still runs once the
// group has started).
#pragma once

#include <cstddef>
#include <cstdint>

namespace karma::engine {

template <class Ops>
int gather_p2p(Ops& ops, int rank, int nranks, int root, const uint32_t* send, size_t count, uint32_t* recv) {
    int e = ops.group_start();
    if (e) return e;
    if (rank == root) {
        for (int p = 0; p < nranks && !e; ++p)
            if (p != root) e = ops.recv(recv + (size_t)p * count, count, p);
    } else {
        e = ops.send(send, count, root);
    }
    const int e2 = ops.group_end();
    if (e) return e;
    if (e2) return e2;
    if (rank == root && count) return ops.copy(recv + (size_t)root * count, send, count);
    return 0;
}

}  // namespace karma::engine
