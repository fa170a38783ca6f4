// karma_amd/csrc/host_stage.h -- host -> HBM uploads through persistent pinned
// staging buffers (library-internal).
//
// The host entry points (karma_crc32c_batch_*_host, karma_wal_*, karma_kfp_*)
// take pageable caller memory.  It is never page-locked per call
// (hipHostRegister / hipHostUnregister churn on caller pages that share pages
// with other heap objects is what round 1's intermittent illegal-address fault
// pointed at): worker threads copy it into pinned buffers owned
// by the library, and each worker DMAs its buffers on its own stream, so the
// memcpy of one chunk overlaps the DMA of the previous and several copies run
// at once.
#pragma once
#include <hip/hip_runtime_api.h>

#include <cstddef>
#include <cstdint>
#include <functional>

namespace karma::engine {

// Fills dst with the source bytes [off, off + n) (offsets relative to the upload's source).
using HostFill = std::function<int(uint8_t* dst, uint64_t off, size_t n)>;

// Streams source bytes [src_off, src_off + bytes) into d_dst (device `dev`, current on
// the calling thread) and returns when every DMA has completed.  One upload at a time
// per device (a per-device lock); the pinned buffers persist across calls.
int staged_upload(int dev, void* d_dst, const HostFill& fill, uint64_t src_off, size_t bytes);

// staged_upload of a plain host buffer.
int staged_copy(int dev, void* d_dst, const void* h_src, size_t bytes);

// True when h is page-locked host memory the device can DMA from directly
// (hipHostMalloc'd or registered by its owner).
bool host_is_pinned(const void* h);
// True when [h, h + bytes) lies inside one page-locked host allocation.
bool host_range_pinned(const void* h, size_t bytes);

// karma_crc32c_trim's per-module releases (engine.h); trim_host_contexts calls them all.
int trim_replay_ctx(int dev);
int trim_host_batch_ctx(int dev);
int trim_append_ctx(int dev);
int trim_kfp_ctx(int dev);
int trim_stage(int dev);
int trim_host_contexts(int dev);

// body(t) for t in [0, n) on n std::threads (n small: the host stages of a call).
void run_threads(int n, const std::function<void(int)>& body);

// body(t) for t in [0, n): t = 0 on the calling thread, the others on the library's
// persistent host threads (created on first use and parked between calls, so a call
// pays a wake-up, not n thread creations).  Returns when every body has returned.
// n is capped at kPoolThreads + 1.  Calls from several threads are serialised.
constexpr int kPoolThreads = 15;
void run_pool(int n, const std::function<void(int)>& body);

}  // namespace karma::engine
