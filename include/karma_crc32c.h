/* include/karma_crc32c.h -- C ABI of the MI355X CRC-32C engine (libkarma_crc32c.so).
 *
 * Plain C: pointers, sizes and integer status codes; no HIP, torch or C++
 * types.  Streams are passed as `karma_stream_t` (a hipStream_t cast to
 * void*, NULL = the default stream).  Device-pointer ("d_") entry points are
 * stream-ordered and asynchronous: they enqueue work on `stream` and return;
 * the caller synchronises.  Host-pointer ("h_") entry points are synchronous.
 *
 * Reference interfaces each entry point replaces:
 *   karma_crc32c_extend_host        crc32c::Extend        karma-util/crc32c.h:16, crc32c.cc:275-376
 *   karma_crc32c_batch_fixed        crc32c::Value per record, as called by
 *                                   segment_file::append_record  karma-store/segment_file.cc:22
 *   karma_crc32c_batch_ragged       crc32c::Value per payload, as called by
 *                                   wal::scan_record             karma-store/wal.cc:60
 *   karma_crc32c_stream             crc32c::Extend over one long buffer (a 64 MiB segment image)
 *   karma_crc32c_*_sharded / gather the same, records sharded over GPUs, CRCs gathered over RCCL
 *   karma_wal_append_batch          sivir::build_sqe + segment_file::append_record   sivir.cc:276-317
 *   karma_wal_replay                sivir::open's wal::scan_record loop              sivir.cc:31-41, wal.cc:34-87
 *   karma_wal_replay_multi          the same over several devices of one process
 *   karma_crc32c_*_host_multi       sivir::build_sqe's batch over several devices    sivir.cc:276-317
 *   karma_wal_replay_dir            wal::load_from_path + the same loop              wal.cc:9-27
 *   karma_kfp_encode_batch          transport::frame::encode                         frame.cc:41-60
 *   karma_kfp_parse_batch           connection::read_frame's frame::parse loop       connection.cc:20-27, frame.cc:62-130
 *
 * Errors: 0 = success, negative = KARMA_E_* below.  No entry point throws.
 * There is no CPU fallback behind the device entry points: without a usable
 * MI355X they return KARMA_E_NO_DEVICE.
 */
#ifndef KARMA_CRC32C_H_
#define KARMA_CRC32C_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define KARMA_CRC32C_ABI_VERSION 1

#define KARMA_OK 0
#define KARMA_E_INVALID (-1)    /* bad argument (null pointer with n > 0, misuse) */
#define KARMA_E_NO_DEVICE (-2)  /* no HIP device / runtime unavailable */
#define KARMA_E_HIP (-3)        /* a HIP runtime call failed */
#define KARMA_E_NOMEM (-4)      /* device or host allocation failed */
#define KARMA_E_RCCL (-5)       /* an RCCL call failed */
#define KARMA_E_IO (-6)         /* reading a file failed (karma_wal_replay_dir) */

typedef void* karma_stream_t;         /* hipStream_t */
typedef struct karma_comm* karma_comm_t;
#define KARMA_UNIQUE_ID_BYTES 128     /* == sizeof(ncclUniqueId) */

int karma_crc32c_abi_version(void);
const char* karma_crc32c_strerror(int status);
/* Thread-local detail of the last failure (HIP/RCCL error string), or "". */
const char* karma_crc32c_last_error(void);

/* ---- host, single buffer ------------------------------------------------- */
/* crc32c::Extend(init_crc, data, n); total, never fails. */
uint32_t karma_crc32c_extend_host(uint32_t init_crc, const void* data, size_t n);
/* The same through the portable slicing-by-8 path only (the default path uses
 * the SSE4.2 CRC32 instruction when present); tests compare the two. */
uint32_t karma_crc32c_extend_host_portable(uint32_t init_crc, const void* data, size_t n);
/* CRC-32C of A || B from crc_a = CRC(A), crc_b = CRC(B) and len_b = |B| (host, GF(2)). */
uint32_t karma_crc32c_combine(uint32_t crc_a, uint32_t crc_b, uint64_t len_b);

/* ---- device-resident batches (stream-ordered) ---------------------------- */
/* d_out[r] = Extend(init_r, d_data + r*rec_bytes, rec_bytes), r < n_rec,
 * init_r = d_init ? d_init[r] : init.  Any rec_bytes and alignment. */
int karma_crc32c_batch_fixed(const void* d_data, size_t rec_bytes, size_t n_rec, const uint32_t* d_init,
                             uint32_t init, uint32_t* d_out, karma_stream_t stream);

/* d_out[r] = Extend(init_r, d_arena + d_off[r], d_len[r]).  Records may be
 * unaligned, empty, in any order and may overlap.  total_len sizes the unit
 * table: pass sum(d_len) (or any upper bound) to stay fully asynchronous;
 * pass 0 when unknown and the call reads the unit count back (one host sync).
 * A total_len below sum(d_len) is not an error and never changes a result: the
 * records whose units do not fit the table are checksummed one lane each.
 * Graph capture: a call with total_len > 0 enqueues kernels only, so it may be
 * captured in a hipGraph and the graph replayed any number of times (the plan's
 * block counter and look-back tags live on the device), with new bytes and
 * lengths in the same buffers as long as sum(d_len) stays <= total_len.  Make one
 * uncaptured call of that size on the stream first (it allocates the stream's
 * workspace; a capture cannot).  Per-stream state is per calling thread for
 * hipStreamPerThread. */
int karma_crc32c_batch_ragged(const void* d_arena, const uint64_t* d_off, const uint32_t* d_len, size_t n_rec,
                              size_t total_len, const uint32_t* d_init, uint32_t init, uint32_t* d_out,
                              karma_stream_t stream);

/* The same with an upper bound of every d_len[r] (0 = unknown).  With max_len <= 1 KiB
 * (WAL records, KFP frames) each record is checksummed by one small group of lanes (4)
 * with no planning kernels.  The result is exact whatever the bound: a wrong one costs
 * balance. */
int karma_crc32c_batch_ragged_bounded(const void* d_arena, const uint64_t* d_off, const uint32_t* d_len, size_t n_rec,
                                      size_t total_len, uint32_t max_len, const uint32_t* d_init, uint32_t init,
                                      uint32_t* d_out, karma_stream_t stream);

/* *d_out = Extend(init, d_data, n): one long buffer split over the whole GPU
 * and folded back with a polynomial combine.
 * Forward progress: this call (and karma_crc32c_batch_fixed with n_rec == 1 and a record
 * split over more than 8 units) is ONE kernel whose last workgroup waits on the other
 * workgroups' tagged wave states and folds them.  It assumes that every workgroup of the grid
 * is eventually scheduled while the last one waits: the grid has at most one workgroup per
 * compute unit and the hardware dispatches workgroups in index order, so the ones waited for
 * were dispatched first.  Concurrent kernels on other streams only delay them (they are
 * tested concurrently with other segment scans and ragged batches); do not launch it where a
 * co-resident persistent kernel could hold every compute unit forever. */
int karma_crc32c_stream(uint32_t init, const void* d_data, size_t n, uint32_t* d_out, karma_stream_t stream);

/* ---- resource lifetime ---------------------------------------------------
 * crc32c::Extend (karma-util/crc32c.h) allocates nothing.  The device batch entry points keep,
 * per (device, stream), what their kernels point at: a workspace sized for the largest batch seen
 * on the stream, the ragged plan's look-back words and the single-record combine's words.  For
 * hipStreamPerThread the state is per calling thread.  An outgrown buffer is freed once its
 * stream has drained, unless a hipGraph was ever captured on that stream (a captured call keeps
 * its address): then it is kept until karma_crc32c_trim.  The host-memory, WAL and KFP entry
 * points keep per-device streams, device buffers and pinned staging.  Nothing else is kept.
 *
 * karma_crc32c_release_stream  waits for `stream` and frees its state (before destroying a
 *                              stream, or when a thread is done with hipStreamPerThread).  Do
 *                              not call it while a graph captured on that stream may still be
 *                              launched, nor while the stream is capturing (KARMA_E_INVALID).
 * karma_crc32c_trim            waits for the device and frees what no live stream holds: the
 *                              state of exited threads' hipStreamPerThread, the outgrown buffers
 *                              (unless a graph hold is active) and the per-device contexts of the
 *                              host, WAL and KFP entry points (recreated by their next call).
 * karma_crc32c_graph_hold      counts the captured graphs a caller keeps (delta +1 / -1); while
 *                              the count is above 0, trim keeps outgrown buffers and the state of
 *                              exited threads whose hipStreamPerThread saw a capture.  Returns the
 *                              count (>= 0) or a KARMA_E_* status.
 * device: the device index, or -1 for the calling thread's current device. */
int karma_crc32c_release_stream(int device, karma_stream_t stream);
int karma_crc32c_trim(int device);
int karma_crc32c_graph_hold(int device, int delta);
/* The per-(device, stream) states the library holds, over all devices (live streams' states;
 * not the exited threads' states a trim has yet to free).  For leak checks: after trim the
 * library's own streams hold none. */
int karma_crc32c_stream_states(void);

/* ---- host-memory batches (synchronous; H2D, kernel, D2H overlapped) ------- */
int karma_crc32c_batch_fixed_host(const void* h_data, size_t rec_bytes, size_t n_rec, uint32_t init,
                                  uint32_t* h_out, int device);
int karma_crc32c_batch_ragged_host(const void* h_arena, size_t arena_bytes, const uint64_t* h_off,
                                   const uint32_t* h_len, size_t n_rec, uint32_t init, uint32_t* h_out, int device);

/* The same over several devices of this process (one host thread per device, each device's
 * PCIe link, staging and streams at once): the records are cut into contiguous ranges -- equal
 * counts (fixed) or equal bytes (ragged) -- one per listed device, and the CRCs written into
 * h_out in record order.  A device may be listed more than once (its shares then run one
 * after the other).  Synchronous; any share's failure fails the call. */
int karma_crc32c_batch_fixed_host_multi(const void* h_data, size_t rec_bytes, size_t n_rec, uint32_t init,
                                        uint32_t* h_out, const int* devices, int n_dev);
int karma_crc32c_batch_ragged_host_multi(const void* h_arena, size_t arena_bytes, const uint64_t* h_off,
                                         const uint32_t* h_len, size_t n_rec, uint32_t init, uint32_t* h_out,
                                         const int* devices, int n_dev);

/* ---- multi-GPU: one process per GPU, RCCL over xGMI ---------------------- */
int karma_crc32c_get_unique_id(void* uid, size_t uid_bytes);
int karma_crc32c_comm_init(karma_comm_t* comm, int nranks, const void* uid, int rank);
int karma_crc32c_comm_destroy(karma_comm_t comm);
/* *nranks = the ranks RCCL itself reports for the communicator (ncclCommCount). */
int karma_crc32c_comm_count(karma_comm_t comm, int* nranks);
/* d_recv (root only, count*nranks words) <- every rank's d_send (count words), rank order. */
int karma_crc32c_gather_u32(karma_comm_t comm, const uint32_t* d_send, size_t count, uint32_t* d_recv, int root,
                            karma_stream_t stream);
/* This rank's shard of a fixed-size batch, then the gather of its CRCs to root. */
int karma_crc32c_batch_fixed_sharded(karma_comm_t comm, const void* d_local, size_t rec_bytes, size_t n_local,
                                     uint32_t init, uint32_t* d_local_out, uint32_t* d_all_out, int root,
                                     karma_stream_t stream);

/* ---- WAL segment images (karma-store framing) ------------------------------
 * Record = [crc u32 LE = Value(payload)][len<<8 | type u32 LE][payload]
 * (segment_file.cc:21-31, common.h:11); type 1 = padding to the segment end
 * ('0' bytes, crc 0; segment_file.cc:33-49).  The WAL image is a host buffer of
 * wal_bytes = k * seg_bytes (segments back to back, WAL offset = byte offset). */
#define KARMA_WAL_END 0      /* replay walked past the last segment */
#define KARMA_WAL_CORRUPT 1  /* stopped where wal.cc logs "Corrupt record" */
#define KARMA_WAL_BAD_TYPE 2 /* stopped at a record type other than 0 / 1 */

/* Batched append (sivir::build_sqe + segment_file::append_record / append_footer):
 * frame payloads i = 0..n-1 (h_src + h_src_off[i], h_len[i]) at WAL offset *h_cursor,
 * closing a segment with a footer when a record does not fit (can_hold).  The payload
 * CRCs are computed on the GPU, block by block while the host frames (the payloads are
 * streamed through the library's pinned staging; the caller's memory is never
 * page-locked).  Updates *h_cursor, writes the header offset of record i to
 * h_rec_off[i] (optional) and the number framed to *h_n_framed (records that do not fit
 * in the image are left out).  Batches of more than 1 GiB of payload are framed in
 * passes; on an error *h_cursor / *h_n_framed cover the passes completed, and bytes
 * past *h_cursor may have been written (without valid CRC fields). */
int karma_wal_append_batch(const void* h_src, const uint64_t* h_src_off, const uint32_t* h_len, size_t n,
                           void* h_wal, size_t wal_bytes, size_t seg_bytes, uint64_t* h_cursor, uint64_t* h_rec_off,
                           size_t* h_n_framed, int device);

/* Batched replay (sivir::open's wal::scan_record loop, wal.cc:34-87) from WAL offset
 * `start`, entirely on the device: segment-parallel header walk (sub-range walkers
 * stitched along the real chain when there are few segments), all payload CRCs in one
 * GPU batch, first mismatch.  A replay whose first record (at `start`) has a payload of at
 * most 1 KiB first tries the uniform-stride pass: the segments read as records of that
 * size, each header and CRC checked in one batch with no walk; its result is used only when
 * it is scan_record's (nothing before replay's stop breaks the stride), otherwise the walk
 * decides.  The image is d_wal when the caller already holds a device
 * copy (h_wal may then be NULL), else h_wal is streamed into HBM (pinned staging, no
 * page-locking of the caller's buffer).  seg_bytes < 2^31.
 * Outputs: *h_n_records type-0 records accepted, their header offsets in h_rec_off
 * (optional, up to rec_cap), *h_stop the WAL offset where replay stops (the writer's
 * resume point; up to 4 bytes past wal_bytes when an accepted size-0 record ends the image,
 * and such a stop is accepted back as `start`: it replays nothing), *h_status KARMA_WAL_*.  Keeps the reference's size-0 quirk (the CRC
 * of an empty type-0 record is taken over the stale 4-byte len/type word). */
int karma_wal_replay(const void* h_wal, const void* d_wal, size_t wal_bytes, size_t seg_bytes, uint64_t start,
                     uint64_t* h_n_records, uint64_t* h_stop, int* h_status, uint64_t* h_rec_off, size_t rec_cap,
                     int device);

/* karma_wal_replay of a host image over several devices: the segments from start's segment on
 * are cut into contiguous ranges, one per listed device, replayed at once (each range streamed
 * over its own device's link), and merged in WAL order: a range's records count while every
 * range before it ended cleanly at its last segment's end, as the one-device replay would have
 * walked on.  When an accepted size-0 record carries the chain 1-4 bytes past a range's end, the
 * next range alone is replayed again from there, on its own device (one extra range replay per
 * such spill).  Same outputs as karma_wal_replay. */
int karma_wal_replay_multi(const void* h_wal, size_t wal_bytes, size_t seg_bytes, uint64_t start, uint64_t* h_n_records,
                           uint64_t* h_stop, int* h_status, uint64_t* h_rec_off, size_t rec_cap, const int* devices,
                           int n_dev);

/* Plan overrides of karma_wal_replay_tuned.  Every setting gives the same result (the
 * replay is exact whatever the plan); they exist for tests and tuning.  Zero = the
 * planner's choice. */
#define KARMA_WAL_CRC_PLAN 0    /* the walk, then one small-record batch over the gathered lists when every
                                   payload <= 1 KiB (LDS-staged up to 183 B, 4-lane groups above), else the
                                   unit plan */
#define KARMA_WAL_CRC_DIRECT 1  /* always the small-record batch */
#define KARMA_WAL_CRC_UNITS 2   /* always the unit plan (karma_crc32c_batch_ragged) */
#define KARMA_WAL_CRC_SEPARATE 3 /* = PLAN (kept for callers of round 2's ABI) */
#define KARMA_WAL_CRC_INLINE 4  /* as PLAN, but payloads <= 1 KiB checksummed inside the walk kernel
                                   (k_wal_walk_crc: faster when the image is cache-resident, slower from HBM) */
typedef struct karma_wal_tuning {
    uint64_t walk_sub_bytes; /* header-walk sub-range size, rounded down to a 4 KiB multiple (>= 4 KiB);
                                >= seg_bytes: one walker per segment; 0 = planned (non-zero also
                                skips the uniform-stride pass: always the walk) */
    int32_t crc_batch;       /* KARMA_WAL_CRC_* */
    int32_t reserved;        /* 0 */
} karma_wal_tuning;
/* karma_wal_replay with plan overrides (tuning may be NULL = karma_wal_replay). */
int karma_wal_replay_tuned(const void* h_wal, const void* d_wal, size_t wal_bytes, size_t seg_bytes, uint64_t start,
                           uint64_t* h_n_records, uint64_t* h_stop, int* h_status, uint64_t* h_rec_off, size_t rec_cap,
                           int device, const karma_wal_tuning* tuning);

/* Replay of a segment directory (wal::load_from_path + sivir::open, wal.cc:9-27): the
 * regular files of `dir` named by the decimal WAL offset of their first byte, equal
 * sizes (seg_bytes, or 0 = the first file's size), no gaps.  The files are read by the
 * staging threads straight into pinned buffers and streamed into HBM; then the same
 * device replay as karma_wal_replay.  `start`, *h_stop and h_rec_off are WAL offsets;
 * *h_base = the first segment's offset.  An empty directory replays nothing (END).
 * KARMA_E_IO when a file cannot be opened or read. */
int karma_wal_replay_dir(const char* dir, size_t seg_bytes, uint64_t start, uint64_t* h_base, uint64_t* h_n_records,
                         uint64_t* h_stop, int* h_status, uint64_t* h_rec_off, size_t rec_cap, int device);

/* ---- KFP frames (karma-transport) ------------------------------------------
 * Frame (frame.cc:29-60): [frame_length u32][magic u8 = 123][operation_code i16][flag u8]
 * [seq u32][header_length u32][header][payload][crc u32], integers little-endian,
 * frame_length = 16 + header + payload + 4, crc = Extend(Value(header), payload). */
#define KARMA_KFP_MAGIC 123                 /* frame.h:20 */
#define KARMA_KFP_FIXED_HEADER 16           /* frame.h:21 */
#define KARMA_KFP_MAX_FRAME (4096u * 128u)  /* frame.h:23 */
#define KARMA_KFP_OK 0              /* every complete frame parsed; the rest is an incomplete frame */
#define KARMA_KFP_BAD_SIZE 1        /* frame_length > MAX_FRAME_SIZE        (frame.cc:70-73 throws) */
#define KARMA_KFP_BAD_MAGIC 2       /* magic != 123                          (frame.cc:86-89 throws) */
#define KARMA_KFP_BAD_HEADER_LEN 3  /* header_length > frame_length - 20     (frame.cc:101-104 throws) */
#define KARMA_KFP_BAD_CRC 4         /* stored crc != computed                (frame.cc:125-128 throws) */
#define KARMA_KFP_BAD_LENGTH 5      /* frame_length < 20: undefined behaviour in the reference
                                       (unsigned wrap at frame.cc:101,111); refused here */

/* Encode frames i = 0..n-1 back to back into h_out (frame::encode): header bytes
 * h_hdr + h_hdr_off[i] (h_hdr_len[i]), payload h_pay + h_pay_off[i] (h_pay_len[i]),
 * operation code, flag and seq per frame.  The CRCs of all frames come from one GPU
 * batch.  Frames that do not fit out_bytes are left for the next call: *h_n_encoded
 * frames, *h_bytes bytes written; h_frame_off[i] (optional) = offset of frame i. */
int karma_kfp_encode_batch(const void* h_hdr, const uint64_t* h_hdr_off, const uint32_t* h_hdr_len,
                           const void* h_pay, const uint64_t* h_pay_off, const uint32_t* h_pay_len,
                           const int16_t* h_op, const uint8_t* h_flag, const uint32_t* h_seq, size_t n, void* h_out,
                           size_t out_bytes, uint64_t* h_frame_off, size_t* h_n_encoded, uint64_t* h_bytes,
                           int device);

/* Parse a receive buffer the way connection::read_frame drains it: frame::parse at the
 * cursor, advance by frame_length, repeat (at most max_frames).  *h_n_frames frames were
 * accepted (offsets in h_frame_off, optional, capacity max_frames); *h_consumed = bytes
 * they occupy = where parsing stopped; *h_status = KARMA_KFP_*.  All frame CRCs are
 * verified in one GPU batch, from d_buf when a device copy of the buffer is given. */
int karma_kfp_parse_batch(const void* h_buf, const void* d_buf, size_t buf_bytes, size_t max_frames,
                          uint64_t* h_frame_off, size_t* h_n_frames, uint64_t* h_consumed, int* h_status,
                          int device);

/* ---- synthetic data and probes (bench / tests) ---------------------------- */
/* d_dst[i] = byte (first_byte + i) of the little-endian splitmix64 stream of
 * `seed` (word j = mix(seed + (j+1)*0x9E3779B97F4A7C15)); first_byte % 8 == 0. */
int karma_fill_splitmix64(void* d_dst, size_t n_bytes, uint64_t seed, uint64_t first_byte, karma_stream_t stream);
/* Read-only streaming probe (xor of all 16-byte words) for the achievable HBM rate. */
int karma_stream_probe(const void* d_src, size_t n_bytes, uint32_t* d_out, karma_stream_t stream);
/* Number of compute units of the current device (grid sizing, reporting). */
int karma_device_cu_count(void);

/* Instrumentation: arm two hipEvent_t (created by the caller with timing enabled).  The next
 * batch call on this thread records them on its stream immediately before and after its
 * dominant kernel (the units kernel: k_units_fixed / k_units_ragged), so a caller can time that
 * kernel alone.  Passing (NULL, NULL) disarms. */
int karma_crc32c_time_next_units(void* start_event, void* stop_event);

#ifdef __cplusplus
}
#endif

#endif /* KARMA_CRC32C_H_ */
