// karma_amd/csrc/engine.h -- internal interface between the C ABI (capi.cc)
// and the gfx950 kernels (crc32c_kernels.hip).  Not installed; the public
// surface is include/karma_crc32c.h and include/karma-util/crc32c.h.
#pragma once
#include <hip/hip_runtime_api.h>

#include <cstddef>
#include <cstdint>
#include <vector>

namespace karma {
namespace engine {

// ---- geometry of the streaming kernel -----------------------
constexpr int kGroupLanes = 8;                 // lanes that share one unit
constexpr int kChunk = 16 * kGroupLanes;       // bytes a group consumes per step (S)
constexpr int kBlockThreads = 1024;            // one workgroup per CU
constexpr int kWavesPerBlock = kBlockThreads / 64;
constexpr int kGroupsPerWave = 64 / kGroupLanes;
constexpr int kStgWaves = 7;  // k_ragged_staged: one 448-thread workgroup per CU (LDS-bound)
constexpr int kStgWaves8 = 10;  // ... its plain-stage form on the 8-copy stride image (tools build A/B)
// Consecutive payloads up to this length (with 8-byte WAL headers between them) put 64 records
// in one wave's 12 KiB stage (crc_device.h kStgBytes: (12288 - 64) / 64 - 8).
constexpr uint32_t kStgGateLen = 183;
#ifndef KARMA_RAGGED_UNIT
#define KARMA_RAGGED_UNIT 8192  // a build-time A/B knob (tools/ragged_study.py over builds with -DKARMA_RAGGED_UNIT=...)
#endif
constexpr uint64_t kDefaultUnit = KARMA_RAGGED_UNIT;  // unit size for ragged batches
// WAL images up to this take replay's device-planned path (wal.cc); wal_device.hip's fused plan
// sums its candidate counts in 32 bits on that bound (static_assert there).
constexpr uint64_t kDevicePlanMax = uint64_t(256) << 20;

// ---- table blob of the streaming kernel (uint32 words) ---------------------
constexpr int kBlobStride = 0;     // Z_S slicing tables, 4 x 256
constexpr int kBlobZ4 = 1024;      // Z_4   (in-lane fold)
constexpr int kBlobZ16 = 2048;     // Z_16  (group tree, level 0)
constexpr int kBlobZ32 = 3072;     // Z_32  (level 1)
constexpr int kBlobZ64 = 4096;     // Z_64  (level 2)
constexpr int kBlobT8 = 5120;      // byte table (one zero byte, low byte index)
constexpr int kBlobWords = 5376;

// ---- table blob of the combine kernels --------------------------------------
// maps Z_{D * 2^k}, k = 0..6 (k = 6 is the Horner step of 64 states), Z4 and
// the byte table (head/tail steps), then Z_{16 * 2^i}, i = 0..7, which
// compose Z_L for any L = 16n < 4096 (the short last unit of a ragged record).
constexpr int kCombMaps = 7;
constexpr int kCombZ4 = kCombMaps * 1024;
constexpr int kCombT8 = kCombZ4 + 1024;
constexpr int kCombCoreWords = kCombT8 + 256;  // what the fixed combine and the head steps need
constexpr int kCombSmall = kCombT8 + 1024;
#ifndef KARMA_RAGGED_DYN_SHIFT
#define KARMA_RAGGED_DYN_SHIFT 3  // RaggedArgs::dyn_shift (a build-time A/B knob; the tools build's KARMA_RAGGED_DYN)
#endif
// The dynamic tail's size (RaggedArgs::dyn_shift): at most kDynMaxSteps steps (~70 us of the whole
// GPU streaming), taken in chunks of 16 (one per workgroup grab); a workgroup's chunk bases live in
// kDynChunks LDS words, enough for every chunk (the static part ends on a whole round, up to
// nwaves steps earlier than nws - kDynMaxSteps).
constexpr uint32_t kDynMaxSteps = 8192, kDynChunks = 1024;
constexpr int kCombSmallMaps = KARMA_RAGGED_UNIT > 8192 ? 10 : 9;  // Z_16n, n < 2^maps (>= a ragged unit / 16)
// (a partial last unit is shorter than the unit: n = its length / 16 < unit / 16)
static_assert((16ull << kCombSmallMaps) >= (unsigned long long)KARMA_RAGGED_UNIT,
              "finalize's last-unit maps Z_16n must reach a whole unit");
// Z_1^-1, Z_2^-1, Z_4^-1, Z_8^-1 (the inverse zero-byte maps): ragged records are stepped over
// their whole 16-byte blocks with the bytes outside the record masked to zero; the plan moves ~init
// back over the 1-3 masked bytes before the record's start, finalize takes the register back over
// the 0-15 masked bytes after its end.
constexpr int kCombInv = kCombSmall + kCombSmallMaps * 1024;
constexpr int kCombWords = kCombInv + 4 * 1024;
// A unit descriptor's span word: bytes in the low 16 bits; for a record's first unit the masked head
// bytes (the window at us holds h bytes before the record), for its last the masked tail bytes.
constexpr uint32_t kDescSpanMask = 0xffffu, kDescHeadShift = 16, kDescTailShift = 20;
static_assert(KARMA_RAGGED_UNIT < (1u << 16), "a unit's bytes fit the span word's low 16 bits");

// ---- table blob of the one-block combine (k_combine_block) -----------------
// For states of D bytes folded m per thread: Z_D (the in-thread Horner step),
// Z_{mD*2^d} for d = 0..5 (the 64-lane tree), Z_{64mD} (the fold of the 16
// wave results), Z4 and the byte table (the record tail).
constexpr int kBcZD = 0;
constexpr int kBcTree = 1024;
constexpr int kBcWave = 7 * 1024;
constexpr int kBcZ4 = 8 * 1024;
constexpr int kBcT8 = 9 * 1024;
constexpr int kBlockCombWords = 9 * 1024 + 256;
constexpr uint64_t kBlockCombMaxPerThread = 64;  // one launch folds up to 64 Ki states per record

// Host builders (gf2.h): fill a blob for stride kChunk / for unit size D.
void build_stream_blob(uint32_t* out /*kBlobWords*/);
// The same layout with Z_16 as the stride tables: k_ragged_lanes, one record per lane.
void build_lane_blob(uint32_t* out /*kBlobWords*/);
// ... and with Z_64: k_ragged_direct4, one record per group of 4 lanes.
void build_quad_blob(uint32_t* out /*kBlobWords*/);
void build_combine_blob(uint64_t unit_bytes, uint32_t* out /*kCombWords*/);
void build_block_combine_blob(uint64_t unit_bytes, uint64_t per_thread, uint32_t* out /*kBlockCombWords*/);

struct FixedArgs {
    const uint8_t* arena;      // record r at arena + r * rec_bytes
    uint64_t rec_bytes;
    uint64_t n_rec;
    const uint32_t* init;      // per-record init crc, or nullptr -> init_scalar
    uint32_t init_scalar;
    uint64_t unit_bytes;       // multiple of kChunk
    uint64_t units_per_rec;    // k (same for every record)
    uint32_t* out;             // final crc per record (written when k == 1)
    uint32_t* partial;         // per-unit register contributions (k > 1); with comb_maps, one per 8 units
    const uint32_t* blob;      // kBlobWords, device
    const uint32_t* comb_maps; // k % 8 == 0: Z_U, Z_2U, Z_4U (3 x 1024 words): the 8 groups of a
                               // wave fold their 8 consecutive units into one state (else nullptr)
    uint32_t fold_k;           // 2, 4 or 8: k == fold_k units of a record sit in one wave, which folds
                               // them with comb_maps and writes out[] itself (0: not used)
    // Fused record combine (one record, WAVE_COMB; k_units_fixed FUSE): the wave states go out
    // tagged, (tag << 32 | state), as agent-scope atomic stores into partial (as uint64); the
    // grid's last workgroup folds them like k_combine_block with block_blob, waiting on each
    // state's tag, and writes the CRC.  fctl[1] = the last finished call's tag (device-resident,
    // so a captured graph replays correctly; fctl[0]: k_segment_once's arrival tickets when the
    // last-arriving workgroup folds, zero between calls).  nullptr: not fused.
    unsigned long long* fctl;
    const uint32_t* block_blob; // kBlockCombWords (block_comb_blob for D = 8 units, m states per thread)
    uint64_t comb_m;            // states per thread of the fused fold
};

// One unit of a ragged batch: the 16-aligned span [us, us + span) of a record's whole 16-byte
// blocks.  span: bytes (kDescSpanMask), and for the record's first unit the head bytes h masked to
// zero in the window at us (bits kDescHeadShift..+3), for its last unit the tail bytes t masked in
// the window ending at us + span (bits kDescTailShift..+3).  inj is xored into word h / 4 of the
// window at us: for the record's first unit ~init moved back over the h % 4 masked bytes before
// the record (Z_{h%4}^-1(~init), the plan), else 0.
struct UnitDesc {
    uint64_t us;
    uint32_t span;
    uint32_t inj;
};
static_assert(sizeof(UnitDesc) == 16, "one 16-byte load per unit descriptor");

// Ragged batches cut record bodies at absolute unit_bytes boundaries (so full
// units are unit-aligned and every chunk is a whole cache line) and order the
// units for balance: all full units first, in record order, then
// each block's partial first/last units bucketed by chunk count, longest first,
// so the 8 units a wave streams together have (nearly) equal length.
constexpr int kBuckets = (int)(kDefaultUnit / kChunk) + 1;  // chunk counts of a partial unit (index = chunks; 65 for 8 KiB units)
static_assert(kDefaultUnit / kChunk < kBuckets, "a partial unit has at most unit/kChunk chunks");

struct WalSpec;  // the uniform-stride WAL replay's probe result (below)
struct RaggedArgs {
    const uint8_t* arena;
    const uint64_t* off;       // payload offset per record
    const uint32_t* len;       // payload length per record
    uint64_t n_rec;
    const uint32_t* init;
    uint32_t init_scalar;
    uint64_t unit_bytes;       // kDefaultUnit
    uint64_t* fbase;           // n_rec + 2: slot of the record's first full unit;
                               //   [n_rec] = total units, [n_rec+1] = full units
    uint64_t* pslot;           // 2 * n_rec: slots of the record's partial first / last unit
    uint64_t* block_sums;      // per scan block: full-unit offset
    uint64_t* block_psums;     // per scan block: partial units (k_ragged_scan)
    // Single-pass plan (k_ragged_plan): decoupled look-back over per-block status words.
    // lb[0] counts the blocks that started (plan-block ids in start order); lb[1 + b] =
    // seq << 42 | flag << 40 | value (flag 1: block b's own full-unit count, 2: the full units
    // of blocks 0..b); lbp[b] the same for partial units.  The call's tag seq (1 .. lb_seq_max
    // - 1) and the counter live on the device (lb_ctl), so that a call replayed from a captured
    // graph gets fresh ids and a fresh tag: the plan takes seq = lb_ctl[0] + 1 and records it
    // in lb_ctl[1]; k_ragged_finalize (the call's last kernel) resets lb[0] and moves lb_ctl[0]
    // to seq, or, at lb_seq_max, clears the lb_words status words and restarts the tags at 1.
    unsigned long long* lb;
    unsigned long long* lbp;   // the same for the blocks' partial unit counts
    unsigned long long* lb_ctl;  // [0] the last finished call's tag, [1] the running call's, [2] dyn steps taken
    uint64_t lb_words;         // status words after lb[0] (both arrays)
    uint32_t lb_seq_max;       // 2^22 (the tools build lowers it to test the wrap)
    // k_units_ragged: the last nws >> dyn_shift wave-steps (0: none) are taken from a global
    // counter (lb_ctl[2], reset by k_ragged_finalize) instead of each workgroup's static share
    uint32_t dyn_shift;
    UnitDesc* desc;            // unit_cap entries
    uint64_t unit_cap;         // capacity of desc / partial
    uint64_t part_base;        // first slot of the partial units (full units take [0, part_base))
    uint32_t* out;
    uint32_t* partial;         // register contribution per unit slot
    const uint32_t* blob;      // stream blob (kBlobWords)
    const uint32_t* comb_blob; // kCombWords for unit_bytes
    uintptr_t kb_lo, kb_hi;    // bounds build only: the arena's allocation (bounds.h); else 0
    // Device-sized batches (WAL replay's small-record path): when n_dev is set the kernel reads
    // n_rec there, and does nothing unless gate_min <= *gate_len <= gate_max.  (k_ragged_direct4 and
// k_ragged_staged_pipe only.)
    const uint64_t* n_dev;
    const uint32_t* gate_len;
    uint32_t gate_max;
    uint32_t gate_min;         // ... and *gate_len >= gate_min (the staged and 4-lane kernels split the range)
    // ... and, when cmp_stored is set, the kernel also compares each record's CRC with
    // cmp_stored[r] (records of length 0 excepted) and keeps the first mismatch in *cmp_bad.
    const uint32_t* cmp_stored;
    unsigned long long* cmp_bad;
    // k_ragged_staged_pipe: set to 1 when a batch's records start on few LDS banks (the skewed
    // stage's case), whichever stage the kernel has; nullptr: not reported
    uint32_t* stage_skew_seen;
    // the uniform-stride WAL replay (k_ragged_staged_pipe's SPEC form, wal.cc): the records are
    // the slots of spec_nseg segments of spec_seg bytes at arena - 8 (WalSpec), not lists;
    // nullptr otherwise
    WalSpec* spec;
    uint64_t spec_nseg, spec_seg;
    uint64_t spec_first;                // where replay enters segment 0 (its first slot)
    uint64_t spec_base0, spec_wal_end;  // WAL offsets of the image start and end (the summary's)
    struct WalSummary* spec_out;        // page-locked: the pass's summary (its last workgroup writes it)
};

// Instrumentation (capi.cc): events armed by karma_crc32c_time_next_units are
// recorded on `s` immediately around the next units kernel launched by this thread.
#ifdef KARMA_AB
hipError_t set_wave_log_ragged(void* p, uint64_t cap);  // wavelog.h (tools build)
hipError_t set_wave_log_fixed(void* p, uint64_t cap);
hipError_t set_seg_log(void* p);  // k_segment_once's per-workgroup stamps (8 words each)
hipError_t set_plan_log(void* p);  // k_ragged_plan's / k_ragged_finalize's (8 words per workgroup)
#endif
void units_timer_begin(hipStream_t s);
void units_timer_end(hipStream_t s);

// Launchers (stream-ordered, no allocation, no synchronisation).
hipError_t launch_fixed(const FixedArgs& a, int grid_blocks, hipStream_t s);
// One record streamed one wave-step per wave (k_segment_once: a segment scan up to grid x 128
// units of <= 2 KiB): units_per_rec = 128 x grid_blocks, comb_maps = the unit's combine blob,
// block_blob = the combine blob of 128 units, fctl / partial = the fused words.
// arrive: the last-arriving workgroup folds (a ticket counter in fctl[0]), not the grid's last one.
hipError_t launch_segment_once(const FixedArgs& a, int grid_blocks, hipStream_t s, bool arrive);
// Its largest unit: 16 chunk loads per lane, so 2 KiB when the body's end (16-aligned) sits on the
// 128-byte grid, else 1,920 bytes (units are end-aligned: one then spans a chunk more).
inline uint64_t segment_once_max_unit(const uint8_t* rec, uint64_t rec_bytes) {
    const uintptr_t b = (reinterpret_cast<uintptr_t>(rec) + rec_bytes) & ~uintptr_t(15);
    return b % 128 == 0 ? 16 * 128 : 15 * 128;
}
// One combine level for the fixed layout: k_in states per record -> k_out = ceil(k_in / 64).
hipError_t launch_combine_fixed(const FixedArgs& a, const uint32_t* in_states, uint64_t k_in, uint32_t* out_states,
                                uint64_t k_out, const uint32_t* comb_blob, hipStream_t s);
// All of a record's k_in states (D bytes each, end-aligned) -> its CRC in one
// launch: one 1024-thread block per record, m = ceil(k_in / 1024) states per thread.
hipError_t launch_combine_block(const FixedArgs& a, const uint32_t* in_states, uint64_t k_in, uint64_t m,
                                const uint32_t* block_blob, hipStream_t s);
#ifndef KARMA_SCAN_BLOCK
#define KARMA_SCAN_BLOCK 1024  // records per scan/desc block: a build-time A/B knob (tools/scan_block_ab.sh)
#endif
constexpr int kScanBlock = KARMA_SCAN_BLOCK;
inline uint64_t ragged_scan_blocks(uint64_t n_rec) { return (n_rec + kScanBlock - 1) / kScanBlock; }
// Ragged: the plan (one pass: unit slots, descriptors and the entering registers; total
// units at fbase[n_rec]), then the unit kernel and the per-record finalize.
// launch_ragged_scan only counts units (block_sums / block_psums), for callers that must size
// the unit table first.
hipError_t launch_ragged_scan(const RaggedArgs& a, hipStream_t s);
hipError_t launch_ragged_main(const RaggedArgs& a, int grid_blocks, hipStream_t s);
// One record per group of 4 lanes, no plan kernels (uses arena, off, len, n_rec, init, out, and
// blob = build_quad_blob's; the tools build's KARMA_DIRECT_VARIANT=20 runs the LDS-staged
// kernel instead, with blob = build_lane_blob's).
hipError_t launch_ragged_direct(const RaggedArgs& a, int grid_blocks, hipStream_t s);
// k_ragged_direct4 with a device-sized batch (a.n_dev / a.gate_len set): WAL replay's
// device-planned path, whatever the tools build's variant.
hipError_t launch_ragged_staged_dev(const RaggedArgs& a, int grid_blocks, hipStream_t s, bool skew = true);
hipError_t launch_ragged_direct_dev(const RaggedArgs& a, int grid_blocks, hipStream_t s);
// Library-internal entry (capi.cc) for callers that know every record is small
// (WAL replay): CRCs of arena[off[r], off[r] + len[r]) with Value's init.
int ragged_small_batch(const void* d_arena, const uint64_t* d_off, const uint32_t* d_len, size_t n_rec,
                       uint32_t* d_out, hipStream_t s);
// The 4-lane small-record kernel's table blob on the current device (k_wal_walk_crc's tables).
int device_quad_blob(int dev, const uint32_t** out);
// The staged kernels' blob (Z_16 stride tables: k_ragged_staged, k_wal_list_crc).
int device_lane_blob(int dev, const uint32_t** out);
// The same as ragged_small_batch with the record count in device memory (*d_n, at most n_cap
// records), run only when *d_gate_len <= gate_max (else the kernels do nothing).  `which` picks
// the launches: kSmallBoth = the LDS-staged kernel up to kStgGateLen and the 4-lane kernel above
// it (one of the two returns at once); kSmallStaged / kSmallDirect = only that one (the caller
// checks the batch's largest payload afterwards and runs the batch again when it was not
// covered: small_batch_covers).  With d_stored set it is also the CRC check: the first record
// whose CRC differs from d_stored[r] (length 0 excepted) goes to *d_first_bad (atomicMin).
enum SmallWhich : int { kSmallBoth = 0, kSmallStaged = 1, kSmallDirect = 2 };
inline bool small_batch_covers(int which, uint32_t max_len, uint32_t gate_max) {
    if (max_len > gate_max) return false;
    return which == kSmallBoth || (which == kSmallStaged ? max_len <= kStgGateLen : max_len > kStgGateLen);
}
int ragged_small_batch_dev(const void* d_arena, const uint64_t* d_off, const uint32_t* d_len, const uint64_t* d_n,
                           uint64_t n_cap, const uint32_t* d_gate_len, uint32_t gate_max, uint32_t* d_out,
                           const uint32_t* d_stored, uint64_t* d_first_bad, hipStream_t s, int which = kSmallBoth,
                           bool stage_skew = true, uint32_t* d_skew_seen = nullptr);

// ---- the uniform-stride WAL replay (wal.cc replay_pass) ------------------------
// Segment 0's first header (type 0, payload n, 1 <= n <= kStgGateLen) gives a stride sigma = n + 8;
// the pass assumes every segment holds m = seg / sigma records at slots i * sigma and checks it.
// Slot g = s * m + i; events are keyed 2 g (slot g) and 2 (s + 1) m - 1 (the header after segment
// s's last slot).  stop_key: the first exact stop scan_record makes there (a CRC mismatch, an
// all-zero header: "Corrupt record"); dev_key: the first place the assumption breaks (any other
// header).  The result is scan_record's whenever stop_key <= dev_key; otherwise the walk runs.
// (tests/wal_model.py spec_replay restates the rule; tests/test_wal_model.py holds it to the model.)
struct WalSpec {
    unsigned long long stop_key, dev_key;  // ~0 between calls
    uint32_t done;                         // workgroups finished (0 between calls)
    uint32_t skew;                         // a batch's records started on few LDS banks (0 between calls)
};
// The SPEC form of k_ragged_staged_pipe over the slots of a.spec_nseg segments of a.spec_seg bytes
// (a.arena = image + 8): every workgroup reads the stride from segment 0's first header; per slot
// the header check and the payload CRC against the header's field, one atomicMin per wave; the
// last workgroup writes the summary to a.spec_out and resets a.spec.  One launch per pass.
hipError_t launch_ragged_staged_spec(const RaggedArgs& a, int grid_blocks, hipStream_t s, bool skew);
// The same pass over payloads up to kSpecDirectMax bytes: the SPEC form of k_ragged_direct4 (4-lane
// groups reading global memory, the quad blob).  A pass whose first payload is outside its kernel's
// range reports WalSummary::spec = 3 with that payload in max_len (the host takes the other kernel).
constexpr uint32_t kSpecDirectMax = 1024;
hipError_t launch_ragged_direct_spec(const RaggedArgs& a, int grid_blocks, hipStream_t s);
// ... enqueued by the library (capi.cc): the blob, one workgroup per CU; direct: the 4-lane form.
int ragged_spec_batch_dev(const void* d_wal, uint64_t nseg, uint64_t seg_bytes, uint64_t first_pos, uint64_t base0,
                          uint64_t wal_end, WalSpec* d_spec, WalSummary* h_out, hipStream_t s, bool stage_skew,
                          bool direct);

// ---- WAL replay on the device (wal_device.hip, driven by wal.cc) -----------
struct WalSegMeta {
    uint32_t count;  // type-0 records (candidates) the walk found
    uint32_t kind;   // KARMA_WAL_END / _CORRUPT / _BAD_TYPE, or kWalSpill
    uint64_t stop;   // WAL offset where the segment's walk stopped (segment end for END; for
                     // kWalSpill the offset past the segment end where the chain continues)
    uint32_t max_len;  // an upper bound of the candidates' payload lengths
    uint32_t first_bad;  // inline CRCs: ordinal of the first mismatching candidate (~0u: none;
                         // ~0u - 1: not all checksummed); other walks: ~0u - 1
};
static_assert(sizeof(WalSegMeta) == 24, "one 24-byte record per segment");

// An accepted size-0 record advances replay by 12 bytes, not 8: scan_record appends the 4
// stale bytes to the record (wal.cc:66) and sivir::open advances by record.size()
// (sivir.cc:38).  When that carries the chain 1-4 bytes past a segment's end, the next
// segment is entered at that offset instead of 0; the walk reports the segment with this
// internal kind, replay stops there (k_wal_plan), and replay_core continues from the
// reported offset with another device pass (wal.cc).  Never returned to a caller.
constexpr uint32_t kWalSpill = 16;

// What replay reads, from the segments' metas (k_wal_plan, on the device): segments [0, w1),
// n_all candidates in them, their largest payload, and the structural stop.
struct WalSummary {
    uint64_t n_all;
    uint64_t end;        // WAL offset where the walk stopped (the image end when every segment ended cleanly)
    uint32_t w1;
    uint32_t status;     // KARMA_WAL_END / _CORRUPT / _BAD_TYPE (structural)
    uint32_t max_len;    // an upper bound of the payload lengths
    uint32_t crc_unknown;  // inline CRCs (k_wal_walk_crc): 1 = some candidate of [0, w1) was not checksummed
    uint64_t first_bad;  // the first candidate whose payload CRC differs (~0: none), set by the CRC check
    uint64_t bad_off;    // inline CRCs: that candidate's header offset relative to wal (k_wal_plan)
    uint32_t stage_skew; // the staged small-record batch met records on few LDS banks (RaggedArgs::stage_skew_seen)
    uint32_t spec;       // the uniform-stride pass: 0 not run, 1 its result is final (n_all accepted
                         // records, w1 = slots per segment, max_len = payload, bad_off = the stop's
                         // header offset relative to wal), 2 declined: the walk decides, 3 the first
                         // payload (max_len) is the other kernel's size class: the walk decides
};
static_assert(sizeof(WalSummary) == 56, "one 56-byte summary, read back in one copy");

// One sub-range walker's result: where it started (a header it found, or the
// sub-range end: none), its list length, its stop kind / offset and where it left
// the sub-range (segment-relative).
struct WalSubMeta {
    uint32_t first, count, kind, stop, exit, max_len, pad[2];
};
struct WalArgs {
    const uint8_t* wal;        // first byte of segment s0 (WAL offset base0)
    uint64_t base0;            // s0 * seg_bytes
    uint64_t seg_bytes;        // < 2^31
    uint64_t first_pos;        // where replay enters segment s0 (start - base0)
    uint32_t* cand_rec;        // per segment: cand_cap header offsets within the segment
    uint32_t* cand_len;        //              payload lengths
    uint32_t* cand_crc;        //              and the CRC fields of their headers
    uint64_t cand_cap;         // seg_bytes / 8 + 1
    WalSegMeta* meta;          // per segment
    uint64_t* cand_base;       // per segment: first slot in the contiguous lists (k_wal_plan)
    uint64_t* off;             // header offset relative to wal, per candidate
    uint32_t* len;
    uint32_t* stored;          // CRC field of the header
    const uint32_t* crc;       // payload CRC from the ragged batch
    uint64_t* first_bad;       // min candidate index with crc != stored (&sum->first_bad)
    // The walk splits each segment into nsub sub-ranges of sub_bytes (wal_walk_plan).
    uint64_t nsub;
    uint64_t sub_bytes;        // a multiple of the walker's 4 KiB tile
    uint64_t sub_cap;          // list slots per sub-range: sub_bytes / 8 + 1 (cand_cap = nsub * sub_cap)
    WalSubMeta* sub;           // per (segment, sub-range) walker
    uint32_t* span;            // per (segment, sub-range): first list slot of the accepted run, candidates before it
    uint64_t img_bytes;        // bytes at wal (nwork segments)
    uint64_t nwork;            // segments walked
    uint64_t n_all;            // capacity of the contiguous lists (bounds build checks)
    WalSummary* sum;           // k_wal_plan's result
    uint64_t wal_end;          // WAL offset of the image end
    const uint32_t* crc_blob;  // k_wal_walk_crc: the quad blob (its tables' LDS image; empty units' address)
    uint32_t direct_streak;    // the walkers read headers straight from global memory after a fast round
                               // of at least this many headers (0: tiles only; wal.cc kDirectStreak)
    uintptr_t kb_lo, kb_hi;    // bounds build: the image's allocation (the inline CRC loads)
    // the fused resolve + gather (k_wal_resolve_gather): per segment two tagged words (count and
    // stop flag; largest payload), and this call's tag (1..65535; the words are zeroed when it wraps)
    unsigned long long* rg_words;
    uint32_t rg_tag;
};
constexpr uint32_t kWalkTile = 4096;  // the one-wave walker's LDS tile (wal_device.hip)
constexpr uint32_t kMaxSub = 4096;    // sub-ranges per segment (k_wal_gather stages their runs in LDS)
struct WalWalkPlan {
    uint64_t nsub, sub_bytes, sub_cap, cand_cap;
    int kernel;  // 0: sub-range walkers (+ resolve when nsub > 1), 1: one workgroup per segment,
                 // 2: sub-range walkers with the CRCs inline (k_wal_walk_crc, + resolve),
                 // 3: sub-range walkers, then their lists checksummed (k_wal_list_crc, + resolve)
    int cu;      // CUs of the device (the list kernel's grid)
};
// Host planner (wal.cc).  sub_bytes: 0 = the planner's split, else the forced sub-range
// size (karma_wal_tuning).
WalWalkPlan wal_walk_plan(uint64_t seg_bytes, uint64_t nseg, int cu, uint64_t sub_bytes, bool inline_crc = false,
                          bool list_crc = false);
constexpr int kWalFuseWaves = 15;  // walkers per workgroup of k_wal_walk_crc (wal_device.hip)
hipError_t launch_wal_walk(const WalArgs& a, uint64_t nseg, const WalWalkPlan& plan, hipStream_t s,
                           bool resolve = true);
// The replay plan on the device: a.sum, a.cand_base (first list slot per segment) and
// *a.first_bad = ~0, from the walk's metas of nseg segments.
hipError_t launch_wal_plan(const WalArgs& a, uint64_t nseg, hipStream_t s);
// Gather: one block per segment of the nseg walked; segments from sum->w1 on do nothing.
// fused_plan (nseg <= 1024): the gather computes the plan itself (no launch_wal_plan before it).
hipError_t launch_wal_gather(const WalArgs& a, uint64_t nseg, bool fused_plan, int cu, hipStream_t s);
// The resolve (sub-range walkers, nsub > 1) and the fused-plan gather in one launch, one 1024-thread
// block per segment (nseg <= 1024): wave 0 resolves the segment, the block's list offset comes from
// the earlier segments' tagged counts (a look-back), then the block gathers.  Replaces
// k_wal_resolve + k_wal_gather<true>; a.rg_words / a.rg_tag set.
hipError_t launch_wal_resolve_gather(const WalArgs& a, uint64_t nseg, hipStream_t s);
// The first of n candidates whose payload CRC differs from the stored one (atomicMin into *first_bad).
hipError_t launch_wal_compare(const WalArgs& a, uint64_t n, int cu, hipStream_t s);
// The summary (device memory) into page-locked host memory by one wave's stores: the host reads it
// after the stream syncs.  A 56-byte hipMemcpyAsync D2H is a copy kernel of its own (~4 us on the
// replay's stream); this is one small launch (wal.cc's summary readback).
hipError_t launch_wal_publish(const WalSummary* src, WalSummary* dst_host, hipStream_t s);
// Segments the uniform-stride pass takes at most (its slot keys stay far below 2^64).
constexpr uint64_t kSpecMaxSeg = 1u << 20;

// ---- KFP frames (kfp.cc) ----------------------------------------------------
struct KfpWalk {
    std::vector<uint64_t> frame, span_off;  // frame offsets; the CRC span of each (header + payload)
    std::vector<uint32_t> span_len, stored;  // span lengths; the CRC stored in each frame
    uint64_t consumed = 0;                   // bytes of the accepted frames
};
// The structural part of connection::read_frame's parse loop over buf; returns KARMA_KFP_*.
int kfp_walk(const uint8_t* buf, size_t buf_bytes, size_t max_frames, KfpWalk* out);

// karma_crc32c_trim: the per-device contexts of the host-memory, WAL and KFP entry points (their
// streams, events, device buffers and pinned staging) released after their in-flight call, if
// any, has finished; recreated by the next call.  0 or the first error.
int trim_host_contexts(int dev);
int trim_replay_ctx(int dev);      // wal.cc
int trim_host_batch_ctx(int dev);  // host_batch.cc
int trim_append_ctx(int dev);      // wal_append.cc
int trim_kfp_ctx(int dev);         // kfp.cc
int trim_stage(int dev);           // host_stage.cc
// A context's own stream: its per-stream batch state (workspace, look-back and fused words) freed
// before the context destroys the handle (capi.cc).
int release_internal_stream(int dev, hipStream_t s);
size_t stream_state_count();

// Synthetic data: bytes of the counter-based splitmix64 stream.
hipError_t launch_fill_splitmix(uint8_t* dst, uint64_t n_bytes, uint64_t seed, uint64_t first_byte, hipStream_t s);
// Read-only streaming probe (achievable-HBM reference): xor-reduces n_bytes.
hipError_t launch_stream_probe(const uint8_t* src, uint64_t n_bytes, uint32_t* out, int grid_blocks, hipStream_t s);

}  // namespace engine
}  // namespace karma
