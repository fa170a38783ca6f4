/*
 * oracle/crc32c_port.c -- TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of Karma's portable CRC-32C (karma-util/crc32c.cc) used as
 * the parity checker for the MI355X engine.  Only tests/, __graft_entry__.smoke()
 * and bench.py's cpu_baseline leg may load this file's library; the product
 * (karma_amd/) never links or calls it.
 *
 * Pinned: tests/test_oracle.py checks it against tests/golden/*.json, which
 * were produced by the reference's own crc32c.cc compiled from
 * /root/reference (oracle/Makefile -> oracle/_ref/), see
 * tests/golden/make_golden.py.
 *
 * Algorithm (restated, tables generated from the polynomial, not copied):
 *   - reflected Castagnoli polynomial 0x82F63B78, pre/post xor 0xFFFFFFFF
 *     (crc32c.cc:244-245 kCRC32Xor, :283 `l = crc ^ kCRC32Xor`, :375);
 *   - byte step `l = T1[(l ^ b) & 0xff] ^ (l >> 8)` (STEP1, crc32c.cc:286-290)
 *     with T1[i] = i advanced by one byte (kByteExtensionTable, :19-62);
 *   - 4 interleaved 4-byte lanes advanced 16 bytes per step through four
 *     "stride extension" tables (STEP4/STEP16, :293-309, tables :64-242);
 *   - alignment prologue to a 4-byte boundary (:323-329), word rotation for
 *     the trailing whole words (:349-357), sequential fold of the four lanes
 *     (STEP4W, :312-319, :359-364), byte tail (:367-370);
 *   - words are read little-endian (ReadUint32LE :248-250 ->
 *     DecodeFixed32, karma-util/coding.h:77-83).
 */
#include <stdint.h>
#include <stddef.h>
#include <string.h>
#include <pthread.h>

#define ORACLE_POLY 0x82F63B78u

static uint32_t g_byte[256];       /* one byte of advance            */
static uint32_t g_stride[4][256];  /* [k][i]: (i << 8*k) advanced 16 bytes, k = byte lane */
static int g_ready = 0;
static pthread_once_t g_once = PTHREAD_ONCE_INIT;

static uint32_t adv_zero_bytes(uint32_t v, int nbytes) {
    for (int b = 0; b < nbytes; ++b) v = g_byte[v & 0xffu] ^ (v >> 8);
    return v;
}

static void build_tables(void) {
    for (uint32_t i = 0; i < 256; ++i) {
        uint32_t v = i;
        for (int k = 0; k < 8; ++k) v = (v >> 1) ^ ((v & 1u) ? ORACLE_POLY : 0u);
        g_byte[i] = v;
    }
    /* A value placed in the crc register and pushed through 16 zero bytes.
     * The register after a 4-byte word w is adv4(l ^ w); a lane that skips
     * the other three lanes' words therefore advances 16 bytes per word. */
    for (int k = 0; k < 4; ++k)
        for (uint32_t i = 0; i < 256; ++i)
            g_stride[k][i] = adv_zero_bytes(i << (8 * k), 16);
    g_ready = 1;
}

static inline void ensure_tables(void) { pthread_once(&g_once, build_tables); }

static inline uint32_t le32(const uint8_t* q) {
    return (uint32_t)q[0] | ((uint32_t)q[1] << 8) | ((uint32_t)q[2] << 16) | ((uint32_t)q[3] << 24);
}

static inline uint32_t stride16(uint32_t lane, uint32_t word) {
    return word ^ g_stride[0][lane & 0xffu] ^ g_stride[1][(lane >> 8) & 0xffu] ^
           g_stride[2][(lane >> 16) & 0xffu] ^ g_stride[3][lane >> 24];
}

/* crc32c::Extend(init_crc, data, n)  (karma-util/crc32c.h:16, crc32c.cc:275-376) */
uint32_t oracle_crc32c_extend(uint32_t init_crc, const void* data, size_t n) {
    ensure_tables();
    const uint8_t* p = (const uint8_t*)data;
    const uint8_t* end = p + n;
    uint32_t l = init_crc ^ 0xffffffffu;

    /* prologue: bytes until p is 4-byte aligned, only if that point is inside the buffer */
    uintptr_t mis = (uintptr_t)p & 3u;
    if (mis) {
        const uint8_t* al = p + (4 - mis);
        if (al <= end)
            while (p != al) { l = g_byte[(l ^ *p++) & 0xffu] ^ (l >> 8); }
    }

    if (end - p >= 16) {
        uint32_t lane[4];
        lane[0] = le32(p) ^ l;
        lane[1] = le32(p + 4);
        lane[2] = le32(p + 8);
        lane[3] = le32(p + 12);
        p += 16;
        while (end - p >= 16) {
            for (int s = 0; s < 4; ++s) lane[s] = stride16(lane[s], le32(p + 4 * s));
            p += 16;
        }
        /* single words: lane 0 takes the word, then the lanes rotate */
        while (end - p >= 4) {
            uint32_t t = stride16(lane[0], le32(p));
            lane[0] = lane[1]; lane[1] = lane[2]; lane[2] = lane[3]; lane[3] = t;
            p += 4;
        }
        /* fold: l = adv4(lane ^ l) for lanes 0..3 in order */
        l = 0;
        for (int s = 0; s < 4; ++s) l = adv_zero_bytes(lane[s] ^ l, 4);
    }
    while (p != end) l = g_byte[(l ^ *p++) & 0xffu] ^ (l >> 8);
    return l ^ 0xffffffffu;
}

uint32_t oracle_crc32c_value(const void* data, size_t n) { return oracle_crc32c_extend(0, data, n); }

/* crc32c::Mask / Unmask (karma-util/crc32c.h:21-37) */
uint32_t oracle_crc32c_mask(uint32_t crc) { return ((crc >> 15) | (crc << 17)) + 0xa282ead8u; }
uint32_t oracle_crc32c_unmask(uint32_t m) {
    uint32_t r = m - 0xa282ead8u;
    return (r >> 17) | (r << 15);
}

/* ---------------------------------------------------------------------------
 * Synthetic-data generator shared with the GPU fill kernel (DESIGN.md
 * "Synthetic data"): byte stream = little-endian splitmix64 outputs, word i of
 * the stream is mix(seed + (i + 1) * 0x9E3779B97F4A7C15).
 * ------------------------------------------------------------------------- */
static inline uint64_t splitmix_word(uint64_t seed, uint64_t i) {
    uint64_t z = seed + (i + 1) * 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

/* Bytes [byte_off, byte_off + n) of the splitmix64 stream `seed`. */
void oracle_splitmix_bytes(uint64_t seed, uint64_t byte_off, uint8_t* dst, size_t n) {
    size_t k = 0;
    while (k < n) {
        uint64_t pos = byte_off + k;
        if ((pos & 7u) == 0 && n - k >= 8) {  /* whole words (little-endian host) */
            uint64_t w = splitmix_word(seed, pos >> 3);
            memcpy(dst + k, &w, 8);
            k += 8;
            continue;
        }
        uint64_t w = splitmix_word(seed, pos >> 3);
        unsigned sh = (unsigned)(pos & 7u);
        size_t take = 8 - sh;
        if (take > n - k) take = n - k;
        for (size_t t = 0; t < take; ++t) dst[k + t] = (uint8_t)(w >> (8 * (sh + t)));
        k += take;
    }
}

/* Multi-threaded: CRCs of n_rec fixed-size records of a splitmix64 arena,
 * record r = stream bytes [r*rec_bytes, (r+1)*rec_bytes), r in [first, first+n_rec). */
typedef struct {
    uint64_t seed, rec_bytes, first, n, stride, tid;
    uint32_t init;
    uint32_t* out;
} fixed_job;

#include <stdlib.h>
static void* fixed_worker(void* arg) {
    fixed_job* j = (fixed_job*)arg;
    uint8_t* buf = (uint8_t*)malloc(j->rec_bytes ? j->rec_bytes : 1);
    for (uint64_t r = j->tid; r < j->n; r += j->stride) {
        uint64_t rec = j->first + r;
        oracle_splitmix_bytes(j->seed, rec * j->rec_bytes, buf, j->rec_bytes);
        j->out[r] = oracle_crc32c_extend(j->init, buf, j->rec_bytes);
    }
    free(buf);
    return NULL;
}

int oracle_splitmix_fixed_crcs(uint64_t seed, uint64_t rec_bytes, uint64_t first, uint64_t n_rec,
                               uint32_t init, uint32_t* out, int nthreads) {
    ensure_tables();
    if (nthreads < 1) nthreads = 1;
    if (nthreads > 256) nthreads = 256;
    pthread_t th[256];
    fixed_job jobs[256];
    for (int t = 0; t < nthreads; ++t) {
        fixed_job j = {seed, rec_bytes, first, n_rec, (uint64_t)nthreads, (uint64_t)t, init, out};
        jobs[t] = j;
        pthread_create(&th[t], NULL, fixed_worker, &jobs[t]);
    }
    for (int t = 0; t < nthreads; ++t) pthread_join(th[t], NULL);
    return 0;
}

/* Multi-threaded CRCs of ragged records already in host memory. */
typedef struct {
    const uint8_t* arena;
    const uint64_t* off;
    const uint32_t* len;
    const uint32_t* init;
    uint64_t n, stride, tid;
    uint32_t* out;
} ragged_job;

static void* ragged_worker(void* arg) {
    ragged_job* j = (ragged_job*)arg;
    for (uint64_t r = j->tid; r < j->n; r += j->stride)
        j->out[r] = oracle_crc32c_extend(j->init ? j->init[r] : 0u, j->arena + j->off[r], j->len[r]);
    return NULL;
}

int oracle_ragged_crcs(const uint8_t* arena, const uint64_t* off, const uint32_t* len, const uint32_t* init,
                       uint64_t n_rec, uint32_t* out, int nthreads) {
    ensure_tables();
    if (nthreads < 1) nthreads = 1;
    if (nthreads > 256) nthreads = 256;
    pthread_t th[256];
    ragged_job jobs[256];
    for (int t = 0; t < nthreads; ++t) {
        ragged_job j = {arena, off, len, init, n_rec, (uint64_t)nthreads, (uint64_t)t, out};
        jobs[t] = j;
        pthread_create(&th[t], NULL, ragged_worker, &jobs[t]);
    }
    for (int t = 0; t < nthreads; ++t) pthread_join(th[t], NULL);
    return 0;
}

/* Fixed-size records in host memory (CPU baseline timing over a real buffer). */
typedef struct {
    const uint8_t* base;
    uint64_t rec_bytes, n, stride, tid;
    uint32_t* out;
} hostfixed_job;

static void* hostfixed_worker(void* arg) {
    hostfixed_job* j = (hostfixed_job*)arg;
    for (uint64_t r = j->tid; r < j->n; r += j->stride)
        j->out[r] = oracle_crc32c_extend(0, j->base + r * j->rec_bytes, j->rec_bytes);
    return NULL;
}

int oracle_fixed_crcs(const uint8_t* base, uint64_t rec_bytes, uint64_t n_rec, uint32_t* out, int nthreads) {
    ensure_tables();
    if (nthreads < 1) nthreads = 1;
    if (nthreads > 256) nthreads = 256;
    pthread_t th[256];
    hostfixed_job jobs[256];
    for (int t = 0; t < nthreads; ++t) {
        hostfixed_job j = {base, rec_bytes, n_rec, (uint64_t)nthreads, (uint64_t)t, out};
        jobs[t] = j;
        pthread_create(&th[t], NULL, hostfixed_worker, &jobs[t]);
    }
    for (int t = 0; t < nthreads; ++t) pthread_join(th[t], NULL);
    return 0;
}
