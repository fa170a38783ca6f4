"""WAL images of the GPU WAL tests, framed on the CPU by tests/wal_model.py (test infrastructure).

The device replay tests (tests/test_gpu_wal.py) frame these payloads with karma_wal_append_batch;
tests/test_gpu_wal.py::test_append_matches_reference_framing pins that framing to wal_model.append
byte for byte, so the images here are the ones the GPU replays.  tests/test_sanitizers.py feeds
them to the CPU emulation of the device walk (tests/cpp/wal_walk_emu.cc).
"""
from __future__ import annotations

import numpy as np

import synth
import wal_model


def frame(src, offs, lens, seg, nseg):
    wal = bytearray(nseg * seg)
    payloads = [src[int(o): int(o) + int(n)] for o, n in zip(offs, lens)]
    cur, rec = wal_model.append(payloads, wal, seg, 0)
    return np.frombuffer(bytes(wal), np.uint8).copy(), rec


def payloads(seed, n, lo, hi):
    lens = synth.uniform_lengths(seed, n, lo, hi)
    offs = np.concatenate([[0], np.cumsum(lens, dtype=np.uint64)[:-1]]).astype(np.uint64)
    src = synth.splitmix_np(seed + 1, 0, int(lens.sum()) + 16).copy()
    return src, offs, lens


def wal_looking_payloads():
    """test_replay_payloads_that_look_like_wal_records: payloads that are slices of a WAL image
    (valid header chains inside records), 256 KiB segments -- the inputs of round 1's faulting run."""
    seg = 256 << 10
    isrc, ioffs, ilens = payloads(31, 400, 1, 200)
    inner, _ = frame(isrc, ioffs, ilens, 64 << 10, 1)
    rng = np.random.default_rng(3)
    chunks, lens = [], []
    for i in range(300):
        if i % 2 == 0:
            a = int(rng.integers(0, 4096))
            n = int(rng.integers(2000, 12000))
            chunks.append(inner[a: a + n])
        else:
            n = int(rng.integers(1, 3000))
            chunks.append(rng.integers(0, 256, n, dtype=np.uint8))
        lens.append(n)
    lens = np.array(lens, np.uint32)
    src = np.concatenate(chunks + [np.zeros(16, np.uint8)])
    offs = np.concatenate([[0], np.cumsum(lens, dtype=np.uint64)[:-1]]).astype(np.uint64)
    nseg = int((lens.astype(np.int64) + 8).sum() // seg) + 2
    wal, rec = frame(src, offs, lens, seg, nseg)
    return wal, seg, rec


def large_records(seg):
    """test_replay_large_records_jumps: log-uniform 1 B-60 KiB payloads."""
    lens = synth.loguniform_lengths(17, 900, 1, 60000)
    offs = np.concatenate([[0], np.cumsum(lens, dtype=np.uint64)[:-1]]).astype(np.uint64)
    src = synth.splitmix_np(18, 0, int(lens.sum()) + 16).copy()
    nseg = int((lens.astype(np.int64) + 8).sum() // seg) + 3
    wal, rec = frame(src, offs, lens, seg, nseg)
    return wal, seg, rec


def segment_sizes(seg):
    """test_replay_segment_sizes_tiles_and_misaligned_segments."""
    n = 6000 if seg >= (64 << 10) else 600
    src, offs, lens = payloads(13, n, 1, min(3000, seg - 8))
    nseg = int((lens.astype(np.int64) + 8).sum() // seg) + 3
    wal, rec = frame(src, offs, lens, seg, nseg)
    return wal, seg, rec


def randomized(case, inner):
    """test_replay_randomized_against_model's case `case` (its own generator state)."""
    rng = np.random.default_rng(2024 + 1000 * case)
    seg = int(rng.choice([4096, 16384 + 4, 65536, 262144, 1 << 20]))
    mix = case % 4
    n = int(rng.integers(200, 3000))
    if mix == 0:
        lens = rng.integers(1, 64, n)
    elif mix == 1:
        lens = rng.integers(1, min(4000, seg - 8), n)
    elif mix == 2:
        lens = np.minimum(synth.loguniform_lengths(case, n, 1, 60000), seg - 8)
    else:
        lens = rng.integers(100, min(6000, seg - 8), n)
    lens = lens.astype(np.uint32)
    if mix == 3:
        src = np.concatenate([inner[int(rng.integers(0, 2048)):][: int(x)] if x <= inner.size - 2048 else
                              rng.integers(0, 256, int(x), dtype=np.uint8) for x in lens] + [np.zeros(16, np.uint8)])
    else:
        src = rng.integers(0, 256, int(lens.sum()) + 16, dtype=np.uint8)
    offs = np.concatenate([[0], np.cumsum(lens, dtype=np.uint64)[:-1]]).astype(np.uint64)
    nseg = int((lens.astype(np.int64) + 8).sum() // seg) + 3
    wal, rec = frame(src, offs, lens, seg, nseg)
    if case % 3 == 1 and len(rec) > 10:
        k = int(rng.integers(1, len(rec)))
        wal[int(rec[k]) + int(rng.choice([5, 8]))] ^= 0x10
    start = int(rec[int(rng.integers(0, len(rec)))]) if case % 2 and len(rec) else 0
    return wal, seg, start


def inner_image():
    isrc, ioffs, ilens = payloads(71, 600, 1, 100)
    inner, _ = frame(isrc, ioffs, ilens, 64 << 10, 1)
    return inner


def uniform_runs(seg, seed=5):
    """test_replay_uniform_runs_speculative_walk: runs of one record size (1 B to past a tile),
    so the walker's header rounds take many headers at once and stop at every size change."""
    rng = np.random.default_rng(seed)
    sizes = [1, 7, 8, 24, 180, 1000, 4088, 5000]
    lens = []
    while len(lens) < 6000:
        size = int(rng.choice(sizes))
        lens += [min(size, seg - 8)] * int(rng.integers(1, 301 if size < 1000 else 20))
    lens = np.array(lens, np.uint32)
    offs = np.concatenate([[0], np.cumsum(lens, dtype=np.uint64)[:-1]]).astype(np.uint64)
    src = synth.splitmix_np(seed, 0, int(lens.sum()) + 16).copy()
    nseg = int((lens.astype(np.int64) + 8).sum() // (seg - 4096) + 3)
    wal, rec = frame(src, offs, lens, seg, nseg)
    return wal, seg, rec, lens


STALE_ZERO = 0x48674BC7  # crc32c::Value("\0\0\0\0"): the stored CRC a size-0 record needs to pass


def stale_empty(seg, nseg, seed):
    """Images with ACCEPTED size-0 records ("Z": header [0x48674BC7][len 0 | type 0]).  scan_record
    checks such a record against the stale len/type word (wal.cc:47-60, segment_file.cc:8) and
    returns it 12 bytes long (wal.cc:66), so sivir::open reads the next header 12 bytes on
    (sivir.cc:38); the 4 bytes after the header are never looked at (random here).  Z records are
    placed
      * inside uniform runs of one record size (the walker's speculative header rounds),
      * at every offset from 14 bytes before to 2 bytes after a 4 KiB tile edge (the tile edges
        are the sub-range edges of the split plans), so the header or the 12-byte advance
        straddles it,
      * at a segment's last header positions seg-8-d (d = 0..5): for d <= 3 the advance carries
        the chain 4-d bytes into the next segment, which the writer here continues at that
        offset (the skipped bytes are random); d = 4 ends exactly at the segment end,
      * at the image end (the chain leaves the image: replay ends past wal_bytes), or followed
        by the never-written zero tail.
    Returns (image, header offsets of every record and Z, in WAL order)."""
    rng = np.random.default_rng(seed)
    wal = np.zeros(nseg * seg, np.uint8)
    heads = []
    c = 0

    def rec(n):
        nonlocal c
        p = rng.integers(0, 256, n, dtype=np.uint8)
        crc = wal_model.oracle_lib.extend(0, p.tobytes())
        wal[c: c + 8] = np.frombuffer(np.array([crc, n << 8], "<u4").tobytes(), np.uint8)
        wal[c + 8: c + 8 + n] = p
        heads.append(c)
        c += 8 + n

    def z():
        nonlocal c
        wal[c: c + 8] = np.frombuffer(np.array([STALE_ZERO, 0], "<u4").tobytes(), np.uint8)
        e = min(c + 12, wal.size)
        wal[c + 8: e] = rng.integers(0, 256, e - c - 8, dtype=np.uint8)
        heads.append(c)
        c += 12

    def goto(t):  # one record from c to exactly t (same segment, t - c >= 9), or False
        if t - c < 9:
            return False
        rec(t - c - 8)
        return True

    def pad():  # append_footer (segment_file.cc:33-49)
        nonlocal c
        end = (c // seg + 1) * seg
        if end - c >= 8:
            wal[c: c + 8] = np.frombuffer(np.array([0, ((end - c - 8) << 8) | 1], "<u4").tobytes(), np.uint8)
            wal[c + 8: end] = ord("0")
        else:
            wal[c: end] = ord("0")
        c = end

    for s in range(nseg):
        base, end = s * seg, (s + 1) * seg
        if c >= end:
            continue
        size = int(rng.choice([1, 24, 180, 500]))
        edge_k = list(range(-14, 3))
        rng.shuffle(edge_k)
        tail_d = int(rng.integers(0, 6)) if s < nseg - 1 else int(rng.choice([0, 1, 3, 7]))
        while True:
            pos = c - base
            room = seg - pos
            if room < 2 * (8 + size) + 64:
                break
            t_edge = (pos // 4096 + 1) * 4096
            r = rng.random()
            if r < 0.06:
                z()
            elif r < 0.12 and edge_k and t_edge + 3 < seg - 64:  # a Z around the next tile edge
                if goto(base + t_edge + edge_k[-1]):
                    edge_k.pop()
                    z()
            else:
                rec(size)
        if s == nseg - 1 and tail_d == 7:  # the zero tail after a Z (stored CRC 0: "Corrupt record")
            z()
            break
        # the segment end: a Z at seg - 8 - tail_d (d <= 3: spill 4 - d bytes; d = 4: exact end)
        zpos = base + seg - 8 - tail_d
        if goto(zpos):
            z()
            if end < c <= wal.size:  # the next segment is entered at c - end; its first bytes are skipped
                wal[end: c] = rng.integers(0, 256, c - end, dtype=np.uint8)
            elif c < end:
                pad()
        else:
            pad()
    return wal, heads
