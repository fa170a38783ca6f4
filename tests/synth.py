"""Synthetic inputs shared by the golden-vector generator and the tests (test infrastructure).

Every fixture under tests/golden/ describes its input by one of these generators, so the
fixtures stay small and the GPU box can rebuild the exact bytes without /root/reference:

* ``pattern(n, start)``      byte i = ((i + start) * 31 + 7) & 0xff   
* ``splitmix(seed, off, n)`` bytes [off, off + n) of the little-endian splitmix64 stream
                             word i = mix(seed + (i + 1) * 0x9E3779B97F4A7C15)
                             (the same stream karma_fill_splitmix64 writes on the GPU)
* ``ragged_layout(...)``     a WAL-segment-like arena: 8-byte [crc][len<<8|type] header,
                             then the payload, records back to back (segment_file.cc:21-31)
"""
from __future__ import annotations

import numpy as np

GAMMA = np.uint64(0x9E3779B97F4A7C15)
M1 = np.uint64(0xBF58476D1CE4E5B9)
M2 = np.uint64(0x94D049BB133111EB)


def splitmix_words(seed: int, first: int, count: int) -> np.ndarray:
    """Words [first, first + count) of the counter-based splitmix64 stream."""
    i = np.arange(first + 1, first + 1 + count, dtype=np.uint64)
    with np.errstate(over="ignore"):
        z = np.uint64(seed) + i * GAMMA
        z = (z ^ (z >> np.uint64(30))) * M1
        z = (z ^ (z >> np.uint64(27))) * M2
        z = z ^ (z >> np.uint64(31))
    return z


def splitmix(seed: int, off: int, n: int) -> bytes:
    """Bytes [off, off + n) of the splitmix64 byte stream for ``seed``."""
    if n == 0:
        return b""
    w0 = off // 8
    w1 = (off + n + 7) // 8
    raw = splitmix_words(seed, w0, w1 - w0).astype("<u8").tobytes()
    s = off - w0 * 8
    return raw[s : s + n]


def splitmix_np(seed: int, off: int, n: int) -> np.ndarray:
    return np.frombuffer(splitmix(seed, off, n), dtype=np.uint8)


def pattern(n: int, start: int = 0) -> bytes:
    i = np.arange(start, start + n, dtype=np.int64)
    return ((i * 31 + 7) & 0xFF).astype(np.uint8).tobytes()


def loguniform_lengths(seed: int, count: int, lo: int, hi: int) -> np.ndarray:
    """Record payload lengths, log-uniform in [lo, hi] (config 3's replay mix)."""
    u = splitmix_words(seed, 0, count).astype(np.float64) / 18446744073709551616.0
    v = np.exp(np.log(lo) + u * (np.log(hi) - np.log(lo)))
    return np.clip(np.floor(v), lo, hi).astype(np.uint32)


def uniform_lengths(seed: int, count: int, lo: int, hi: int) -> np.ndarray:
    w = splitmix_words(seed, 1 << 40, count)
    return (np.uint64(lo) + w % np.uint64(hi - lo + 1)).astype(np.uint32)


def ragged_layout(lengths: np.ndarray, header: int = 8, align: int = 1) -> tuple[np.ndarray, int]:
    """Payload offsets of records packed as [header][payload] back to back; returns (offs, arena_bytes)."""
    lens = lengths.astype(np.uint64)
    step = lens + np.uint64(header)
    if align > 1:
        step = (step + np.uint64(align - 1)) // np.uint64(align) * np.uint64(align)
    starts = np.concatenate([[0], np.cumsum(step)[:-1]]).astype(np.uint64)
    offs = starts + np.uint64(header)
    total = int(starts[-1] + step[-1]) if len(lens) else 0
    return offs, total
