"""Python restatement of Karma's WAL framing and replay (test infrastructure, the checker for
karma_wal_append_batch / karma_wal_replay).

* append  -- sivir::build_sqe's loop (karma-store/sivir.cc:276-317): can_hold
             (segment_file.cc:74-77) else append_footer (:33-49) and the next segment, then
             append_record (:21-31)
* replay  -- sivir::open's loop (sivir.cc:31-41) over wal::scan_record (wal.cc:34-87),
             including the size-0 quirk: read_exact_at returns early for size 0
             (segment_file.cc:8), so the CRC is taken over the stale len/type word (wal.cc:50-60),
             and an accepted size-0 record is 12 bytes long to the loop (wal.cc:66, sivir.cc:38)
CRCs come from the oracle (oracle/crc32c_port.c).
"""
from __future__ import annotations

import struct

import oracle_lib

HEADER = 8
END, CORRUPT, BAD_TYPE = 0, 1, 2


def append(payloads, wal: bytearray, seg: int, cursor: int):
    """Frame payloads into wal from cursor; returns (cursor, header offsets of framed records)."""
    offs = []
    for p in payloads:
        n = len(p)
        if n + HEADER > seg or n >> 24:
            break
        seg_end = (cursor // seg + 1) * seg
        if cursor + HEADER + n > seg_end:  # !can_hold -> append_footer
            room = seg_end - cursor
            if room < HEADER:
                wal[cursor:seg_end] = b"0" * room
            else:
                wal[cursor:seg_end] = struct.pack("<II", 0, ((room - HEADER) << 8) | 1) + b"0" * (room - HEADER)
            cursor = seg_end
        if cursor + HEADER + n > len(wal):
            break
        crc = oracle_lib.extend(0, bytes(p))
        wal[cursor:cursor + HEADER + n] = struct.pack("<II", crc, (n << 8) | 0) + bytes(p)
        offs.append(cursor)
        cursor += HEADER + n
    return cursor, offs


def replay(wal: bytes, seg: int, start: int = 0):
    """(records accepted, their header offsets, stop offset, status) as sivir::open would see them."""
    off = start
    recs = []
    while True:
        if off >= len(wal):
            return recs, off, END
        base = off // seg * seg
        pos = off - base
        if pos + HEADER > seg:  # wal.cc:40-45
            off = base + seg
            continue
        crc, st = struct.unpack_from("<II", wal, off)
        typ, size = st & 0xFF, st >> 8
        if typ == 0:
            if pos + HEADER + size > seg:
                return recs, off, CORRUPT
            data = wal[off + HEADER: off + HEADER + size] if size else wal[off + 4: off + 8]
            if oracle_lib.extend(0, bytes(data)) != crc:
                return recs, off, CORRUPT
            recs.append(off)
            # sivir.cc:38 advances record.size(): for size 0 that is the 8 header bytes plus the 4
            # stale bytes scan_record appended (wal.cc:66), so 12 -- possibly into the next segment
            off += HEADER + size if size else HEADER + 4
        elif typ == 1:
            off = base + seg
        else:
            return recs, off, BAD_TYPE


def spec_replay(wal: bytes, seg: int, start: int = 0, gate: int = 1024):
    """The uniform-stride pass (engine.h WalSpec) restated: replay's first header (at `start`) gives
    the stride (k_ragged_staged_pipe's SPEC prologue); the slots are the rest of that segment from
    `start`, then every later segment from its first byte; every slot's header and CRC and every
    segment's header after its last slot are classified (the SPEC batches), and the last
    workgroup decides (spec_finish).  (records, stop, status) as replay(wal, seg, start) -- or None
    when the pass declines and the walk decides.  Keys: 2 g for slot g, 2 g + 1 for the header
    after a segment's last slot g; stop = scan_record's "Corrupt record" there (a CRC mismatch, an
    all-zero header), dev = any other header.  (The kernel's waves end at their first key: later
    keys are larger and change nothing, as the early break below.)"""
    inf = 1 << 64
    s0, f = start // seg, start % seg
    nseg = len(wal) // seg - s0
    if nseg <= 0 or f + HEADER > seg:
        return None
    base0 = s0 * seg
    c0, st0 = struct.unpack_from("<II", wal, base0 + f)
    n = st0 >> 8
    if st0 & 0xFF or not 1 <= n <= gate or f + n + HEADER > seg:
        return None
    sig = n + HEADER
    m, m0 = seg // sig, (seg - f) // sig

    def rel(g):
        return f + g * sig if g < m0 else (1 + (g - m0) // m) * seg + (g - m0) % m * sig

    total = m0 + (nseg - 1) * m
    stop = dev = inf
    for g in range(total):
        if 2 * g >= min(stop, dev):
            break
        off = base0 + rel(g)
        c, st = struct.unpack_from("<II", wal, off)
        if st == n << 8:
            if oracle_lib.extend(0, bytes(wal[off + HEADER: off + HEADER + n])) != c:
                stop = min(stop, 2 * g)
        elif c == 0 and st == 0:
            stop = min(stop, 2 * g)
        else:
            dev = min(dev, 2 * g)
        last = g == m0 - 1 or (g >= m0 and (g - m0) % m == m - 1)
        seg_end = (off - base0) // seg * seg + seg
        if last and seg_end - (off - base0 + sig) >= HEADER:  # the header after the segment's last slot
            c, st = struct.unpack_from("<II", wal, off + sig)
            if st & 0xFF == 1:
                pass
            elif c == 0 and st == 0:
                stop = min(stop, 2 * g + 1)
            else:
                dev = min(dev, 2 * g + 1)
    if dev < stop:
        return None
    if stop == inf:
        return [base0 + rel(g) for g in range(total)], len(wal), END
    g = stop // 2
    return [base0 + rel(i) for i in range((stop + 1) // 2)], base0 + rel(g) + (sig if stop & 1 else 0), CORRUPT
