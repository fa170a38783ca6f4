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


def spec_replay(wal: bytes, seg: int, gate: int = 183):
    """The uniform-stride pass (engine.h WalSpec) restated: segment 0's first header gives the
    stride (k_ragged_staged_pipe's SPEC prologue), every slot's header and CRC and every segment's
    header after its last slot are classified (the SPEC batches), and k_wal_spec_finish decides.
    (records, stop, status) as replay(wal, seg) from 0 -- or None when the pass declines and the
    walk decides.  Keys: 2 g for slot g, 2 (s + 1) m - 1 for the header after segment s's last
    slot; stop = scan_record's "Corrupt record" there (a CRC mismatch, an all-zero header), dev =
    any other header.  (The kernel's waves end at their first key: later keys are larger and
    change nothing, as the early break below.)"""
    inf = 1 << 64
    nseg = len(wal) // seg
    if nseg == 0:
        return None
    c0, st0 = struct.unpack_from("<II", wal, 0)
    n = st0 >> 8
    if st0 & 0xFF or not 1 <= n <= gate or n + HEADER > seg:
        return None
    sig = n + HEADER
    m = seg // sig
    t = m * sig
    stop = dev = inf
    for g in range(nseg * m):
        if 2 * g >= min(stop, dev):
            break
        off = g // m * seg + g % m * sig
        c, st = struct.unpack_from("<II", wal, off)
        if st == n << 8:
            if oracle_lib.extend(0, bytes(wal[off + HEADER: off + HEADER + n])) != c:
                stop = min(stop, 2 * g)
        elif c == 0 and st == 0:
            stop = min(stop, 2 * g)
        else:
            dev = min(dev, 2 * g)
        if g % m == m - 1 and seg - t >= HEADER:  # the header after the segment's last slot
            c, st = struct.unpack_from("<II", wal, g // m * seg + t)
            key = 2 * (g // m + 1) * m - 1
            if st & 0xFF == 1:
                pass
            elif c == 0 and st == 0:
                stop = min(stop, key)
            else:
                dev = min(dev, key)
    if dev < stop:
        return None
    if stop == inf:
        return [g // m * seg + g % m * sig for g in range(nseg * m)], len(wal), END
    acc = (stop + 1) // 2
    if stop % 2 == 0:
        at = acc // m * seg + acc % m * sig
    else:
        at = (acc // m - 1) * seg + t
    return [g // m * seg + g % m * sig for g in range(acc)], at, CORRUPT
