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
