"""Python restatement of Karma's KFP frame codec (test infrastructure, the checker for
karma_kfp_encode_batch / karma_kfp_parse_batch).

* encode -- transport::frame::encode (karma-transport/frame.cc:41-60): 16-byte fixed header,
            header, payload, crc = Extend(Value(header), payload)
* parse  -- connection::read_frame's loop (connection.cc:20-27) over frame::parse
            (frame.cc:62-130): nullopt when the buffer holds less than a frame, exceptions
            for a frame size over MAX_FRAME_SIZE, a wrong magic, a wrong header length or a
            wrong crc.  frame_length < 20 is undefined behaviour in the reference (unsigned
            wrap at frame.cc:101,111); it is reported as BAD_LENGTH.
CRCs come from the oracle (oracle/crc32c_port.c).
"""
from __future__ import annotations

import struct

import oracle_lib

MAGIC = 123
FIXED = 16
MAX_FRAME = 4096 * 128
OK, BAD_SIZE, BAD_MAGIC, BAD_HEADER_LEN, BAD_CRC, BAD_LENGTH = 0, 1, 2, 3, 4, 5


def encode(header: bytes, payload: bytes, op: int = 0, flag: int = 0, seq: int = 0) -> bytes:
    fl = FIXED + len(header) + len(payload) + 4
    crc = oracle_lib.extend(oracle_lib.extend(0, header), payload)
    return struct.pack("<IBhBII", fl, MAGIC, op, flag, seq, len(header)) + header + payload + struct.pack("<I", crc)


def parse_one(buf: bytes, cur: int):
    """(frame_length, None) for a frame, (None, None) for nullopt, (None, status) for a throw."""
    avail = len(buf) - cur
    if avail < FIXED + 4:
        return None, None
    fl = struct.unpack_from("<I", buf, cur)[0]
    if fl > MAX_FRAME:
        return None, BAD_SIZE
    if avail < fl:
        return None, None
    if buf[cur + 4] != MAGIC:
        return None, BAD_MAGIC
    if fl < FIXED + 4:
        return None, BAD_LENGTH
    hl = struct.unpack_from("<I", buf, cur + 12)[0]
    if hl > fl - FIXED - 4:
        return None, BAD_HEADER_LEN
    header = buf[cur + FIXED: cur + FIXED + hl]
    data = buf[cur + FIXED + hl: cur + fl - 4]
    if oracle_lib.extend(oracle_lib.extend(0, header), data) != struct.unpack_from("<I", buf, cur + fl - 4)[0]:
        return None, BAD_CRC
    return fl, None


def parse_stream(buf: bytes, max_frames: int | None = None):
    """(frame offsets, bytes consumed, status) as read_frame's loop would drain buf."""
    cur, offs = 0, []
    while max_frames is None or len(offs) < max_frames:
        fl, err = parse_one(buf, cur)
        if err is not None:
            return offs, cur, err
        if fl is None:
            break
        offs.append(cur)
        cur += fl
    return offs, cur, OK


def decode(buf: bytes, off: int):
    """(op, flag, seq, header, payload) of the frame at off (already validated)."""
    fl, magic, op, flag, seq, hl = struct.unpack_from("<IBhBII", buf, off)
    return op, flag, seq, buf[off + FIXED: off + FIXED + hl], buf[off + FIXED + hl: off + fl - 4]
