"""The KFP frame model (tests/kfp_model.py) against the contracts of the reference's transport
tests (test/test-karma-transport/transport_test.cc:13-59), on CPU."""
import struct

import kfp_model as M

ECHO = 1  # karma_rpc::OperationCode_ECHO (protocol/rpc_generated.h:89)


def _frame():
    return M.encode(b"I am header", b"I am body", op=ECHO, flag=1, seq=0)


def test_basic_frame_round_trip():
    # BasicFrameTest (transport_test.cc:13-27): parse(encode(f)) re-encodes to the same bytes
    enc = _frame()
    fl, err = M.parse_one(enc, 0)
    assert err is None and fl == len(enc)
    op, flag, seq, hdr, pay = M.decode(enc, 0)
    assert (op, flag, hdr, pay) == (ECHO, 1, b"I am header", b"I am body")
    assert M.encode(hdr, pay, op, flag, seq) == enc


def test_frame_parse_contracts():
    # FrameParseTest (transport_test.cc:28-58)
    enc = _frame()
    tail = enc + b"I am an random string"
    fl, err = M.parse_one(tail, 0)  # BOOST_CHECK_NO_THROW(parse(encoded_str_tail))
    assert err is None and fl == len(enc)
    bad_crc = enc[:-1] + b"F"
    assert M.parse_one(bad_crc, 0) == (None, M.BAD_CRC)
    bad_size = b"\xff\xff\xff\xff" + enc[4:]
    assert M.parse_one(bad_size, 0) == (None, M.BAD_SIZE)
    # read_frame's loop would go on to parse the tail: "I am" as a frame length is > MAX_FRAME_SIZE
    assert M.parse_stream(tail) == ([0], len(enc), M.BAD_SIZE)


def test_frame_layout_and_crc_span():
    enc = M.encode(b"hdr", b"payload", op=-2, flag=1, seq=77)
    fl, magic, op, flag, seq, hl = struct.unpack_from("<IBhBII", enc, 0)
    assert (fl, magic, op, flag, seq, hl) == (len(enc), 123, -2, 1, 77, 3)
    # Extend(Value(header), payload) == Value(header || payload): one contiguous span
    import oracle_lib
    assert struct.unpack_from("<I", enc, fl - 4)[0] == oracle_lib.extend(0, enc[16:fl - 4])


def test_incomplete_and_structural_stops():
    a, b = M.encode(b"h", b"x" * 100), M.encode(b"", b"")
    buf = a + b + a[:30]
    assert M.parse_stream(buf) == ([0, len(a)], len(a) + len(b), M.OK)  # trailing partial frame waits
    assert M.parse_stream(a[:19]) == ([], 0, M.OK)
    bad_magic = a[:4] + b"\x00" + a[5:]
    assert M.parse_stream(a + bad_magic) == ([0], len(a), M.BAD_MAGIC)
    bad_hl = a[:12] + struct.pack("<I", len(a) - 19) + a[16:]
    assert M.parse_stream(bad_hl) == ([], 0, M.BAD_HEADER_LEN)
    short = struct.pack("<I", 12) + a[4:]
    assert M.parse_stream(short) == ([], 0, M.BAD_LENGTH)
    assert M.parse_stream(a + a + a, max_frames=2) == ([0, len(a)], 2 * len(a), M.OK)
