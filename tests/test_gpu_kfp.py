"""Batched KFP frame encode / parse (karma_kfp_encode_batch / karma_kfp_parse_batch) against the
Python restatement of frame::encode / read_frame's parse loop (tests/kfp_model.py)."""
import ctypes
import struct

import numpy as np
import pytest

import kfp_model as M
import synth

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

from karma_amd import _lib  # noqa: E402


@pytest.fixture(scope="module")
def lib():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return _lib.lib()


def _frames(seed, n, max_hdr=64, max_pay=20000):
    rng = np.random.default_rng(seed)
    hl = rng.integers(0, max_hdr + 1, n).astype(np.uint32)
    pl = rng.integers(0, max_pay + 1, n).astype(np.uint32)
    hl[::17] = 0  # empty headers and payloads, as in heartbeat frames
    pl[::13] = 0
    hsrc = synth.splitmix_np(seed, 0, int(hl.sum()) + 8).copy()
    psrc = synth.splitmix_np(seed + 1, 0, int(pl.sum()) + 8).copy()
    hoff = np.concatenate([[0], np.cumsum(hl, dtype=np.uint64)[:-1]]).astype(np.uint64)
    poff = np.concatenate([[0], np.cumsum(pl, dtype=np.uint64)[:-1]]).astype(np.uint64)
    op = rng.integers(-3, 12, n).astype(np.int16)
    flag = rng.integers(0, 2, n).astype(np.uint8)
    seq = np.arange(n, dtype=np.uint32) + 1000
    return hsrc, hoff, hl, psrc, poff, pl, op, flag, seq


def _model_bytes(f, n=None):
    hsrc, hoff, hl, psrc, poff, pl, op, flag, seq = f
    n = hl.size if n is None else n
    return b"".join(M.encode(hsrc[int(hoff[i]): int(hoff[i] + hl[i])].tobytes(),
                             psrc[int(poff[i]): int(poff[i] + pl[i])].tobytes(), int(op[i]), int(flag[i]), int(seq[i]))
                    for i in range(n))


def _encode(lib, f, out_bytes):
    hsrc, hoff, hl, psrc, poff, pl, op, flag, seq = f
    out = np.zeros(out_bytes, np.uint8)
    offs = np.zeros(hl.size, np.uint64)
    ne, nb = ctypes.c_size_t(), ctypes.c_uint64()
    st = lib.karma_kfp_encode_batch(hsrc.ctypes.data, hoff.ctypes.data, hl.ctypes.data, psrc.ctypes.data,
                                    poff.ctypes.data, pl.ctypes.data, op.ctypes.data, flag.ctypes.data,
                                    seq.ctypes.data, hl.size, out.ctypes.data, out_bytes, offs.ctypes.data,
                                    ctypes.byref(ne), ctypes.byref(nb), 0)
    _lib.check("karma_kfp_encode_batch", st)
    return out[: nb.value].tobytes(), list(offs[: ne.value])


def _parse(lib, buf: bytes, max_frames=1 << 30, device_copy=False):
    arr = np.frombuffer(buf, np.uint8).copy() if buf else np.zeros(1, np.uint8)
    d = torch.from_numpy(arr).cuda() if device_copy else None
    cap = max(1, min(max_frames, len(buf) // 20 + 1))
    offs = np.zeros(cap, np.uint64)
    nf, cons, status = ctypes.c_size_t(), ctypes.c_uint64(), ctypes.c_int()
    st = lib.karma_kfp_parse_batch(arr.ctypes.data, d.data_ptr() if d is not None else None, len(buf),
                                   min(max_frames, cap), offs.ctypes.data, ctypes.byref(nf), ctypes.byref(cons),
                                   ctypes.byref(status), 0)
    _lib.check("karma_kfp_parse_batch", st)
    return list(offs[: nf.value]), cons.value, status.value


def test_encode_matches_reference_framing(lib):
    f = _frames(1, 1500)
    want = _model_bytes(f)
    got, offs = _encode(lib, f, len(want) + 64)
    assert got == want and len(offs) == 1500
    assert offs == M.parse_stream(want)[0]


def test_encode_stops_when_out_is_full(lib):
    f = _frames(2, 300)
    want = _model_bytes(f)
    cut = len(want) // 2
    got, offs = _encode(lib, f, cut)
    assert want.startswith(got) and len(got) <= cut
    assert len(got) + 16 + int(f[2][len(offs)] + f[5][len(offs)]) + 4 > cut  # the next frame would not fit


@pytest.mark.parametrize("device_copy", [False, True])
def test_parse_round_trip_with_partial_tail(lib, device_copy):
    f = _frames(3, 2000)
    enc = _model_bytes(f)
    buf = enc + M.encode(b"hh", b"p" * 5000)[:2000]  # a frame still arriving
    got = _parse(lib, buf, device_copy=device_copy)
    assert got == M.parse_stream(buf)
    assert got[1] == len(enc) and got[2] == M.OK and len(got[0]) == 2000


@pytest.mark.parametrize("what", ["payload_bit", "crc_byte", "magic", "header_len", "size_limit", "short_length"])
def test_parse_stops_where_parse_throws(lib, what):
    f = _frames(4, 1200)
    enc = bytearray(_model_bytes(f))
    offs = M.parse_stream(bytes(enc))[0]
    k = 777
    o = offs[k]
    fl = struct.unpack_from("<I", enc, o)[0]
    if what == "payload_bit":  # a bit in the header||payload span (the crc field for an empty frame)
        enc[o + 16 + (fl - 20) // 2 if fl > 20 else o + fl - 1] ^= 0x04
    elif what == "crc_byte":
        enc[o + fl - 1] = ord("F") if enc[o + fl - 1] != ord("F") else ord("G")
    elif what == "magic":
        enc[o + 4] = 0
    elif what == "header_len":
        enc[o + 12: o + 16] = struct.pack("<I", fl - 19)
    elif what == "size_limit":
        enc[o: o + 4] = b"\xff\xff\xff\xff"
    else:
        enc[o: o + 4] = struct.pack("<I", 8)
    buf = bytes(enc)
    got = _parse(lib, buf)
    want = M.parse_stream(buf)
    assert got == want
    assert len(got[0]) == k and got[1] == o
    assert got[2] == {"payload_bit": M.BAD_CRC, "crc_byte": M.BAD_CRC, "magic": M.BAD_MAGIC,
                      "header_len": M.BAD_HEADER_LEN, "size_limit": M.BAD_SIZE, "short_length": M.BAD_LENGTH}[what]


def test_parse_limits_and_empty(lib):
    f = _frames(5, 100, max_pay=300)
    enc = _model_bytes(f)
    assert _parse(lib, enc, max_frames=10) == M.parse_stream(enc, max_frames=10)
    assert _parse(lib, b"") == ([], 0, M.OK)
    assert _parse(lib, enc[:19]) == ([], 0, M.OK)
    # the reference's FrameParseTest buffers, through the batch path
    base = M.encode(b"I am header", b"I am body", op=1, flag=1)
    assert _parse(lib, base + b"I am an random string") == ([0], len(base), M.BAD_SIZE)
    assert _parse(lib, base[:-1] + b"F") == ([], 0, M.BAD_CRC)
    assert _parse(lib, b"\xff\xff\xff\xff" + base[4:]) == ([], 0, M.BAD_SIZE)
