"""The algebra of the LDS-staged small-record kernel and of its fold, restated in Python and checked
against the oracle (CPU only).

`lane_record_end` (karma_amd/csrc/crc_device.h) reads a record as W = ceil(n/16) windows aligned
to the record's END: the first window is front-padded with h0 = 16 W - n bytes of whatever precedes
the record, masked to zero, and ~init is xored into the record's first 4 bytes (a carry into the
second window when they straddle it).  Zero bytes entering a zero register leave it zero, so the
four word slots (Z_16 strides) and the STEP4W fold give the reference register
(karma-util/crc32c.cc:323-370).  The kernel's fold is Z16(a0) ^ Z4(a3 ^ Z4(a2 ^ Z4(a1))), the
same map as crc32c.cc's Z4(a3 ^ Z4(a2 ^ Z4(a1 ^ Z4(a0)))).  Windows are funnel-shifted out of
dwords (v_alignbyte_b32), as the kernel reads its stage.
"""
import random
import struct

import oracle_lib

POLY = 0x82F63B78
T = []
for _i in range(256):
    _c = _i
    for _ in range(8):
        _c = (_c >> 1) ^ (POLY if _c & 1 else 0)
    T.append(_c)


def _steps(r, data):
    for b in data:
        r = T[(r ^ b) & 255] ^ (r >> 8)
    return r


def Z(d, x):
    """The register x advanced over d zero bytes (the map Z_d of DESIGN.md §3)."""
    return _steps(x, bytes(d))


def _alignbyte(hi, lo, sh):
    return ((hi << 32 | lo) >> (8 * sh)) & 0xFFFFFFFF


def _fold(a):
    c = Z(4, a[1])
    c = Z(4, c ^ a[2])
    return Z(16, a[0]) ^ Z(4, c ^ a[3])


def lane_record_end(mem: bytes, sp: int, n: int, init: int) -> int:
    """crc_device.h lane_record_end over the stage bytes `mem` (record at [sp, sp + n), n >= 4)."""
    W = (n + 15) >> 4
    h0 = 16 * W - n
    s0 = sp - h0
    sh, q = s0 & 3, s0 >> 2

    def rd(k):
        return struct.unpack_from("<I", mem, 4 * k)[0]

    def keep(k):
        r = h0 - 4 * k
        return 0xFFFFFFFF if r <= 0 else 0 if r >= 4 else (0xFFFFFFFF << (8 * r)) & 0xFFFFFFFF

    d = [rd(q + i) for i in range(5)]
    w = [_alignbyte(d[k + 1], d[k], sh) & keep(k) for k in range(4)]
    inj, b, k0 = init ^ 0xFFFFFFFF, h0 & 3, h0 >> 2
    lo32, hi32 = (inj << (8 * b)) & 0xFFFFFFFF, (inj >> (32 - 8 * b)) if b else 0
    w[k0] ^= lo32
    carry = 0
    if k0 < 3:
        w[k0 + 1] ^= hi32
    else:
        carry = hi32
    a = list(w)
    for _ in range(1, W):
        q += 4
        d = [d[4]] + [rd(q + i) for i in range(1, 5)]
        v = [_alignbyte(d[k + 1], d[k], sh) for k in range(4)]
        v[0] ^= carry
        carry = 0
        a = [Z(16, a[k]) ^ v[k] for k in range(4)]
    return _fold(a) ^ 0xFFFFFFFF


def test_fold_forms_agree():
    rng = random.Random(11)
    for _ in range(300):
        a = [rng.getrandbits(32) for _ in range(4)]
        c = Z(4, a[0])
        for k in (1, 2, 3):
            c = Z(4, c ^ a[k])
        assert _fold(a) == c


def test_end_aligned_windows_match_the_oracle():
    """Every length 4..200, random lead-in bytes, alignments and inits (0 as WAL replay uses)."""
    rng = random.Random(7)
    for n in list(range(4, 201)) + [rng.randint(201, 1100) for _ in range(20)]:
        sp = rng.randint(16, 63)  # the stage keeps at least 16 bytes before a record
        mem = bytes(rng.getrandbits(8) for _ in range(sp + n + 32))
        init = rng.choice([0, rng.getrandbits(32)])
        assert lane_record_end(mem, sp, n, init) == oracle_lib.extend(init, mem[sp: sp + n]), (n, sp, init)
