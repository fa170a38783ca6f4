"""A lane-level restatement of the ragged byte-grid path (k_ragged_grid_plan, the grid branch of
k_units_ragged and of k_ragged_finalize in karma_amd/csrc/crc_ragged.hip), checked against the
oracle on the CPU by tests/test_grid_math.py.  Test infrastructure: nothing in the product
imports it.

The records of a sorted, non-overlapping batch are cut on the absolute `tile`-byte grid.  A group
of 8 lanes streams one tile as `tile / 128` chunks of 128 bytes, lane l holding bytes
[16 l, 16 l + 16) of every chunk as four word slots that stride 128 bytes.  A
record's bytes are read in those aligned windows with every byte outside the record masked to
zero and ~init xored into its first four bytes: a zero register stepped over zero bytes stays
zero, and the register the reference starts from (`l = ~init`, crc32c.cc:283) is the same as
xoring it into the first word a word step consumes (crc32c.cc:293-299).  So every record is a
span of whole windows, [floor16(p), ceil16(e)), stepped from zero, and its register is read at
ceil16(e): s = ceil16(e) - e zero bytes after its end, undone in finalize with
Z_{-16}(Z_{16 - s}(R)).

A tile emits the register of every record whose last window it holds (gend[r], folded when that
window's chunk has been stepped) and of the record that runs past its end (gstate[t]); finalize
Horner-folds a record's tiles: Z_tile between tile ends, Z_{len of its last piece} before gend.
"""
from __future__ import annotations

POLY = 0x82F63B78
_T8 = []
for _i in range(256):
    _c = _i
    for _ in range(8):
        _c = (_c >> 1) ^ (POLY if _c & 1 else 0)
    _T8.append(_c)


def _steps(r: int, data: bytes) -> int:
    for b in data:
        r = _T8[(r ^ b) & 255] ^ (r >> 8)
    return r


class Map:
    """A GF(2)-linear map of the 32-bit register, by its columns."""

    def __init__(self, cols):
        self.cols = list(cols)

    @staticmethod
    def zero_bytes(d: int) -> "Map":
        return Map(_steps(1 << i, bytes(d)) for i in range(32))

    def __call__(self, x: int) -> int:
        r, i = 0, 0
        while x:
            if x & 1:
                r ^= self.cols[i]
            x >>= 1
            i += 1
        return r

    def inverse(self) -> "Map":
        rows = []
        for r in range(32):
            row = 1 << (32 + r)
            for i in range(32):
                if (self.cols[i] >> r) & 1:
                    row |= 1 << i
            rows.append(row)
        for c in range(32):
            piv = next(k for k in range(c, 32) if (rows[k] >> c) & 1)
            rows[c], rows[piv] = rows[piv], rows[c]
            for k in range(32):
                if k != c and (rows[k] >> c) & 1:
                    rows[k] ^= rows[c]
        return Map(sum((((rows[r] >> (32 + i)) & 1) << r) for r in range(32)) for i in range(32))


_maps = {}


def Z(d: int) -> Map:
    if d not in _maps:
        _maps[d] = Map.zero_bytes(d)
    return _maps[d]


ZINV16 = Z(16).inverse()
CHUNK, LANES = 128, 8


def grid_eligible(recs, tile: int, tile_cap: int, max_gap: int) -> bool:
    """k_ragged_grid_plan's conditions: sorted by address, no overlap, gaps <= max_gap, the
    tiles within tile_cap."""
    for k in range(1, len(recs)):
        e_prev = recs[k - 1][0] + recs[k - 1][1]
        if recs[k][0] < e_prev or recs[k][0] - e_prev > max_gap:
            return False
    tb0 = recs[0][0] // tile
    nt = -(-(recs[-1][0] + recs[-1][1]) // tile) - tb0
    return nt <= tile_cap


def grid_plan(recs, tile: int):
    """tiles (relative to tile tb0): owner[t] = first record whose end lies past the tile's
    start, and whether it covers the tile with no edge and no init bytes in it."""
    tb0 = recs[0][0] // tile
    nt = -(-(recs[-1][0] + recs[-1][1]) // tile) - tb0
    owner, interior = [0] * nt, [False] * nt
    for r, (p, n, _) in enumerate(recs):
        e = p + n
        lo = 0 if r == 0 else -(-(recs[r - 1][0] + recs[r - 1][1]) // tile) - tb0
        hi = -(-e // tile) - tb0
        for t in range(lo, hi):
            ta = (tb0 + t) * tile
            owner[t] = r
            interior[t] = p + 4 <= ta and e > ta + tile
    return tb0, nt, owner, interior


def _masked_words(mem: bytes, w_abs: int, cp: int, ce: int, inj: int, w_rel: int):
    """The window's four words with bytes outside [cp, ce) (tile-relative) zeroed and inj xored
    into [cp, cp + 4) (the kernel's grid_mask)."""
    out = []
    for k in range(4):
        a = w_rel + 4 * k
        word = int.from_bytes(mem[w_abs + 4 * k: w_abs + 4 * k + 4], "little")
        lo = min(max(cp - a, 0), 4)
        hi = min(max(ce - a, 0), 4)
        keep = (((1 << (8 * hi)) - 1) & ~((1 << (8 * lo)) - 1)) & 0xFFFFFFFF if hi > lo else 0
        word &= keep
        d = cp - a
        if 0 <= d < 4:
            word ^= (inj << (8 * d)) & 0xFFFFFFFF
        elif -4 < d < 0:
            word ^= inj >> (-8 * d)
        out.append(word)
    return out


def _group_fold(acc, m: int) -> int:
    """Lane fold (crc32c.cc STEP4W order), lanes rotated so lane m (the one holding the last
    window) comes last, then the 3-level tree Z_{16 * 2^d}."""
    c = []
    for a in acc:
        x = Z(4)(a[0])
        x = Z(4)(x ^ a[1])
        x = Z(4)(x ^ a[2])
        c.append(Z(4)(x ^ a[3]))
    v = [c[(l + m + 1) % LANES] for l in range(LANES)]
    for d in range(3):
        s = 1 << d
        v = [Z(16 * s)(v[l]) ^ (v[l + s] if l + s < LANES else 0) for l in range(LANES)]
    return v[0]


def grid_units(mem: bytes, recs, tile: int, tb0: int, nt: int, owner, interior):
    """The units kernel's grid branch, tile by tile: returns (gstate, gend)."""
    nch = tile // CHUNK
    gstate, gend = [None] * nt, [None] * len(recs)
    zs = Z(CHUNK)
    for t in range(nt):
        ta = (tb0 + t) * tile
        # the group's record list: records from owner[t] that start inside the tile, with >= 4 bytes
        if interior[t]:
            lst = [(-64, tile + 64, 0, owner[t])]
        else:
            lst = []
            r = owner[t]
            while r < len(recs) and recs[r][0] < ta + tile:
                p, n, init = recs[r]
                if n >= 4:
                    lst.append((max(p - ta, -64), min(p + n - ta, tile + 64), init ^ 0xFFFFFFFF, r))
                r += 1
        acc = [[0, 0, 0, 0] for _ in range(LANES)]
        j = 0
        for c in range(nch):
            while j < len(lst):
                cp, ce, inj, r = lst[j]
                cend = (ce + 15) & ~15
                for l in range(LANES):
                    w = c * CHUNK + 16 * l
                    if w < cend and w + 16 > cp:
                        x = _masked_words(mem, ta + w, cp, ce, inj, w)
                        acc[l] = [zs(acc[l][k]) ^ x[k] for k in range(4)]
                if cend > (c + 1) * CHUNK:
                    break  # the record runs past this chunk
                gend[r] = _group_fold(acc, ((cend - 16) >> 4) & 7)
                acc = [[0, 0, 0, 0] for _ in range(LANES)]
                j += 1
                if j < len(lst) and lst[j][0] >= (c + 1) * CHUNK:
                    break  # the next record starts in a later chunk
        if j < len(lst) and lst[j][1] > tile:
            gstate[t] = _group_fold(acc, 7)
    return gstate, gend


def grid_finalize(mem: bytes, recs, tile: int, tb0: int, gstate, gend):
    """One lane per record: Horner over its tiles, Z_{-s} back to its end, ~R."""
    out = []
    for r, (p, n, init) in enumerate(recs):
        if n < 4:
            out.append(_steps(init ^ 0xFFFFFFFF, mem[p:p + n]) ^ 0xFFFFFFFF)
            continue
        e = p + n
        P, E = p & ~15, (e + 15) & ~15
        t0, t1 = P // tile - tb0, (E - 1) // tile - tb0
        if t0 == t1:
            R = gend[r]
        else:
            acc = gstate[t0]
            for t in range(t0 + 1, t1):
                acc = Z(tile)(acc) ^ gstate[t]
            R = Z(E - (tb0 + t1) * tile)(acc) ^ gend[r]
        s = E - e
        if s:
            R = ZINV16(Z(16 - s)(R))
        out.append(R ^ 0xFFFFFFFF)
    return out


def grid_crcs(mem: bytes, recs, tile: int = 2048):
    """CRCs of recs = [(address, length, init)] (sorted, non-overlapping) through the grid."""
    tb0, nt, owner, interior = grid_plan(recs, tile)
    gstate, gend = grid_units(mem, recs, tile, tb0, nt, owner, interior)
    return grid_finalize(mem, recs, tile, tb0, gstate, gend)
