"""The ragged byte-grid path's algebra (tests/grid_model.py, a lane-level restatement of
k_ragged_grid_plan and of the grid branches of k_units_ragged / k_ragged_finalize) against the
oracle, on the CPU: sorted layouts with every kind of record edge a tile can hold -- records
shorter than a window, records straddling tile and chunk edges, ~init bytes split over two
windows or two tiles, empty and 1-3-byte records, interior tiles -- and the grid's conditions."""
import numpy as np
import pytest

import grid_model as G
import oracle_lib


def _layout(rng, n, lens_fn, gap_hi, start):
    lens = lens_fn(rng, n).astype(np.int64)
    gaps = rng.integers(0, gap_hi + 1, n)
    offs = start + np.concatenate([[0], np.cumsum(lens[:-1] + gaps[1:])]) + gaps[0]
    return offs.astype(np.int64), lens


SHAPES = {
    "mixed": (lambda rng, n: np.where(rng.random(n) < 0.3, rng.integers(0, 40, n), rng.integers(40, 5000, n)), 24),
    "tiny": (lambda rng, n: rng.integers(0, 12, n), 6),
    "wal": (lambda rng, n: np.full(n, 180), 8),
    "large": (lambda rng, n: rng.integers(2000, 9000, n), 8),
    "packed": (lambda rng, n: rng.integers(1, 300, n), 0),
}


@pytest.mark.parametrize("shape", list(SHAPES))
@pytest.mark.parametrize("tile", [1024, 2048])
def test_grid_model_matches_oracle(shape, tile):
    rng = np.random.default_rng(list(SHAPES).index(shape) * 10007 + tile)
    fn, gap = SHAPES[shape]
    n = {"tiny": 600, "wal": 500, "large": 40, "packed": 700, "mixed": 120}[shape]
    start = int(rng.integers(0, 64))
    offs, lens = _layout(rng, n, fn, gap, start)
    size = int(offs[-1] + lens[-1]) + 64
    mem = rng.integers(0, 256, size, dtype=np.uint8)
    init = rng.integers(0, 1 << 32, n, dtype=np.uint64).astype(np.uint32)
    recs = [(int(o), int(l), int(i)) for o, l, i in zip(offs, lens, init)]
    assert G.grid_eligible(recs, tile, 1 << 30, tile)
    got = G.grid_crcs(bytes(mem), recs, tile)
    want = oracle_lib.ragged_crcs(mem, offs.astype(np.uint64), lens.astype(np.uint32), init)
    assert np.array_equal(np.array(got, np.uint32), want)


def test_grid_model_edges_on_tile_and_chunk_boundaries():
    """Records that start and end exactly on, and 1-3 bytes either side of, tile and chunk edges
    (the ~init word split over two tiles), and one record over many tiles."""
    tile = 1024
    rng = np.random.default_rng(5)
    recs, pos = [], 0
    for target in [tile - 3, 2 * tile - 2, 3 * tile - 1, 4 * tile, 5 * tile + 1, 6 * tile - 128, 7 * tile + 127,
                   8 * tile + 13, 9 * tile - 4]:
        start = target
        assert start >= pos
        n = int(rng.integers(4, 300))
        recs.append((start, n, int(rng.integers(0, 1 << 32))))
        pos = start + n
    recs.append((pos, 9 * tile + 5, 0xFFFFFFFF))  # interior tiles
    pos += 9 * tile + 5
    recs.append((pos + 1, 3, 7))
    mem = rng.integers(0, 256, pos + 64, dtype=np.uint8)
    got = G.grid_crcs(bytes(mem), recs, tile)
    want = oracle_lib.ragged_crcs(mem, np.array([r[0] for r in recs], np.uint64), np.array([r[1] for r in recs], np.uint32),
                                  np.array([r[2] for r in recs], np.uint32))
    assert np.array_equal(np.array(got, np.uint32), want)


def test_grid_conditions():
    recs = [(0, 100, 0), (100, 50, 0), (160, 10, 0)]
    assert G.grid_eligible(recs, 2048, 4, 2048)
    assert not G.grid_eligible([(0, 100, 0), (99, 50, 0)], 2048, 4, 2048)        # overlap
    assert not G.grid_eligible([(100, 10, 0), (0, 50, 0)], 2048, 4, 2048)        # unsorted
    assert not G.grid_eligible([(0, 100, 0), (100 + 2049, 5, 0)], 2048, 4, 2048)  # gap past the limit
    assert G.grid_eligible([(0, 100, 0), (100 + 2048, 5, 0)], 2048, 4, 2048)
    assert not G.grid_eligible([(0, 10000, 0)], 2048, 4, 2048)                     # tiles past tile_cap


def test_inverse_of_sixteen_zero_bytes():
    for x in (1, 0x80000000, 0x12345678, 0xFFFFFFFF):
        assert G.ZINV16(G.Z(16)(x)) == x
        assert G.ZINV16(G.Z(20)(x)) == G.Z(4)(x)
