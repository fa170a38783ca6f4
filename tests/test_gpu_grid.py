"""The ragged byte grid on the GPU (k_ragged_grid_plan + the grid branches of k_units_ragged and
k_ragged_finalize, crc_ragged.hip): sorted, non-overlapping batches of every shape against the
oracle, bit for bit; batches that break a grid condition take the unit plan and stay exact; the
tools build says which path ran (karma_ab_ragged_took_grid), so each case also checks that the
path it is meant to exercise is the one that ran.  The algebra itself is pinned on the CPU by
tests/test_grid_math.py.  The grid measured slower than the unit plan, so the
shipped library is built without it (KARMA_GRID=0, engine.h): these tests run it in the tools
build, and the same batches through the shipped library's unit plan."""
import ctypes

import numpy as np
import pytest

import oracle_lib
import synth

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

import karma_amd as K  # noqa: E402
from karma_amd import _lib  # noqa: E402


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda:0")


@pytest.fixture(scope="module")
def raw(dev):
    rng = np.random.default_rng(11)
    host = rng.integers(0, 256, size=(48 << 20) + 4096, dtype=np.uint8)
    return host, torch.from_numpy(host).to(dev)


def _eq(got, want):
    got = np.asarray(got, dtype=np.uint32)
    want = np.asarray(want, dtype=np.uint32)
    bad = np.nonzero(got != want)[0]
    assert bad.size == 0, f"{bad.size} mismatches, first {[(int(i), hex(int(got[i])), hex(int(want[i]))) for i in bad[:4]]}"


def _sorted_layout(rng, lens, gap_lo, gap_hi, start):
    lens = np.asarray(lens, dtype=np.int64)
    gaps = rng.integers(gap_lo, gap_hi + 1, lens.size)
    offs = start + np.concatenate([[0], np.cumsum(lens[:-1] + gaps[1:])]) + gaps[0]
    return offs.astype(np.uint64), lens.astype(np.uint32)


def _run(dbuf, offs, lens, init=None, total=None, lib_path=None):
    """The batch through the shipped library (or lib_path); returns (crcs, took_grid or None)."""
    d_off = torch.from_numpy(offs.astype(np.int64)).to(dbuf.device)
    d_len = torch.from_numpy(lens.astype(np.int32)).to(dbuf.device)
    d_ini = None if init is None else torch.from_numpy(init.astype(np.uint32).view(np.int32)).to(dbuf.device)
    tot = int(lens.sum()) if total is None else total
    if lib_path is None:
        return K.extend_batch_ragged(dbuf, d_off, d_len, init=d_ini, total_len=tot).cpu().numpy(), None
    with _lib.using(lib_path):
        got = K.extend_batch_ragged(dbuf, d_off, d_len, init=d_ini, total_len=tot).cpu().numpy()
        took = ctypes.c_int(-1)
        assert _lib.lib().karma_ab_ragged_took_grid(ctypes.byref(took)) == 0
    return got, took.value


SHAPES = {
    # (lengths, gap range)
    "config3_like": (lambda rng, n: synth.loguniform_lengths(int(rng.integers(1 << 30)), n, 64, 65536), (8, 8)),
    "mixed": (lambda rng, n: np.where(rng.random(n) < 0.3, rng.integers(0, 40, n), rng.integers(40, 5000, n)), (0, 24)),
    "tiny": (lambda rng, n: rng.integers(0, 12, n), (0, 6)),
    "wal180": (lambda rng, n: np.full(n, 180), (8, 8)),
    "packed": (lambda rng, n: rng.integers(1, 300, n), (0, 0)),
    "gaps": (lambda rng, n: rng.integers(100, 3000, n), (0, 2048)),
    "large": (lambda rng, n: rng.integers(40000, 300000, n), (0, 64)),
}
COUNTS = {"config3_like": 3000, "mixed": 8000, "tiny": 30000, "wal180": 20000, "packed": 30000, "gaps": 4000,
          "large": 100}


@pytest.mark.parametrize("shape", list(SHAPES))
@pytest.mark.parametrize("start", [0, 5, 2040])
def test_grid_sorted_batches_match_oracle(raw, shape, start):
    host, dbuf = raw
    rng = np.random.default_rng(list(SHAPES).index(shape) * 10007 + start)
    fn, (glo, ghi) = SHAPES[shape]
    offs, lens = _sorted_layout(rng, fn(rng, COUNTS[shape]), glo, ghi, start)
    assert int(offs[-1]) + int(lens[-1]) <= host.size
    init = rng.integers(0, 1 << 32, lens.size, dtype=np.uint64).astype(np.uint32)
    want = oracle_lib.ragged_crcs(host, offs, lens, init)
    got, took = _run(dbuf, offs, lens, init, lib_path=_lib.AB_LIB_PATH)
    assert took == 1, "a sorted batch must take the byte grid"
    _eq(got, want)
    _eq(_run(dbuf, offs, lens, init)[0], want)  # the shipped library
    # scalar init
    _eq(_run(dbuf, offs, lens)[0], oracle_lib.ragged_crcs(host, offs, lens))


def test_grid_edges_on_tile_and_chunk_boundaries(raw):
    """Records starting 3..0 bytes before and 1 byte after tile and chunk edges (the ~init word
    split over two tiles and two lanes), records ending on them, 1-3-byte and empty records
    between them, and records over many tiles (> 64: finalize folds them with the whole wave)."""
    host, dbuf = raw
    rng = np.random.default_rng(3)
    recs, pos = [], 0
    for k in range(1, 600):
        edge = (pos // 2048 + 1) * 2048 + int(rng.choice([-3, -2, -1, 0, 1, 128 - 3, 128, 1024 - 1]))
        if edge < pos:
            edge += 2048
        if edge - pos > 64:  # a filler record up to a few bytes before the edge (gaps stay small)
            recs.append((pos + 1, edge - pos - int(rng.integers(2, 8))))
            pos = recs[-1][0] + recs[-1][1]
        n = int(rng.choice([0, 1, 2, 3, 4, 5, 15, 16, 17, 127, 128, 129, int(rng.integers(200, 1500))]))
        recs.append((edge, n))
        pos = edge + n
        if k % 100 == 0:  # a long record over many tiles
            big = int(rng.choice([64 * 2048 - 5, 65 * 2048 + 9, 200 * 2048 + 1, 3 << 20]))
            recs.append((pos + 7, big))
            pos += 7 + big
    offs = np.array([r[0] for r in recs], np.uint64)
    lens = np.array([r[1] for r in recs], np.uint32)
    assert pos <= host.size
    init = rng.integers(0, 1 << 32, lens.size, dtype=np.uint64).astype(np.uint32)
    got, took = _run(dbuf, offs, lens, init, lib_path=_lib.AB_LIB_PATH)
    assert took == 1
    _eq(got, oracle_lib.ragged_crcs(host, offs, lens, init))


@pytest.mark.parametrize("case", ["overlap", "unsorted", "gap", "low_total", "duplicate"])
def test_batches_outside_the_grid_take_the_unit_plan(raw, case):
    """A batch that breaks a grid condition is checksummed by the unit plan, exactly."""
    host, dbuf = raw
    rng = np.random.default_rng(["overlap", "unsorted", "gap", "low_total", "duplicate"].index(case) + 40)
    offs, lens = _sorted_layout(rng, rng.integers(10, 6000, 5000), 0, 16, 0)
    total = None
    if case == "overlap":
        k = 3000
        offs[k] = offs[k - 1] + lens[k - 1] - 1
    elif case == "unsorted":
        perm = rng.permutation(lens.size)
        offs, lens = offs[perm].copy(), lens[perm].copy()
    elif case == "gap":
        offs[4000:] += np.uint64(2049)
    elif case == "low_total":
        total = int(lens.sum()) // 4  # the grid's tiles do not fit its tile table
    else:  # the same record twice
        offs[2000] = offs[1999]
        lens[2000] = lens[1999]
    want = oracle_lib.ragged_crcs(host, offs, lens)
    got, took = _run(dbuf, offs, lens, total=total, lib_path=_lib.AB_LIB_PATH)
    assert took == 0
    _eq(got, want)
    _eq(_run(dbuf, offs, lens, total=total)[0], want)


def test_grid_and_unit_plan_alternate_on_one_stream(raw, dev):
    """Grid batches and unit-plan batches back to back on one stream (the unit plan's look-back
    tags are not advanced by grid calls), each exact."""
    host, dbuf = raw
    rng = np.random.default_rng(8)
    cases = []
    for i in range(6):
        offs, lens = _sorted_layout(rng, rng.integers(0, 9000, 4000 + 100 * i), 0, 16, i)
        if i % 2:
            perm = rng.permutation(lens.size)
            offs, lens = offs[perm].copy(), lens[perm].copy()
        cases.append((offs, lens, oracle_lib.ragged_crcs(host, offs, lens)))
    s = torch.cuda.Stream()
    torch.cuda.synchronize()
    with _lib.using(_lib.AB_LIB_PATH), torch.cuda.stream(s):
        for rnd in range(3):
            for offs, lens, want in cases:
                _eq(_run(dbuf, offs, lens)[0], want)


def test_grid_graph_capture_replays(dev):
    """A grid batch captured in a hipGraph replays with new bytes and new (sorted) lengths in the
    same buffers: the plan's flags, tile words and tile count come from the device."""
    n, arena_bytes = 50_000, 64 << 20
    cap_total = 48 << 20
    arena = torch.empty(arena_bytes, dtype=torch.uint8, device=dev)
    d_off = torch.empty(n, dtype=torch.int64, device=dev)
    d_len = torch.empty(n, dtype=torch.int32, device=dev)
    out = torch.empty(n, dtype=torch.uint32, device=dev)

    def load(seed):
        rng = np.random.default_rng(seed)
        lens = rng.integers(0, 1800, n).astype(np.uint32)
        offs, lens = _sorted_layout(rng, lens, 0, 12, int(rng.integers(0, 100)))
        host = rng.integers(0, 256, arena_bytes, dtype=np.uint8)
        arena.copy_(torch.from_numpy(host))
        d_off.copy_(torch.from_numpy(offs.astype(np.int64)))
        d_len.copy_(torch.from_numpy(lens.astype(np.int32)))
        return oracle_lib.ragged_crcs(host, offs, lens)

    s = torch.cuda.Stream()
    want = load(1)
    with _lib.using(_lib.AB_LIB_PATH):
        with torch.cuda.stream(s):
            K.extend_batch_ragged(arena, d_off, d_len, out=out, total_len=cap_total, stream=s)
        s.synchronize()
        _eq(out.cpu().numpy(), want)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            K.extend_batch_ragged(arena, d_off, d_len, out=out, total_len=cap_total, stream=s)
        for seed in (2, 3):
            torch.cuda.synchronize()
            want = load(seed)
            torch.cuda.synchronize()
            out.view(torch.int32).fill_(-0x5A5A5A5B)
            g.replay()
            torch.cuda.synchronize()
            _eq(out.cpu().numpy(), want)
