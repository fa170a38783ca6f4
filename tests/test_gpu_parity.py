"""Parity of the gfx950 kernels with the oracle (run on the MI355X box: pytest -m gpu).

Bit-exact comparisons through the C ABI (karma_amd wraps it with ctypes) against
oracle/crc32c_port.c (itself pinned to the reference build by tests/test_oracle.py) and the
committed golden fixtures; full BASELINE sizes (configs 2-4) are checked record by record.
"""
import contextlib
import ctypes
import os

import numpy as np
import pytest

import oracle_lib
import synth
from golden_inputs import ragged_inputs

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
    rng = np.random.default_rng(5)
    host = rng.integers(0, 256, size=(1 << 23) + 64, dtype=np.uint8)
    return host, torch.from_numpy(host).to(dev)


def _eq(got, want):
    got = np.asarray(got, dtype=np.uint32)
    want = np.asarray(want, dtype=np.uint32)
    bad = np.nonzero(got != want)[0]
    assert bad.size == 0, f"{bad.size} mismatches, first {[(int(i), hex(int(got[i])), hex(int(want[i]))) for i in bad[:4]]}"


def test_native_library_is_what_runs(dev):
    buf = torch.zeros(4096, dtype=torch.uint8, device=dev)
    K.value_batch_fixed(buf, 4096)
    torch.cuda.synchronize()
    maps = open("/proc/self/maps").read()
    # the shipped build (or, under --karma-lib bounds, the bounds-checked build of the same sources)
    assert _lib.lib()._name in (_lib.LIB_PATH, _lib.BOUNDS_LIB_PATH)
    assert os.path.realpath(_lib.lib()._name) in maps
    assert K.device_cu_count() >= 1


@pytest.mark.parametrize("rec", [1, 2, 3, 4, 7, 15, 16, 17, 31, 32, 33, 63, 64, 65, 100, 127, 128, 129, 255, 256,
                                 257, 1000, 2047, 2048, 2049, 4095, 4096, 4097, 5000, 8192, 12000, 16384, 65535, 65536,
                                 100000])
@pytest.mark.parametrize("mis", [0, 1, 4, 8, 13])
def test_fixed_sizes_and_alignments(raw, rec, mis):
    host, dbuf = raw
    n = min(3000, ((1 << 23) - mis) // rec)
    got = K.value_batch_fixed(dbuf[mis: mis + n * rec], rec).cpu().numpy()
    _eq(got, oracle_lib.fixed_crcs(host[mis: mis + n * rec], rec))


@pytest.mark.parametrize("rec,n", [(1 << 23, 1), (3 << 20, 2), ((1 << 22) - 7, 2), (1 << 20, 8), (123457, 60),
                                   (777777, 10), (40000, 200)])
@pytest.mark.parametrize("mis", [0, 3])
def test_split_records_multilevel_combine(raw, rec, n, mis):
    host, dbuf = raw
    if mis + n * rec > host.size:
        n = (host.size - mis) // rec
    got = K.value_batch_fixed(dbuf[mis: mis + n * rec], rec).cpu().numpy()
    _eq(got, oracle_lib.fixed_crcs(host[mis: mis + n * rec], rec))


@pytest.mark.parametrize("rec", [4096, 4100, 4111, 8192, 12345, 20000])
@pytest.mark.parametrize("max_k", ["2", "8"])
def test_in_wave_split_fold(dev, rec, max_k, monkeypatch):
    """Batches that fill the GPU cut each record into 2/4/8 units whose groups share a wave
    (k_units_fixed KW); unaligned record starts, a partial last wave, scalar and array inits."""
    if max_k != "2":  # the shipped planner splits in 2; 4 and 8 are the tools build's KARMA_FOLD_MAX_K
        monkeypatch.setenv("KARMA_FOLD_MAX_K", max_k)
        ctx = _lib.using(_lib.AB_LIB_PATH)
    else:
        ctx = contextlib.nullcontext()
    with ctx:
        _in_wave_split_fold(dev, rec)


def _in_wave_split_fold(dev, rec):
    n = 4 * K.device_cu_count() * 128 + 37
    buf = torch.empty(n * rec, dtype=torch.uint8, device=dev)
    K.fill_splitmix64(buf, 11)
    got = K.value_batch_fixed(buf, rec).cpu().numpy()
    want = oracle_lib.splitmix_fixed_crcs(11, rec, 0, n, threads=16)
    _eq(got, want)
    if rec in (4100, 20000):
        _eq(K.value_batch_fixed(buf, rec, init=0xCAFEF00D).cpu().numpy(),
            oracle_lib.splitmix_fixed_crcs(11, rec, 0, n, init=0xCAFEF00D, threads=16))
        init = (np.arange(n, dtype=np.uint64) * 2654435761 % (1 << 32)).astype(np.uint32)
        d_ini = torch.from_numpy(init.view(np.int32)).to(dev)
        got = K.value_batch_fixed(buf, rec, init=d_ini).cpu().numpy()
        sel = np.r_[0:64, n // 2:n // 2 + 64, n - 64:n]  # Extend(c, D) = Combine(c, Value(D), |D|)
        _eq(got[sel], [K.Combine(int(init[r]), int(want[r]), rec) for r in sel])


def test_init_array_and_scalar(raw, dev):
    host, dbuf = raw
    rng = np.random.default_rng(9)
    for rec, n in [(333, 2000), (4096, 500), (20, 1000), (70000, 40)]:
        init = rng.integers(0, 1 << 32, size=n, dtype=np.uint64).astype(np.uint32)
        got = K.value_batch_fixed(dbuf[: n * rec], rec, init=torch.from_numpy(init).to(dev)).cpu().numpy()
        want = [oracle_lib.extend(int(init[r]), host[r * rec:(r + 1) * rec].tobytes()) for r in range(n)]
        _eq(got, want)
        got = K.value_batch_fixed(dbuf[: n * rec], rec, init=0xDEADBEEF).cpu().numpy()
        want = [oracle_lib.extend(0xDEADBEEF, host[r * rec:(r + 1) * rec].tobytes()) for r in range(n)]
        _eq(got, want)


@pytest.mark.parametrize("key", ["ragged_replay_mix", "ragged_small_init", "ragged_tiny_unaligned"])
@pytest.mark.parametrize("with_total", [True, False])
def test_ragged_golden(records, dev, key, with_total):
    data, offs, lens, init, want = ragged_inputs(records[key])
    got = K.extend_batch_ragged(torch.from_numpy(data).to(dev), torch.from_numpy(offs.astype(np.int64)).to(dev),
                                torch.from_numpy(lens.astype(np.int32)).to(dev),
                                init=None if init is None else torch.from_numpy(init).to(dev),
                                total_len=int(lens.sum()) if with_total else None).cpu().numpy()
    _eq(got, want)


def test_ragged_edge_lengths_every_alignment(raw, dev):
    host, dbuf = raw
    offs, lens = [], []
    for a in range(16):  # every start alignment mod 16 ...
        for n in range(0, 301):  # ... times every length 0..300 (head / body / tail / short paths)
            i = len(offs)
            offs.append(((i * 397) % (1 << 22)) // 16 * 16 + a)
            lens.append(n)
    offs = np.array(offs, dtype=np.uint64)
    lens = np.array(lens, dtype=np.uint32)
    init = synth.splitmix_words(77, 0, offs.size).astype(np.uint32)
    got = K.extend_batch_ragged(dbuf, torch.from_numpy(offs.astype(np.int64)).to(dev),
                                torch.from_numpy(lens.astype(np.int32)).to(dev),
                                init=torch.from_numpy(init).to(dev)).cpu().numpy()
    _eq(got, oracle_lib.ragged_crcs(host, offs, lens, init))


def test_ragged_overlapping_large_and_end_of_buffer(raw, dev):
    host, dbuf = raw
    size = (1 << 23) + 64
    rng = np.random.default_rng(4)
    lens = np.concatenate([rng.integers(0, 300000, 500), [size, size - 1, 1 << 20, 5, 0, 17, 1 << 22]]).astype(np.uint32)
    offs = np.array([int(rng.integers(0, size - int(n) + 1)) for n in lens[:-7]] +
                    [0, 1, size - (1 << 20), size - 5, size, size - 17, 3], dtype=np.uint64)
    got = K.extend_batch_ragged(dbuf, torch.from_numpy(offs.astype(np.int64)).to(dev),
                                torch.from_numpy(lens.astype(np.int32)).to(dev)).cpu().numpy()
    _eq(got, oracle_lib.ragged_crcs(host, offs, lens))


@pytest.mark.parametrize("n_small", [300_000, 1_200_000])
def test_ragged_many_records_per_lane_with_huge_records(raw, dev, n_small):
    """The plan and finalize with several records per thread / lane (300K records: R = FR = 2;
    1.2M: R = FR = 4, finalize lanes taking two passes), with records of more than 64 units
    (the whole wave folds them) at the start, in the middle and at the end of the batch, empty
    and short records among them, and per-record inits."""
    host, dbuf = raw
    rng = np.random.default_rng(n_small)
    lens = rng.integers(0, 300, n_small).astype(np.uint32)
    lens[rng.integers(0, n_small, 2000)] = rng.integers(0, 16, 2000)  # short records: finalize alone
    huge_at = [0, 1, n_small // 3, n_small // 2 + 7, n_small - 2, n_small - 1]
    lens[huge_at] = [(1 << 23) - 3, 1 << 22, (3 << 20) + 17, 600_000, 1 << 23, (5 << 20) + 1]
    offs = (rng.integers(0, host.size - 300, n_small)).astype(np.uint64)
    for i in huge_at:
        offs[i] = int(rng.integers(0, host.size - int(lens[i]) + 1))
    init = rng.integers(0, 1 << 32, n_small, dtype=np.uint64).astype(np.uint32)
    got = K.extend_batch_ragged(dbuf, torch.from_numpy(offs.astype(np.int64)).to(dev),
                                torch.from_numpy(lens.astype(np.int32)).to(dev),
                                init=torch.from_numpy(init.view(np.int32)).to(dev), total_len=int(lens.sum()))
    _eq(got.cpu().numpy(), oracle_lib.ragged_crcs(host, offs, lens, init))


def test_empty_batches(dev):
    buf = torch.zeros(16, dtype=torch.uint8, device=dev)
    out = torch.full((1,), 7, dtype=torch.int32, device=dev)
    assert _lib.lib().karma_crc32c_batch_fixed(buf.data_ptr(), 16, 0, None, 0, out.data_ptr(), None) == 0
    torch.cuda.synchronize()
    assert int(out.item()) == 7  # nothing written for zero records
    # zero-length records: Extend(c, D, 0) = c
    outs = torch.zeros(5, dtype=torch.uint32, device=dev)
    assert _lib.lib().karma_crc32c_batch_fixed(None, 0, 5, None, 0x55, outs.data_ptr(), None) == 0
    torch.cuda.synchronize()
    _eq(outs.cpu().numpy(), [0x55] * 5)
    e = torch.zeros(0, dtype=torch.int64, device=dev)
    assert K.extend_batch_ragged(buf, e, e.to(torch.int32)).numel() == 0
    z = torch.zeros(0, dtype=torch.uint8, device=dev)
    assert int(K.extend_stream(0x1234, z).item()) == 0x1234  # Extend(c, D, 0) = c


def test_stream_64mib_pattern_kat(dev):
    pat = torch.from_numpy(np.frombuffer(synth.pattern(64 << 20), dtype=np.uint8).copy()).to(dev)
    assert int(K.extend_stream(0, pat).item()) == 0x0C49B210
    # streaming semantics: Extend(Value(A), B) == Value(A || B) at an unaligned cut
    a, b = pat[: 12345677], pat[12345677:]
    va = int(K.extend_stream(0, a).item())
    assert int(K.extend_stream(va, b).item()) == 0x0C49B210
    assert K.Combine(va, int(K.extend_stream(0, b).item()), b.numel()) == 0x0C49B210


def test_stream_1gib_with_init(dev):
    n = 1 << 30
    buf = torch.empty(n, dtype=torch.uint8, device=dev)
    K.fill_splitmix64(buf, 1234)
    got = int(K.extend_stream(0xCAFEF00D, buf).item())
    want = int(oracle_lib.splitmix_fixed_crcs(1234, n, 0, 1, init=0xCAFEF00D, threads=1)[0])
    assert got == want


def test_stream_fused_combine_segments_and_graph_replay(dev):
    """One record per call (a segment scan) takes the fused combine: the units kernel's last
    workgroup folds the wave states, read through per-call tags (k_units_fixed FUSE).  64 distinct
    64 MiB segments back to back on one stream, sizes from one wave state to the 64 Ki states one
    launch folds (1 GiB), a second stream interleaved, and the call captured in a hipGraph and
    replayed with new bytes in the buffer: every CRC against the oracle."""
    seg, nseg = 64 << 20, 64
    buf = torch.empty(seg * nseg, dtype=torch.uint8, device=dev)
    K.fill_splitmix64(buf, 99)
    out = torch.empty(nseg, dtype=torch.uint32, device=dev)
    for i in range(nseg):
        K.extend_stream(0, buf[i * seg:(i + 1) * seg], out=out[i:i + 1])
    _eq(out.cpu().numpy(), oracle_lib.splitmix_fixed_crcs(99, seg, 0, nseg, threads=16))
    # sizes: 16 KiB (one wave state) .. 1 GiB, unaligned starts, two streams alternating
    s2 = torch.cuda.Stream()
    host = buf[: (1 << 30) + 64].cpu().numpy()
    for i, (off, n) in enumerate([(0, 16 << 10), (3, (16 << 10) + 5), (100, 1 << 20), (7, (8 << 20) + 77),
                                  (0, 64 << 20), (1, (1 << 30) - 1), (0, 1 << 30)]):
        st = s2 if i % 2 else torch.cuda.current_stream()
        with torch.cuda.stream(st):
            got = K.extend_stream(0x1234567, buf[off: off + n], stream=st)
        st.synchronize()
        assert int(got.item()) == oracle_lib.extend(0x1234567, host[off: off + n].tobytes()), (off, n)
    # captured once, replayed with new bytes (the tags come from the device)
    s = torch.cuda.Stream()
    part = buf[:seg]
    o1 = torch.empty(1, dtype=torch.uint32, device=dev)
    with torch.cuda.stream(s):
        K.extend_stream(0, part, out=o1, stream=s)
    s.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        K.extend_stream(0, part, out=o1, stream=s)
    for seed in (5, 6, 7):
        torch.cuda.synchronize()
        K.fill_splitmix64(part, seed)
        torch.cuda.synchronize()
        g.replay()
        torch.cuda.synchronize()
        assert int(o1.item()) == int(oracle_lib.splitmix_fixed_crcs(seed, seg, 0, 1, threads=16)[0])


def test_segment_once_sizes_and_alignments(dev):
    """One record of 256 KiB .. 64 MiB takes k_segment_once (every wave one wave-step of 8 units,
    its loads in flight at once; workgroup folds, then the last workgroup's).  Sizes at its
    thresholds, units from 128 B to 2 KiB, starts and ends off the 16- and 128-byte grids (an end
    off the 128-byte grid caps the unit at 1,920 B: the largest such records fall back to the
    looping kernel), repeated calls (tags), against the oracle."""
    n = (64 << 20) + 256
    buf = torch.empty(n, dtype=torch.uint8, device=dev)
    K.fill_splitmix64(buf, 31)
    host = buf.cpu().numpy()
    cases = [(0, (256 << 10) - 1), (0, 256 << 10), (5, (256 << 10) + 1), (3, (1 << 20) + 17), (64, 3 << 20),
             (9, (48 << 20) + 5), (0, 64 << 20), (128, 64 << 20), (16, 64 << 20), (1, (64 << 20) - 1),
             (5, 60 << 20), (0, (60 << 20) + 7), (77, (32 << 20) - 77), (0, 16 << 20)]
    for init in (0, 0x9E3779B9):
        for off, m in cases:
            got = int(K.extend_stream(init, buf[off: off + m]).item())
            assert got == oracle_lib.extend(init, host[off: off + m].tobytes()), (hex(init), off, m)
    # one record with a one-element per-record init array (batch_fixed's d_init) takes the same
    # kernel: the array's value seeds it, not the scalar
    for off, m in [(0, 1 << 20), (3, (16 << 20) + 5), (0, 64 << 20)]:
        ini = torch.from_numpy(np.array([0x7A5C31E9], dtype=np.uint32)).to(dev)
        got = int(K.value_batch_fixed(buf[off: off + m], m, init=ini).cpu().numpy().astype(np.uint32)[0])
        assert got == oracle_lib.extend(0x7A5C31E9, host[off: off + m].tobytes()), ("init array", off, m)


def test_segment_once_8copy_tables(dev, monkeypatch):
    """The tools build's k_segment_once on the 8-copy stride image (KARMA_SEGMENT_R8=1: half the
    table fill) is held to the shipped form's parity: every size, alignment and init case above."""
    monkeypatch.setenv("KARMA_SEGMENT_R8", "1")
    with _lib.using(_lib.AB_LIB_PATH):
        test_segment_once_sizes_and_alignments(dev)


def test_segment_once_arrival_fold(dev, monkeypatch):
    """k_segment_once with the last-ARRIVING workgroup folding (one ticket per workgroup; the
    tools build's KARMA_SEGMENT_ONCE=2): sizes at the thresholds and unaligned, repeated calls
    (the ticket counter is reset by each call's folder), 4 streams launched with no
    synchronisation, and a graph captured once and replayed with new bytes."""
    monkeypatch.setenv("KARMA_SEGMENT_ONCE", "2")
    n = (64 << 20) + 256
    buf = torch.empty(n * 4, dtype=torch.uint8, device=dev)
    K.fill_splitmix64(buf, 57)
    host = buf[:n].cpu().numpy()
    with _lib.using(_lib.AB_LIB_PATH) as L:
        for init in (0, 0x1F2E3D4C):
            for off, m in [(0, 256 << 10), (5, (256 << 10) + 1), (3, (1 << 20) + 17), (0, 64 << 20), (1, (64 << 20) - 1),
                           (77, (32 << 20) - 77)]:
                for _ in range(2):
                    got = int(K.extend_stream(init, buf[off: off + m]).item())
                    assert got == oracle_lib.extend(init, host[off: off + m].tobytes()), (hex(init), off, m)
        seg = 64 << 20
        want = oracle_lib.splitmix_fixed_crcs(57, seg, 0, 4, threads=16)
        streams = [torch.cuda.Stream() for _ in range(4)]
        outs = [torch.full((4,), -1, dtype=torch.int32, device=dev) for _ in range(4)]
        torch.cuda.synchronize()
        for i in range(8):
            for k, st in enumerate(streams):
                j = (i + k) % 4
                _lib.check("stream", L.karma_crc32c_stream(0, buf.data_ptr() + j * seg, seg,
                                                           outs[k].data_ptr() + 4 * j, st.cuda_stream))
        torch.cuda.synchronize()
        for k in range(4):
            _eq(outs[k].cpu().numpy().view(np.uint32), want)
        s = torch.cuda.Stream()
        part = buf[:seg]
        o1 = torch.empty(1, dtype=torch.uint32, device=dev)
        with torch.cuda.stream(s):
            K.extend_stream(0, part, out=o1, stream=s)
        s.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            K.extend_stream(0, part, out=o1, stream=s)
        for seed in (8, 9):
            torch.cuda.synchronize()
            K.fill_splitmix64(part, seed)
            torch.cuda.synchronize()
            g.replay()
            torch.cuda.synchronize()
            assert int(o1.item()) == int(oracle_lib.splitmix_fixed_crcs(seed, seg, 0, 1, threads=16)[0])
        for st in streams + [s]:
            assert L.karma_crc32c_release_stream(-1, st.cuda_stream) == 0


def test_config2_full_1m_x_4k(dev):
    n, rec = 1 << 20, 4096
    buf = torch.empty(n * rec, dtype=torch.uint8, device=dev)
    K.fill_splitmix64(buf, 42)
    got = K.value_batch_fixed(buf, rec).cpu().numpy()
    want = oracle_lib.splitmix_fixed_crcs(42, rec, 0, n, threads=16)
    _eq(got, want)
    # size-independent properties at full size: a flipped byte changes exactly that record,
    # and by the CRC's linearity the change equals Value(delta) ^ Value(zeros)
    r, pos = 777777, 1234
    old = int(got[r])
    buf[r * rec + pos] ^= 0x40
    got2 = K.value_batch_fixed(buf, rec).cpu().numpy()
    changed = np.nonzero(got2 != got)[0]
    assert changed.tolist() == [r]
    delta = np.zeros(rec, np.uint8)
    delta[pos] = 0x40
    assert int(got2[r]) ^ old == K.Value(delta) ^ K.Value(np.zeros(rec, np.uint8))


def test_config3_full_ragged_replay_mix(dev):
    count = int((4 << 30) / (((65536 - 64) / np.log(1024)) + 8))
    lens = synth.loguniform_lengths(7, count, 64, 65536)
    offs, arena = synth.ragged_layout(lens, header=8)
    buf = torch.empty(arena + 16, dtype=torch.uint8, device=dev)
    K.fill_splitmix64(buf, 42)
    got = K.extend_batch_ragged(buf, torch.from_numpy(offs.astype(np.int64)).to(dev),
                                torch.from_numpy(lens.astype(np.int32)).to(dev), total_len=int(lens.sum()))
    host = buf.cpu().numpy()
    _eq(got.cpu().numpy(), oracle_lib.ragged_crcs(host, offs, lens, threads=16))


def test_config4_64_segments_of_64mib(dev):
    seg, nseg = 64 << 20, 64
    buf = torch.empty(seg * nseg, dtype=torch.uint8, device=dev)
    K.fill_splitmix64(buf, 42)
    got = K.value_batch_fixed(buf, seg).cpu().numpy()
    _eq(got, oracle_lib.splitmix_fixed_crcs(42, seg, 0, nseg, threads=16))


def test_config5_shards_concatenate_to_whole_batch(dev):
    # 8 record shards computed separately (as 8 ranks would) == the unsharded batch
    from karma_amd.shard import shard_range
    n, rec = 1 << 17, 4096
    buf = torch.empty(n * rec, dtype=torch.uint8, device=dev)
    K.fill_splitmix64(buf, 42)
    whole = K.value_batch_fixed(buf, rec).cpu().numpy()
    parts = []
    for r in range(8):
        lo, hi = shard_range(n, 8, r)
        sub = torch.empty((hi - lo) * rec, dtype=torch.uint8, device=dev)
        K.fill_splitmix64(sub, 42, first_byte=lo * rec)  # the rank's own slice of the global stream
        parts.append(K.value_batch_fixed(sub, rec).cpu().numpy())
    _eq(np.concatenate(parts), whole)


def test_config5_full_shard(dev):
    """BASELINE configs[4]'s per-GPU work on one GPU: rank 7's shard of 256M x 4 KiB records,
    33,554,432 records = 128 GiB at first_byte = 7 * shard * 4096 (bench.py's N = 8 default),
    generated on the device as that rank's slice of the global stream.  Every one of the 33.5M
    CRCs is checked against the oracle, computed in slices of 4M records on the host threads
    (SURVEY §8(d) config 5 asks for a 1M-record sample + a rolling digest; the full comparison
    covers both), and the XOR / 64-bit-sum digests of the two arrays are compared as well.
    Per-record independence: karma-store/segment_file.cc:22, wal.cc:60."""
    from karma_amd.shard import shard_range
    n_total, world, rank, rec = 1 << 28, 8, 7, 4096
    lo, hi = shard_range(n_total, world, rank)
    n = hi - lo
    assert n == 33_554_432
    buf = torch.empty(n * rec, dtype=torch.uint8, device=dev)
    K.fill_splitmix64(buf, 42, first_byte=lo * rec)
    got = K.value_batch_fixed(buf, rec).cpu().numpy()
    del buf
    torch.cuda.empty_cache()
    threads = max(1, min(16, len(os.sched_getaffinity(0))))
    step = 1 << 22
    want = np.empty(n, np.uint32)
    for a in range(0, n, step):
        b = min(n, a + step)
        want[a:b] = oracle_lib.splitmix_fixed_crcs(42, rec, lo + a, b - a, threads=threads)
    assert int(np.bitwise_xor.reduce(got)) == int(np.bitwise_xor.reduce(want))
    assert int(got.astype(np.uint64).sum()) == int(want.astype(np.uint64).sum())
    _eq(got, want)


def test_rccl_gather_world1(dev):
    L = _lib.lib()
    uid = (ctypes.c_char * _lib.UNIQUE_ID_BYTES)()
    _lib.check("uid", L.karma_crc32c_get_unique_id(uid, _lib.UNIQUE_ID_BYTES))
    comm = ctypes.c_void_p()
    _lib.check("init", L.karma_crc32c_comm_init(ctypes.byref(comm), 1, uid, 0))
    try:
        n, rec = 4096, 4096
        buf = torch.empty(n * rec, dtype=torch.uint8, device=dev)
        K.fill_splitmix64(buf, 5)
        loc = torch.empty(n, dtype=torch.uint32, device=dev)
        allc = torch.empty(n, dtype=torch.uint32, device=dev)
        s = torch.cuda.current_stream().cuda_stream
        _lib.check("sharded", L.karma_crc32c_batch_fixed_sharded(comm, buf.data_ptr(), rec, n, 0, loc.data_ptr(),
                                                                 allc.data_ptr(), 0, s))
        torch.cuda.synchronize()
        _eq(allc.cpu().numpy(), oracle_lib.splitmix_fixed_crcs(5, rec, 0, n))
    finally:
        L.karma_crc32c_comm_destroy(comm)


def test_host_memory_paths(raw):
    host, _ = raw
    rec = 4096
    n = host.size // rec
    got = K.value_batch_fixed_host(host[: n * rec], rec)
    _eq(got, oracle_lib.fixed_crcs(host[: n * rec], rec))
    big = synth.splitmix_np(8, 0, 300 << 20).copy()  # > one 64 MiB chunk: exercises the 2-stream pipeline
    got = K.value_batch_fixed_host(big, 1000)
    _eq(got, oracle_lib.fixed_crcs(big[: (big.size // 1000) * 1000], 1000))
    lens = synth.uniform_lengths(2, 5000, 0, 3000)
    offs, arena = synth.ragged_layout(lens, header=8)
    got = K.extend_batch_ragged_host(host[: arena], offs, lens, init=0x77)
    _eq(got, oracle_lib.ragged_crcs(host, offs, lens, np.full(lens.size, 0x77, np.uint32)))


def test_ragged_host_chunks_and_order():
    # > 64 MiB of records: several staged chunks over the two streams; then the same
    # records in shuffled order (one chunk over the whole arena) and repeated calls
    # reusing the cached slots
    lens = synth.loguniform_lengths(9, 24000, 64, 65536)
    offs, arena = synth.ragged_layout(lens, header=8)
    buf = synth.splitmix_np(10, 0, arena + 16).copy()
    want = oracle_lib.ragged_crcs(buf, offs, lens)
    assert arena > 3 * (64 << 20)
    _eq(K.extend_batch_ragged_host(buf[:arena], offs, lens), want)
    perm = np.random.default_rng(3).permutation(lens.size)
    _eq(K.extend_batch_ragged_host(buf[:arena], offs[perm], lens[perm]), want[perm])
    few = slice(100, 140)
    _eq(K.extend_batch_ragged_host(buf[:arena], offs[few], lens[few]), want[few])
    _eq(K.extend_batch_ragged_host(buf[:arena], offs[:0], lens[:0]), want[:0])


def test_rejects_bad_arguments(dev):
    L = _lib.lib()
    buf = torch.zeros(64, dtype=torch.uint8, device=dev)
    assert L.karma_fill_splitmix64(buf.data_ptr() + 1, 32, 1, 0, None) == _lib.KARMA_E_INVALID
    assert L.karma_fill_splitmix64(buf.data_ptr(), 32, 1, 3, None) == _lib.KARMA_E_INVALID
    with pytest.raises(ValueError):
        K.value_batch_fixed(buf, 7)


@pytest.mark.parametrize("env,val", [("KARMA_CRC_VARIANT", v) for v in "127"] + [("KARMA_FOLD_MAX_K", "1")])
def test_kernel_variants_match_oracle(raw, dev, env, val, monkeypatch):
    """The A/B kernels of the tools build (karma_amd/csrc/ab.h, tools/variant_bench.py) are held to
    the same parity as the shipped ones."""
    monkeypatch.setenv(env, val)
    with _lib.using(_lib.AB_LIB_PATH):
        _variants_match_oracle(raw, dev)


def _variants_match_oracle(raw, dev):
    host, dbuf = raw
    for rec, n in [(4096, 2000), (512, 5000), (1 << 16, 100), (3 << 20, 2)]:
        got = K.value_batch_fixed(dbuf[: n * rec], rec).cpu().numpy()
        _eq(got, oracle_lib.fixed_crcs(host[: n * rec], rec))
    got = K.value_batch_fixed(dbuf[: 1000 * 4096], 4096, init=0x1234).cpu().numpy()
    offs4 = np.arange(1000, dtype=np.uint64) * 4096
    _eq(got, oracle_lib.ragged_crcs(host, offs4, np.full(1000, 4096, np.uint32), np.full(1000, 0x1234, np.uint32)))
    lens = synth.loguniform_lengths(4, 1500, 1, 16384)
    offs, arena = synth.ragged_layout(lens, header=8)
    assert arena <= host.size
    ini = (np.arange(lens.size, dtype=np.uint64) * 2654435761 % (1 << 32)).astype(np.uint32)
    d_off = torch.from_numpy(offs.astype(np.int64)).to(dev)
    d_len = torch.from_numpy(lens.astype(np.int32)).to(dev)
    d_ini = torch.from_numpy(ini.astype(np.uint32).view(np.int32)).to(dev)
    got = K.extend_batch_ragged(dbuf[:arena], d_off, d_len, init=d_ini, total_len=int(lens.sum())).cpu().numpy()
    _eq(got, oracle_lib.ragged_crcs(host, offs, lens, ini.astype(np.uint32)))


@pytest.mark.parametrize("form", ["40", "41", "60", "61"])
def test_ragged_units_stream_form_matches_oracle(raw, dev, form, monkeypatch):
    """The tools build's descriptor-driven stream form of the ragged units kernel
    (k_units_ragged_stream: stream_unit with masked edges, KARMA_RAGGED_UNITS_STREAM = PF, dynamic
    tail) is held to the shipped kernel's parity: every length 0..300 at every alignment with
    per-record inits, records of many units and of one, WAL-framed whole units, the variants mix."""
    host, dbuf = raw
    monkeypatch.setenv("KARMA_RAGGED_UNITS_STREAM", form)
    with _lib.using(_lib.AB_LIB_PATH):
        test_ragged_edge_lengths_every_alignment(raw, dev)
        test_ragged_overlapping_large_and_end_of_buffer(raw, dev)
        test_ragged_many_records_per_lane_with_huge_records(raw, dev, 300_000)
        test_ragged_wal_framed_units_fill_whole_units(raw, dev, 8)
        _variants_match_oracle(raw, dev)
        shorts = np.full(5000, 9, np.uint32)  # only short records: no units at all
        soffs = (np.arange(5000, dtype=np.uint64) * 37).astype(np.uint64)
        _eq(K.extend_batch_ragged(dbuf, torch.from_numpy(soffs.astype(np.int64)).to(dev),
                                  torch.from_numpy(shorts.astype(np.int32)).to(dev), total_len=int(shorts.sum()))
            .cpu().numpy(), oracle_lib.ragged_crcs(host, soffs, shorts))


def test_ragged_finalize_lite_fill_matches_oracle(raw, dev, monkeypatch):
    """The tools build's finalize with the smaller LDS fill (KARMA_FINALIZE_LITE=1: records of more
    than 64 units fold with the maps read from global memory): huge records at the batch's start,
    middle and end with FR = 2 and 4 records per lane, every edge length and alignment."""
    monkeypatch.setenv("KARMA_FINALIZE_LITE", "1")
    with _lib.using(_lib.AB_LIB_PATH):
        test_ragged_many_records_per_lane_with_huge_records(raw, dev, 300_000)
        test_ragged_many_records_per_lane_with_huge_records(raw, dev, 1_200_000)
        test_ragged_edge_lengths_every_alignment(raw, dev)
        test_ragged_overlapping_large_and_end_of_buffer(raw, dev)
        test_ragged_low_total_len_is_still_exact(raw, dev)


@pytest.mark.parametrize("build", ["shipped", "tag_wrap"])
def test_ragged_plan_many_blocks_lookback(raw, dev, build, monkeypatch):
    """The single-pass plan (k_ragged_plan) chains its blocks' unit counts by a decoupled
    look-back: 2M records = 2048 plan blocks, alternating with small batches on one stream, so
    every call's status words overwrite older ones.  tag_wrap: the tools build with the 22-bit
    call tag wrapping every 2 calls (KARMA_LB_SEQ_MAX), so the words are cleared between calls."""
    host, dbuf = raw
    rng = np.random.default_rng(21)
    big = rng.integers(32, 300, 2 << 20).astype(np.uint32)
    big_off = rng.integers(0, host.size - 300, big.size).astype(np.uint64)
    small = rng.integers(0, 40000, 3000).astype(np.uint32)
    small_off = rng.integers(0, host.size - 40000, small.size).astype(np.uint64)
    want_big = oracle_lib.ragged_crcs(host, big_off, big)
    want_small = oracle_lib.ragged_crcs(host, small_off, small)
    cases = [(big, big_off, want_big), (small, small_off, want_small)]
    dl = [(torch.from_numpy(o.astype(np.int64)).to(dev), torch.from_numpy(n.astype(np.int32)).to(dev)) for n, o, _ in cases]
    if build == "tag_wrap":
        monkeypatch.setenv("KARMA_LB_SEQ_MAX", "3")
        ctx = _lib.using(_lib.AB_LIB_PATH)
    else:
        ctx = contextlib.nullcontext()
    s = torch.cuda.Stream()
    torch.cuda.synchronize()
    with ctx, torch.cuda.stream(s):
        for i in range(7):
            (n, o, want), (d_off, d_len) = cases[i % 2], dl[i % 2]
            _eq(K.extend_batch_ragged(dbuf, d_off, d_len, total_len=int(n.sum())).cpu().numpy(), want)


def test_ragged_graph_capture_replays(dev):
    """A ragged call captured in a hipGraph replays any number of times: the single-pass plan's
    block ids and look-back tags come from the device (k_ragged_plan / k_ragged_finalize), not
    from host state baked into the captured arguments.  200K records = 196 plan blocks, replayed
    three times with new payload bytes AND new lengths / offsets in the same buffers (sum(len) <=
    total_len), each replay exact against the oracle; uncaptured calls of other sizes run on the
    same stream between replays (they grow the stream's workspace: the graph's buffers must
    survive that)."""
    n, arena_bytes = 200_000, 48 << 20
    cap_total = 96 << 20
    arena = torch.empty(arena_bytes, dtype=torch.uint8, device=dev)
    d_off = torch.empty(n, dtype=torch.int64, device=dev)
    d_len = torch.empty(n, dtype=torch.int32, device=dev)
    out = torch.empty(n, dtype=torch.uint32, device=dev)

    def load(seed):
        rng = np.random.default_rng(seed)
        lens = np.where(rng.random(n) < 0.01, rng.integers(0, 30000, n), rng.integers(0, 400, n)).astype(np.uint32)
        offs = rng.integers(0, arena_bytes - 30000, n).astype(np.uint64)
        host = rng.integers(0, 256, arena_bytes, dtype=np.uint8)
        assert int(lens.sum()) <= cap_total
        arena.copy_(torch.from_numpy(host))
        d_off.copy_(torch.from_numpy(offs.astype(np.int64)))
        d_len.copy_(torch.from_numpy(lens.astype(np.int32)))
        return oracle_lib.ragged_crcs(host, offs, lens)

    s = torch.cuda.Stream()
    want = load(1)
    with torch.cuda.stream(s):  # the uncaptured call that sizes the stream's workspace
        K.extend_batch_ragged(arena, d_off, d_len, out=out, total_len=cap_total, stream=s)
    s.synchronize()
    _eq(out.cpu().numpy(), want)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        K.extend_batch_ragged(arena, d_off, d_len, out=out, total_len=cap_total, stream=s)
    for seed in (2, 3, 4):
        torch.cuda.synchronize()
        want = load(seed)
        torch.cuda.synchronize()
        out.view(torch.int32).fill_(-0x5A5A5A5B)  # 0xA5A5A5A5: no stale right answer
        g.replay()
        torch.cuda.synchronize()
        _eq(out.cpu().numpy(), want)
        # an uncaptured, larger call on the same stream between replays
        rng = np.random.default_rng(seed + 10)
        m = 3 * n // 2 + seed
        lens = rng.integers(0, 2000, m).astype(np.uint32)
        offs = rng.integers(0, arena_bytes - 2000, m).astype(np.uint64)
        with torch.cuda.stream(s):
            got = K.extend_batch_ragged(arena, torch.from_numpy(offs.astype(np.int64)).to(dev),
                                        torch.from_numpy(lens.astype(np.int32)).to(dev), total_len=int(lens.sum()),
                                        stream=s)
        s.synchronize()
        _eq(got.cpu().numpy(), oracle_lib.ragged_crcs(arena.cpu().numpy(), offs, lens))


def test_ragged_unknown_total_workspace_growth(raw, dev):
    """Without total_len the batch is scanned, sized and, when its workspace had to grow, scanned
    again; a fresh allocation can land at the old address, so growth (not the pointer) decides."""
    host, dbuf = raw
    s = torch.cuda.Stream()  # its own, initially empty workspace
    for nrec, hi in [(40, 100), (300, 1 << 16), (20, 1 << 21), (2000, 3000), (60, 1 << 22)]:
        rng = np.random.default_rng(nrec)
        lens = rng.integers(0, hi, nrec).astype(np.uint32)
        offs = np.array([int(rng.integers(0, host.size - int(n) + 1)) for n in lens], dtype=np.uint64)
        with torch.cuda.stream(s):
            got = K.extend_batch_ragged(dbuf, torch.from_numpy(offs.astype(np.int64)).to(dev),
                                        torch.from_numpy(lens.astype(np.int32)).to(dev), stream=s)
        s.synchronize()
        _eq(got.cpu().numpy(), oracle_lib.ragged_crcs(host, offs, lens))


def test_ragged_low_total_len_is_still_exact(raw, dev):
    """total_len only sizes the unit table: a bound below sum(len) must never change a CRC (the
    records whose units do not fit are stepped by one lane each in k_ragged_finalize)."""
    host, dbuf = raw
    lens = synth.loguniform_lengths(8, 600, 1, 60000)  # 3.6 MB arena, 78 records over 16 KiB
    offs, arena = synth.ragged_layout(lens, header=3)
    assert arena <= host.size
    d_off = torch.from_numpy(offs.astype(np.int64)).to(dev)
    d_len = torch.from_numpy(lens.astype(np.int32)).to(dev)
    want = oracle_lib.ragged_crcs(host, offs, lens)
    for total in (int(lens.sum()), int(lens.sum()) // 3, 1, 8192):
        got = K.extend_batch_ragged(dbuf[:arena], d_off, d_len, total_len=total).cpu().numpy()
        _eq(got, want)


@pytest.mark.parametrize("head", [8, 15, 1])
def test_ragged_wal_framed_units_fill_whole_units(raw, dev, head):
    """Records of U - head bytes at offset head mod U (U = 8 KiB ragged unit; head 8 = the WAL's
    [crc][len|type] header at stride U): each record's whole 16-byte blocks span a full unit, so
    the batch has n full units for a payload sum below n U.  With the exact total_len the unit
    table must still hold them all (capi.cc sizes it for the widened spans); CRCs bit-exact."""
    host, dbuf = raw
    U = 8192
    shift = (-dbuf.data_ptr()) % U  # absolute unit boundaries: offsets are relative to the arena base
    n = (host.size - shift) // U - 1
    offs = (shift + head + np.arange(n, dtype=np.uint64) * np.uint64(U)).astype(np.uint64)
    lens = np.full(n, U - head, dtype=np.uint32)
    d_off = torch.from_numpy(offs.astype(np.int64)).to(dev)
    d_len = torch.from_numpy(lens.astype(np.int32)).to(dev)
    want = oracle_lib.ragged_crcs(host, offs, lens)
    _eq(K.extend_batch_ragged(dbuf, d_off, d_len, total_len=int(lens.sum())).cpu().numpy(), want)
    _eq(K.extend_batch_ragged(dbuf, d_off, d_len).cpu().numpy(), want)
    # no record may take finalize's one-lane fallback (a record whose units did not fit the table
    # is stepped serially by one lane: ~8 KiB of byte-block steps, tens of us): with the exact
    # total_len the call must run about as fast as with a generous one (twice the payload)
    out = torch.empty(n, dtype=torch.uint32, device=dev)

    def t(total):
        ms = []
        for _ in range(7):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            K.extend_batch_ragged(dbuf, d_off, d_len, out=out, total_len=total)
            b.record()
            b.synchronize()
            ms.append(a.elapsed_time(b))
        return float(np.median(ms))

    t(2 * int(lens.sum()))  # (warm: workspaces sized)
    exact, generous = t(int(lens.sum())), t(2 * int(lens.sum()))
    # (the check's sensitivity: a total_len 16 units short makes 16 records take the fallback)
    short = t(int(lens.sum()) - 16 * U)
    assert short > 1.5 * generous + 0.015, (short, generous)
    assert exact <= 1.5 * generous + 0.015, (exact, generous)


@pytest.mark.parametrize("variant", ["shipped", "20", "21", "22"])
@pytest.mark.parametrize("bound", [0, 64, 1024, 1 << 20])
def test_ragged_bounded_direct_path(raw, dev, bound, variant, monkeypatch):
    """karma_crc32c_batch_ragged_bounded: with max_len <= 1 KiB one record per group (no plan
    kernels); any bound -- too low included -- gives the exact CRCs, with per-record inits.
    Variants 20 / 21 / 22 are the tools build's LDS-staged kernel with the skewed stage, the plain
    stage only, and the plain stage on the 8-copy image with 10 waves (KARMA_DIRECT_VARIANT: here
    every batch is too spread out to stage: their global path)."""
    host, dbuf = raw
    if variant == "shipped":
        L = _lib.lib()
    else:
        monkeypatch.setenv("KARMA_DIRECT_VARIANT", variant)
        L = _lib.load(_lib.AB_LIB_PATH)
    rng = np.random.default_rng(bound + 1)
    lens = np.concatenate([rng.integers(0, 1025, 20000), rng.integers(0, 40, 3000),
                           [0, 1, 15, 16, 17, 31, 1023, 1024, 5000]]).astype(np.uint32)
    offs = rng.integers(0, host.size - 6000, lens.size).astype(np.uint64)
    init = rng.integers(0, 1 << 32, lens.size, dtype=np.uint64).astype(np.uint32)
    d_off = torch.from_numpy(offs.astype(np.int64)).to(dev)
    d_len = torch.from_numpy(lens.astype(np.int32)).to(dev)
    d_ini = torch.from_numpy(init.view(np.int32)).to(dev)
    out = torch.full((lens.size,), -1, dtype=torch.int32, device=dev)
    st = L.karma_crc32c_batch_ragged_bounded(dbuf.data_ptr(), d_off.data_ptr(), d_len.data_ptr(), lens.size,
                                             int(lens.sum()), bound, d_ini.data_ptr(), 0, out.data_ptr(),
                                             torch.cuda.current_stream().cuda_stream)
    assert st == 0, L.karma_crc32c_last_error()
    _eq(out.cpu().numpy().view(np.uint32), oracle_lib.ragged_crcs(host, offs, lens, init))



@pytest.mark.parametrize("variant", ["shipped", "20", "21", "22"])
@pytest.mark.parametrize("shape", ["wal180", "mixed", "tiny", "unaligned_arena"])
def test_ragged_bounded_consecutive_records(raw, dev, shape, variant, monkeypatch):
    """Consecutive small records (a WAL image's payloads, a writer's block) through the bounded
    ABI: the LDS-staged kernel (14 / 15) stages a wave's 64 records when their extent fits its
    12,800 bytes and steps the rest from global memory; both paths against the oracle, with
    per-record inits, empty records, every alignment, and batches that straddle the limit."""
    host, dbuf = raw
    if variant == "shipped":
        L = _lib.lib()
    else:
        monkeypatch.setenv("KARMA_DIRECT_VARIANT", variant)
        L = _lib.load(_lib.AB_LIB_PATH)
    rng = np.random.default_rng(["wal180", "mixed", "tiny", "unaligned_arena"].index(shape) + 77)
    n = 40000
    if shape == "wal180":
        lens = np.full(n, 180, np.uint32)
        gaps = np.full(n, 8, np.uint64)
    elif shape == "mixed":  # mostly small, some records of up to 1 KiB: some batches do not fit
        lens = rng.integers(0, 260, n).astype(np.uint32)
        big = rng.random(n) < 0.01
        lens[big] = rng.integers(500, 1025, int(big.sum()))
        lens[rng.random(n) < 0.02] = 0
        gaps = rng.integers(0, 24, n).astype(np.uint64)
    elif shape == "tiny":
        lens = rng.integers(0, 20, n).astype(np.uint32)
        gaps = rng.integers(0, 3, n).astype(np.uint64)
    else:
        lens = rng.integers(1, 200, n).astype(np.uint32)
        gaps = np.full(n, 8, np.uint64)
    start = 3 if shape == "unaligned_arena" else 0
    offs = (np.concatenate([[0], np.cumsum(lens[:-1].astype(np.uint64) + gaps[:-1])]) + gaps[0]).astype(np.uint64)
    end = int(offs[-1]) + int(lens[-1])
    assert start + end <= host.size
    init = rng.integers(0, 1 << 32, n, dtype=np.uint64).astype(np.uint32)
    d_off = torch.from_numpy(offs.astype(np.int64)).to(dev)
    d_len = torch.from_numpy(lens.astype(np.int32)).to(dev)
    d_ini = torch.from_numpy(init.view(np.int32)).to(dev)
    out = torch.full((n,), -1, dtype=torch.int32, device=dev)
    arena = dbuf[start:]
    st = L.karma_crc32c_batch_ragged_bounded(arena.data_ptr(), d_off.data_ptr(), d_len.data_ptr(), n,
                                             int(lens.sum()), 1024, d_ini.data_ptr(), 0, out.data_ptr(),
                                             torch.cuda.current_stream().cuda_stream)
    assert st == 0, L.karma_crc32c_last_error()
    _eq(out.cpu().numpy().view(np.uint32), oracle_lib.ragged_crcs(host[start:], offs, lens, init))


@pytest.mark.parametrize("shift", [1, 2, 3, 16])
def test_ragged_dynamic_tail_steps(dev, shift, monkeypatch):
    """k_units_ragged with the last nws >> shift wave-steps taken from a global counter
    (RaggedArgs::dyn_shift; the tools build's KARMA_RAGGED_DYN): configs[2]'s length mix, short
    records (many wave-steps), a batch too small for any dynamic step, back to back on one stream
    (k_ragged_finalize resets the counter) and replayed from a captured graph, exact against the
    oracle."""
    monkeypatch.setenv("KARMA_RAGGED_DYN", str(shift))
    rng = np.random.default_rng(60 + shift)
    arena_bytes = 256 << 20
    host = rng.integers(0, 256, arena_bytes, dtype=np.uint8)
    arena = torch.from_numpy(host).to(dev)
    shapes = []
    for n, lo, hi in ((20000, 64, 65536), (300000, 1, 700), (50, 1, 20000)):
        lens = (synth.loguniform_lengths(shift + n, n, lo, hi) if hi == 65536 else rng.integers(lo, hi, n)).astype(np.uint32)
        offs = rng.integers(0, arena_bytes - hi, n).astype(np.uint64)
        shapes.append((torch.from_numpy(offs.astype(np.int64)).to(dev), torch.from_numpy(lens.astype(np.int32)).to(dev),
                       int(lens.sum()), oracle_lib.ragged_crcs(host, offs, lens)))
    s = torch.cuda.Stream()
    with _lib.using(_lib.AB_LIB_PATH), torch.cuda.stream(s):
        for i in range(7):
            d_off, d_len, total, want = shapes[i % 3]
            _eq(K.extend_batch_ragged(arena, d_off, d_len, total_len=total, stream=s).cpu().numpy(), want)
        d_off, d_len, total, want = shapes[0]
        out = torch.empty(d_off.numel(), dtype=torch.uint32, device=dev)
        K.extend_batch_ragged(arena, d_off, d_len, out=out, total_len=total, stream=s)
        s.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            K.extend_batch_ragged(arena, d_off, d_len, out=out, total_len=total, stream=s)
        for _ in range(3):
            out.view(torch.int32).fill_(-0x5A5A5A5B)
            g.replay()
            torch.cuda.synchronize()
            _eq(out.cpu().numpy(), want)


def test_ragged_dynamic_tail_streams_concurrently(dev):
    """The shipped ragged path (dynamic tail on, k = 3) on three streams at once, 4 calls each with
    no synchronisation between launches: each stream has its own look-back words and tail counter
    (lb_ctl[2]), so the calls never share a step; every CRC against the oracle."""
    rng = np.random.default_rng(303)
    arena_bytes = 512 << 20
    host = rng.integers(0, 256, arena_bytes, dtype=np.uint8)
    arena = torch.from_numpy(host).to(dev)
    cases = []
    for k in range(3):
        n = (30000, 200000, 60000)[k]
        lens = (synth.loguniform_lengths(k + 11, n, 64, 65536) if k != 1 else rng.integers(1, 2000, n)).astype(np.uint32)
        offs = rng.integers(0, arena_bytes - 65536, n).astype(np.uint64)
        cases.append((torch.from_numpy(offs.astype(np.int64)).to(dev), torch.from_numpy(lens.astype(np.int32)).to(dev),
                      int(lens.sum()), oracle_lib.ragged_crcs(host, offs, lens)))
    streams = [torch.cuda.Stream() for _ in range(3)]
    outs = [[torch.full((c[0].numel(),), -1, dtype=torch.int32, device=dev) for _ in range(4)] for c in cases]
    torch.cuda.synchronize()
    for i in range(4):
        for k, (d_off, d_len, total, _) in enumerate(cases):
            with torch.cuda.stream(streams[k]):
                K.extend_batch_ragged(arena, d_off, d_len, out=outs[k][i], total_len=total, stream=streams[k])
    torch.cuda.synchronize()
    for k, c in enumerate(cases):
        for i in range(4):
            _eq(outs[k][i].cpu().numpy().view(np.uint32), c[3])
