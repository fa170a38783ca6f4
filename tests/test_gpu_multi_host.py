"""Host-memory batches over several devices of one process (karma_crc32c_batch_fixed_host_multi,
_ragged_host_multi, karma_wal_replay_multi; the split and merge are karma_amd/csrc/multi_dev.h,
checked under ASan through stubs by tests/cpp/host_logic_test.cc).  On the one-GPU box the
device list is [0] (the degenerate case) and [0, 0, ...]: the same device listed several times
runs every share on it in turn, which exercises the split, the per-share calls and the ordered
merge end to end.  Every result against the oracle / the one-device replay / tests/wal_model.py."""
import ctypes

import numpy as np
import pytest

import oracle_lib
import synth
import wal_model

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

from karma_amd import _lib  # noqa: E402


@pytest.fixture(scope="module")
def lib():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return _lib.lib()


def _devs(k):
    return (ctypes.c_int * k)(*([0] * k)), k


@pytest.mark.parametrize("k", [1, 2, 3, 8])
def test_fixed_host_multi(lib, k):
    rng = np.random.default_rng(k)
    for rec, n in [(4096, 5000), (100, 333), (7, 10), (65536, 37)]:
        host = rng.integers(0, 256, rec * n, dtype=np.uint8)
        out = np.zeros(n, np.uint32)
        devs, nd = _devs(k)
        _lib.check("fixed_host_multi", lib.karma_crc32c_batch_fixed_host_multi(host.ctypes.data, rec, n, 0x55,
                                                                                out.ctypes.data, devs, nd))
        want = oracle_lib.ragged_crcs(host, np.arange(n, dtype=np.uint64) * rec, np.full(n, rec, np.uint32),
                                      np.full(n, 0x55, np.uint32))
        assert np.array_equal(out, want), (rec, n)


@pytest.mark.parametrize("k", [1, 3])
def test_ragged_host_multi(lib, k):
    rng = np.random.default_rng(10 + k)
    lens = synth.loguniform_lengths(k, 4000, 1, 40000).astype(np.uint32)
    offs, arena = synth.ragged_layout(lens, header=8)
    host = rng.integers(0, 256, arena + 16, dtype=np.uint8)
    out = np.zeros(lens.size, np.uint32)
    devs, nd = _devs(k)
    _lib.check("ragged_host_multi", lib.karma_crc32c_batch_ragged_host_multi(
        host.ctypes.data, host.size, offs.ctypes.data, lens.ctypes.data, lens.size, 7, out.ctypes.data, devs, nd))
    assert np.array_equal(out, oracle_lib.ragged_crcs(host, offs, lens, np.full(lens.size, 7, np.uint32)))


def _replay_multi(lib, wal, seg, start, k):
    n, stop, status = ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_int()
    rec = np.zeros(wal.nbytes // 8 + 2, np.uint64)
    devs, nd = _devs(k)
    _lib.check("wal_replay_multi", lib.karma_wal_replay_multi(wal.ctypes.data, wal.nbytes, seg, start, ctypes.byref(n),
                                                              ctypes.byref(stop), ctypes.byref(status), rec.ctypes.data,
                                                              rec.size, devs, nd))
    return list(rec[: n.value]), stop.value, status.value


def _append(lib, lens, seg, nseg, seed):
    src = synth.splitmix_np(seed, 0, int(lens.sum()) + 16).copy()
    offs = np.concatenate([[0], np.cumsum(lens, dtype=np.uint64)[:-1]]).astype(np.uint64)
    wal = np.zeros(nseg * seg, np.uint8)
    cur, nf = ctypes.c_uint64(0), ctypes.c_size_t()
    rec = np.zeros(lens.size, np.uint64)
    _lib.check("append", lib.karma_wal_append_batch(src.ctypes.data, offs.ctypes.data, lens.ctypes.data, lens.size,
                                                    wal.ctypes.data, wal.nbytes, seg, ctypes.byref(cur), rec.ctypes.data,
                                                    ctypes.byref(nf), 0))
    return wal, rec[: nf.value]


@pytest.mark.parametrize("k", [1, 2, 5])
def test_wal_replay_multi_matches_one_device(lib, k):
    """Clean images, a corruption in a middle share, a bad type in the last, starts inside a share."""
    seg = 1 << 16
    lens = synth.uniform_lengths(3, 6000, 1, 1500).astype(np.uint32)
    wal, rec = _append(lib, lens, seg, 80, 4)
    cases = [(wal, 0)]
    bad = wal.copy()
    bad[int(rec[len(rec) // 2]) + 9] ^= 4  # a payload byte: CRC mismatch
    cases.append((bad, 0))
    bt = wal.copy()
    bt[int(rec[-3]) + 4] = 9  # a bad type near the end
    cases.append((bt, int(rec[10])))
    cases.append((wal, int(rec[len(rec) // 3])))
    for img, start in cases:
        want = wal_model.replay(img.tobytes(), seg, start)
        assert _replay_multi(lib, img, seg, start, k) == (list(want[0]), want[1], want[2]), (k, start)


@pytest.mark.parametrize("k", [2, 3, 6])
def test_wal_replay_multi_size0_spills_across_shares(lib, k):
    """Accepted size-0 records in a segment's last bytes carry the chain 1-4 bytes into the next
    segment (wal.cc:66, sivir.cc:38): when that crosses a share boundary the merge hands the rest
    back to a replay from the real stop."""
    import wal_images
    for seg in (4096 + 4, 1 << 16):
        for seed in range(3):
            wal, heads = wal_images.stale_empty(seg, 6, seed * 5 + k)
            want = wal_model.replay(wal.tobytes(), seg)
            assert _replay_multi(lib, wal, seg, 0, k) == (list(want[0]), want[1], want[2]), (seg, seed)
