"""Concurrent callers (SURVEY.md §8b "Threading": the reference's Extend is pure and reentrant and is
called from the sivir io thread, the open() caller and connection threads, so the batch entry
points must be safe to call from many threads at once).

Threads call the batch API at the same time, on their own streams and on one shared stream,
mixing layouts that use the per-stream workspace (split records, ragged plans, stream combine),
WAL replay and the host Extend.  Every result is checked bit-exact against the oracle.
ctypes releases the GIL for the duration of each foreign call, so the calls really overlap.
"""
import ctypes
import threading

import numpy as np
import pytest

import oracle_lib
import synth

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

import karma_amd as K  # noqa: E402
from karma_amd import _lib  # noqa: E402

N_THREADS = 8
ROUNDS = 6


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda:0")


@pytest.fixture(scope="module")
def cases(dev):
    """(name, call(stream) -> numpy CRCs, expected CRCs) for several layouts over one buffer."""
    rng = np.random.default_rng(21)
    host = rng.integers(0, 256, size=(12 << 20) + 64, dtype=np.uint8)
    d = torch.from_numpy(host).to(dev)
    out = []
    for rec, n in [(4096, 2048), (1 << 20, 6), ((3 << 20) + 5, 3), (333, 5000)]:
        want = oracle_lib.fixed_crcs(host[: n * rec], rec)
        out.append((f"fixed {rec}", lambda s, rec=rec, n=n: K.value_batch_fixed(d[: n * rec], rec, stream=s), want))
    lens = synth.uniform_lengths(4, 3000, 0, 9000)
    offs = rng.integers(0, host.size - 9000, size=lens.size).astype(np.uint64)
    want = oracle_lib.ragged_crcs(host, offs, lens)
    d_off = torch.from_numpy(offs.astype(np.int64)).to(dev)
    d_len = torch.from_numpy(lens.astype(np.int32)).to(dev)
    out.append(("ragged", lambda s: K.extend_batch_ragged(d, d_off, d_len, total_len=int(lens.sum()), stream=s), want))
    out.append(("ragged, total unknown", lambda s: K.extend_batch_ragged(d, d_off, d_len, stream=s), want))
    want = oracle_lib.fixed_crcs(host[: 10 << 20], 10 << 20)
    out.append(("stream 10 MiB", lambda s: K.extend_stream(0, d[: 10 << 20], stream=s), want))
    torch.cuda.synchronize()  # the inputs were copied on the default stream
    return out


def _run_threads(work):
    errors = []

    def body(i):
        try:
            work(i)
        except BaseException as e:  # reported on the main thread
            errors.append((i, repr(e)))

    ts = [threading.Thread(target=body, args=(i,)) for i in range(N_THREADS)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=120)
    assert not any(t.is_alive() for t in ts), "a thread did not finish"
    assert not errors, errors


@pytest.mark.parametrize("shared_stream", [False, True])
def test_batches_from_many_threads(dev, cases, shared_stream):
    shared = torch.cuda.Stream(device=dev)

    def work(i):
        s = shared if shared_stream else torch.cuda.Stream(device=dev)
        with torch.cuda.stream(s):
            for r in range(ROUNDS):
                name, call, want = cases[(i + r) % len(cases)]
                got = call(s)
                s.synchronize()
                got = got.cpu().numpy().astype(np.uint32)
                bad = np.nonzero(got != np.asarray(want, np.uint32))[0]
                assert bad.size == 0, f"{name}: {bad.size} mismatches (thread {i}, round {r})"

    _run_threads(work)


def test_replay_and_host_extend_from_many_threads(dev):
    lib = _lib.lib()
    seg = 64 << 10
    lens = synth.uniform_lengths(8, 4000, 1, 3000)
    offs = np.concatenate([[0], np.cumsum(lens, dtype=np.uint64)[:-1]]).astype(np.uint64)
    src = synth.splitmix_np(9, 0, int(lens.sum()) + 16).copy()
    wal = np.zeros(256 * seg, np.uint8)
    cur, nf = ctypes.c_uint64(0), ctypes.c_size_t()
    rec = np.zeros(lens.size, np.uint64)
    _lib.check("karma_wal_append_batch",
               lib.karma_wal_append_batch(src.ctypes.data, offs.ctypes.data, lens.ctypes.data, lens.size,
                                          wal.ctypes.data, wal.nbytes, seg, ctypes.byref(cur), rec.ctypes.data,
                                          ctypes.byref(nf), 0))
    assert nf.value == lens.size
    payload_crcs = oracle_lib.ragged_crcs(src, offs, lens)

    def work(i):
        for r in range(ROUNDS):
            if (i + r) % 2:
                n, stop, status = ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_int()
                got = np.zeros(wal.nbytes // 8, np.uint64)
                _lib.check("karma_wal_replay",
                           lib.karma_wal_replay(wal.ctypes.data, None, wal.nbytes, seg, 0, ctypes.byref(n),
                                                ctypes.byref(stop), ctypes.byref(status), got.ctypes.data, got.size,
                                                0))
                assert n.value == rec.size and np.array_equal(got[: n.value], rec), f"thread {i} round {r}"
            else:
                for j in range(i, lens.size, 97):
                    o, ln = int(offs[j]), int(lens[j])
                    assert K.Value(src[o: o + ln]) == int(payload_crcs[j])

    _run_threads(work)


def test_uniform_replay_beside_batches_from_many_threads(dev, cases):
    """The uniform-stride replay pass (one launch whose last workgroup writes the summary the host
    polls) while other threads' batches run on their own streams: half the threads replay WALs of
    one record size (a clean one, one with a corrupt record, one that must decline), from the
    start and from a checkpoint, over the device copies; the others run the batch layouts.  Every
    result against the model / the oracle."""
    import wal_model
    lib = _lib.lib()
    seg = 64 << 10
    wals = []
    for size, bad in ((180, None), (100, 700), (56, "length")):
        n = 3000
        lens = np.full(n, size, np.uint32)
        offs = (np.arange(n, dtype=np.uint64) * size).astype(np.uint64)
        src = synth.splitmix_np(size, 0, n * size + 16).copy()
        wal = np.zeros((n * (size + 8) // (seg - 256) + 2) * seg, np.uint8)
        cur, nf = ctypes.c_uint64(0), ctypes.c_size_t()
        rec = np.zeros(n, np.uint64)
        _lib.check("karma_wal_append_batch",
                   lib.karma_wal_append_batch(src.ctypes.data, offs.ctypes.data, lens.ctypes.data, n, wal.ctypes.data,
                                              wal.nbytes, seg, ctypes.byref(cur), rec.ctypes.data, ctypes.byref(nf), 0))
        if bad == "length":
            wal[int(rec[1500]) + 5] ^= 1
        elif bad is not None:
            wal[int(rec[bad]) + 8] ^= 1
        starts = (0, int(rec[1234]))
        wals.append((torch.from_numpy(wal).to(dev), wal.nbytes,
                     {st: wal_model.replay(wal.tobytes(), seg, st) for st in starts}))
    torch.cuda.synchronize()

    def work(i):
        s = torch.cuda.Stream(device=dev)
        for r in range(ROUNDS):
            if i % 2:
                d_wal, nbytes, want = wals[(i + r) % len(wals)]
                for st, w in want.items():
                    n, stop, status = ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_int()
                    got = np.zeros(nbytes // 8, np.uint64)
                    _lib.check("karma_wal_replay",
                               lib.karma_wal_replay(None, d_wal.data_ptr(), nbytes, seg, st, ctypes.byref(n),
                                                    ctypes.byref(stop), ctypes.byref(status), got.ctypes.data,
                                                    got.size, 0))
                    assert (list(got[: n.value]), stop.value, status.value) == (list(w[0]), w[1], w[2]), (i, r, st)
            else:
                with torch.cuda.stream(s):
                    name, call, want = cases[(i + r) % len(cases)]
                    got = call(s)
                    s.synchronize()
                    assert np.array_equal(got.cpu().numpy().astype(np.uint32), np.asarray(want, np.uint32)), name

    _run_threads(work)
