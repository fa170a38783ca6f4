"""The Python mirror of the WAL / KFP batch calls (karma_amd.wal) against the restatements of
Karma's loops (tests/wal_model.py, tests/kfp_model.py)."""
import numpy as np
import pytest

import kfp_model
import synth
import wal_model

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

from karma_amd import wal as W  # noqa: E402


@pytest.fixture(scope="module")
def gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def test_append_replay_and_dir(gpu, tmp_path):
    seg = 32 << 10
    lens = synth.uniform_lengths(51, 700, 0, 1500)
    data = synth.splitmix_np(52, 0, int(lens.sum()) + 16).tobytes()
    offs = np.concatenate([[0], np.cumsum(lens, dtype=np.uint64)[:-1]])
    payloads = [data[int(o): int(o) + int(n)] for o, n in zip(offs, lens)]
    wal = np.zeros(48 * seg, np.uint8)
    a = W.append(payloads, wal, seg)
    model = bytearray(wal.nbytes)
    mcur, mrec = wal_model.append(payloads, model, seg, 0)
    assert (a.cursor, list(a.records), a.framed) == (mcur, mrec, len(payloads)) and wal.tobytes() == bytes(model)
    want = wal_model.replay(wal.tobytes(), seg)
    for got in (W.replay(wal, seg), W.replay(seg_bytes=seg, d_wal=torch.from_numpy(wal).cuda())):
        assert (list(got.records), got.stop, got.status) == (list(want[0]), want[1], want[2])
    for i in range(wal.nbytes // seg):
        wal[i * seg:(i + 1) * seg].tofile(str(tmp_path / str(i * seg)))
    got = W.replay_dir(str(tmp_path))
    assert (list(got.records), got.stop, got.status) == (list(want[0]), want[1], want[2])


def test_kfp_encode_parse(gpu):
    rng = np.random.default_rng(8)
    frames = [(int(rng.integers(-5, 5)), int(rng.integers(0, 256)), int(rng.integers(0, 1 << 32)),
               rng.integers(0, 256, int(rng.integers(0, 40)), dtype=np.uint8).tobytes(),
               rng.integers(0, 256, int(rng.integers(0, 3000)), dtype=np.uint8).tobytes()) for _ in range(400)]
    enc = W.kfp_encode(frames)
    want = b"".join(kfp_model.encode(h, p, op, fl, sq) for op, fl, sq, h, p in frames)
    assert enc.n == len(frames) and enc.data.tobytes() == want
    buf = np.frombuffer(want + want[:30], np.uint8)  # a partial frame at the end: wait for more
    got = W.kfp_parse(buf)
    moffs, mused, mst = kfp_model.parse_stream(bytes(buf))
    assert (list(got.offsets), got.consumed, got.status) == (moffs, mused, mst)
    bad = bytearray(want)
    bad[int(enc.offsets[7]) + 20] ^= 1  # a header byte of frame 7: "Wrong crc32"
    got = W.kfp_parse(np.frombuffer(bytes(bad), np.uint8))
    assert (len(got.offsets), got.status) == (7, W.KFP_BAD_CRC)
