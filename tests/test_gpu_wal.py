"""Batched WAL append / replay (karma_wal_append_batch / karma_wal_replay) against the Python
restatement of Karma's framing and scan_record loop (tests/wal_model.py)."""
import ctypes

import numpy as np
import pytest

import synth
import wal_model

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

from karma_amd import _lib  # noqa: E402

SEG = 64 << 10


@pytest.fixture(scope="module")
def lib():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return _lib.lib()


def _payloads(seed, n, lo, hi):
    lens = synth.uniform_lengths(seed, n, lo, hi)
    offs = np.concatenate([[0], np.cumsum(lens, dtype=np.uint64)[:-1]]).astype(np.uint64)
    src = synth.splitmix_np(seed + 1, 0, int(lens.sum()) + 16).copy()
    return src, offs, lens


def _append(lib, src, offs, lens, wal, cursor=0, seg=SEG):
    cur = ctypes.c_uint64(cursor)
    nf = ctypes.c_size_t()
    rec = np.zeros(lens.size, np.uint64)
    st = lib.karma_wal_append_batch(src.ctypes.data, offs.ctypes.data, lens.ctypes.data, lens.size, wal.ctypes.data,
                                    wal.nbytes, seg, ctypes.byref(cur), rec.ctypes.data, ctypes.byref(nf), 0)
    _lib.check("karma_wal_append_batch", st)
    return cur.value, rec[: nf.value]


# Replay plans (every one must give scan_record's result): (tools build?, karma_wal_tuning fields)
WALKS = {
    "workgroup": (True, 0, _lib.KARMA_WAL_CRC_PLAN),      # k_wal_walk, one workgroup per segment (tools build)
    "whole": (False, 1 << 30, _lib.KARMA_WAL_CRC_PLAN),   # k_wal_walk_sub, one walker per segment
    "split": (False, 0, _lib.KARMA_WAL_CRC_PLAN),         # the plan: few segments -> sub-range walkers
    "split4k": (False, 4096, _lib.KARMA_WAL_CRC_DIRECT),  # one-tile sub-ranges + k_wal_resolve, and every
                                                          # CRC batch one record per group (any length)
    "sep": (False, 0, _lib.KARMA_WAL_CRC_SEPARATE),       # the walk, the gathered lists, one small-record batch
    "sepdirect4": (True, 0, _lib.KARMA_WAL_CRC_SEPARATE),  # the same with the 4-lane kernel only (tools build)
    "inline": (False, 0, _lib.KARMA_WAL_CRC_INLINE),      # the CRCs inside the walk kernel (k_wal_walk_crc)
    "inline4k": (False, 4096, _lib.KARMA_WAL_CRC_INLINE),
    "listcrc": (True, 0, _lib.KARMA_WAL_CRC_INLINE),      # the walk, then the walkers' lists checksummed by
    "listcrc4k": (True, 4096, _lib.KARMA_WAL_CRC_INLINE), # the LDS-staged kernel (k_wal_list_crc; tools build)
    "r8": (True, 0, _lib.KARMA_WAL_CRC_PLAN),             # the plan, the plain-stage small-record kernel on the
                                                          # 8-copy image with 10 waves (KARMA_STAGE_R8; tools build)
    "sliced": (True, 0, _lib.KARMA_WAL_CRC_PLAN),         # the pass in two slices of segments, slice 1's walk beside
                                                          # slice 0's CRCs (KARMA_WAL_SLICES=2; tools build)
    "sliced_r8": (True, 0, _lib.KARMA_WAL_CRC_PLAN),      # the same with the 6-wave 8-copy staged kernel
    "rg0": (True, 0, _lib.KARMA_WAL_CRC_PLAN),            # the resolve and the gather as two launches (round 5's;
                                                          # the plan fuses them, k_wal_resolve_gather): KARMA_WAL_RG=0
    "spec": (True, 0, _lib.KARMA_WAL_CRC_PLAN),           # the uniform-stride pass tried on every call (KARMA_WAL_SPEC=2;
                                                          # the plan tries it unless the last try declined)
    "spec0": (True, 0, _lib.KARMA_WAL_CRC_PLAN),          # the plan with the uniform-stride pass off: the walk always
    "specnarrow": (True, 0, _lib.KARMA_WAL_CRC_PLAN),     # "spec" without the phased window loop (KARMA_SPEC_WIDE=0)
    "narrow": (True, 0, _lib.KARMA_WAL_CRC_PLAN),         # the walk's staged kernel without it (KARMA_STAGE_WIDE=0, pass off)
    "specnoal": (True, 0, _lib.KARMA_WAL_CRC_PLAN),       # "spec" without the dword-aligned fast path (KARMA_SPEC_AL=0)
}
_LIST_CRC = ("listcrc", "listcrc4k")  # KARMA_WAL_LIST_CRC=1
_NO_STAGED = ("sepdirect4",)  # KARMA_SMALL_STAGED=0
_R8 = ("r8",)  # KARMA_STAGE_R8=1
_SLICED = {"sliced": {"KARMA_WAL_SLICES": "2"},
           "sliced_r8": {"KARMA_WAL_SLICES": "2", "KARMA_STAGE_R8": "6", "KARMA_STAGE_SKEW": "0"},
           "rg0": {"KARMA_WAL_RG": "0"},
           "spec": {"KARMA_WAL_SPEC": "2"},
           "spec0": {"KARMA_WAL_SPEC": "0"},
           "specnarrow": {"KARMA_WAL_SPEC": "2", "KARMA_SPEC_WIDE": "0"},
           "narrow": {"KARMA_WAL_SPEC": "0", "KARMA_STAGE_WIDE": "0"},
           "specnoal": {"KARMA_WAL_SPEC": "2", "KARMA_SPEC_AL": "0"}}
_WALK = {"name": "split"}


def _walk_env(monkeypatch, walk):
    monkeypatch.setitem(_WALK, "name", walk)
    if walk in _LIST_CRC:
        monkeypatch.setenv("KARMA_WAL_LIST_CRC", "1")
    else:
        monkeypatch.delenv("KARMA_WAL_LIST_CRC", raising=False)
    if walk in _NO_STAGED:
        monkeypatch.setenv("KARMA_SMALL_STAGED", "0")
    else:
        monkeypatch.delenv("KARMA_SMALL_STAGED", raising=False)
    if walk in _R8:
        monkeypatch.setenv("KARMA_STAGE_R8", "1")
    else:
        monkeypatch.delenv("KARMA_STAGE_R8", raising=False)
    for k in ("KARMA_WAL_SLICES", "KARMA_STAGE_SKEW", "KARMA_WAL_RG", "KARMA_WAL_SPEC", "KARMA_SPEC_WIDE", "KARMA_STAGE_WIDE", "KARMA_SPEC_AL"):
        monkeypatch.delenv(k, raising=False)
    for k, v in _SLICED.get(walk, {}).items():
        monkeypatch.setenv(k, v)
    if WALKS[walk][0] and walk not in _LIST_CRC and walk not in _NO_STAGED and walk not in _R8 and walk not in _SLICED:
        monkeypatch.setenv("KARMA_WALK_VARIANT", "1")  # read by the tools build only (ab.h)
    else:
        monkeypatch.delenv("KARMA_WALK_VARIANT", raising=False)
    monkeypatch.delenv("KARMA_DIRECT_VARIANT", raising=False)


def _replay(lib, wal, start=0, d_wal=None, seg=SEG, host=True):
    """karma_wal_replay over the host image, or (host=False) over the device copy d_wal only, with
    the plan of the current walk (_walk_env)."""
    ab, sub, batch = WALKS[_WALK["name"]]
    L = _lib.load(_lib.AB_LIB_PATH) if ab else lib
    tuning = _lib.WalTuning(sub, batch, 0)
    n, stop, status = ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_int()
    rec = np.zeros(wal.nbytes // 8, np.uint64)
    st = L.karma_wal_replay_tuned(wal.ctypes.data if host else None, d_wal.data_ptr() if d_wal is not None else None,
                                  wal.nbytes, seg, start, ctypes.byref(n), ctypes.byref(stop), ctypes.byref(status),
                                  rec.ctypes.data, rec.size, 0, ctypes.byref(tuning))
    if st:
        raise _lib.KarmaError("karma_wal_replay_tuned", st, L.karma_crc32c_last_error().decode())
    return list(rec[: n.value]), stop.value, status.value


def test_append_matches_reference_framing(lib):
    src, offs, lens = _payloads(3, 3000, 1, 3000)
    wal = np.zeros(32 * SEG, np.uint8)
    cur, rec = _append(lib, src, offs, lens, wal)
    model = bytearray(32 * SEG)
    payloads = [src[int(o): int(o) + int(n)] for o, n in zip(offs, lens)]
    mcur, mrec = wal_model.append(payloads, model, SEG, 0)
    assert cur == mcur and list(rec) == mrec
    assert wal.tobytes() == bytes(model)


@pytest.mark.parametrize("call_bytes", [1, 20000, 1 << 20])
def test_append_in_several_passes_matches_reference_framing(call_bytes, monkeypatch):
    """A batch whose payload exceeds one pass (kCallBytes, 1 GiB in the shipped library; lowered
    here through the tools build's KARMA_APPEND_CALL_BYTES): the cursor, the record offsets and
    the image bytes carry across passes exactly as one pass over the model, including an image
    that fills up during a later pass."""
    monkeypatch.setenv("KARMA_APPEND_CALL_BYTES", str(call_bytes))
    ab = _lib.load(_lib.AB_LIB_PATH)
    src, offs, lens = _payloads(5, 4000, 1, 3000)
    for nseg in (200, 17):  # 17 segments: the image fills up after a few passes
        wal = np.zeros(nseg * SEG, np.uint8)
        for cursor in (0, 5 * SEG + 1000):
            if cursor:  # a writer resuming from a checkpoint: the image before the cursor as framed
                wal[:] = 0
            cur, rec = _append(ab, src, offs, lens, wal, cursor=cursor)
            model = bytearray(nseg * SEG)
            payloads = [src[int(o): int(o) + int(n)] for o, n in zip(offs, lens)]
            mcur, mrec = wal_model.append(payloads, model, SEG, cursor)
            assert cur == mcur and list(rec) == mrec, (call_bytes, nseg, cursor)
            assert wal.tobytes() == bytes(model), (call_bytes, nseg, cursor)
            assert (len(rec) == lens.size) == (nseg == 200)
            # the same into a page-locked image: each pass DMAs its framed image spans (no pack copy)
            pw = torch.zeros(wal.nbytes, dtype=torch.uint8).pin_memory().numpy()
            cur2, rec2 = _append(ab, src, offs, lens, pw, cursor=cursor)
            assert cur2 == mcur and list(rec2) == mrec, ("pinned", call_bytes, nseg, cursor)
            assert pw.tobytes() == bytes(model), ("pinned", call_bytes, nseg, cursor)


@pytest.mark.parametrize("mix", ["small", "mixed", "large"])
def test_append_into_pinned_image_matches_pageable(lib, mix):
    """A page-locked image (a writer's own buffer): append gives the pageable image's bytes and the
    model's (segment footers, padding records, records > 1 KiB, an image that fills up, a pass
    from a checkpoint cursor); replay from the pinned image (one DMA, no staging copies) gives
    the pageable image's result."""
    if mix == "small":
        src, offs, lens = _payloads(41, 30000, 1, 300)
    elif mix == "mixed":
        src, offs, lens = _payloads(42, 6000, 1, 6000)
    else:
        src, offs, lens = _payloads(43, 600, 1000, 60000)
    seg = SEG if mix != "large" else 256 << 10
    # every segment loses less than one record to its footer
    nseg = int((lens.astype(np.int64) + 8).sum() // (seg - int(lens.max()) - 8)) + 2
    for cut in (0, nseg // 2):  # cut: an image too small (not every record fits)
        wal = np.zeros((nseg - cut) * seg, np.uint8)
        cur, rec = _append(lib, src, offs, lens, wal, seg=seg)
        pinned = torch.zeros(wal.nbytes, dtype=torch.uint8).pin_memory()
        pw = pinned.numpy()
        cur2, rec2 = _append(lib, src, offs, lens, pw, seg=seg)
        assert cur2 == cur and list(rec2) == list(rec)
        assert np.array_equal(pw, wal)
        assert (len(rec) == lens.size) == (cut == 0)
        if cut == 0:
            want = wal_model.replay(pw.tobytes(), seg)
            assert want[0] == list(rec)
        # replay from the pinned image (one DMA, no staging) == from the pageable one
        for start in (0, int(rec[len(rec) // 3])):
            assert _replay(lib, pw, start=start, seg=seg) == _replay(lib, wal, start=start, seg=seg)
        # appended to from a checkpoint cursor (the pass starts mid-image)
        k = len(rec) // 2
        pw2 = pw.copy()
        pw2[int(rec[k]):] = 0
        p2 = torch.from_numpy(pw2).pin_memory()
        cur3, rec3 = _append(lib, src, offs[k:], lens[k:], p2.numpy(), cursor=int(rec[k]), seg=seg)
        assert cur3 == cur and list(rec3) == list(rec[k:])
        assert np.array_equal(p2.numpy(), wal)


def test_replay_round_trip_and_zero_tail(lib):
    src, offs, lens = _payloads(5, 4000, 1, 2000)
    wal = np.zeros(64 * SEG, np.uint8)
    cur, rec = _append(lib, src, offs, lens, wal)
    got = _replay(lib, wal)
    want = wal_model.replay(wal.tobytes(), SEG)
    assert got == (list(want[0]), want[1], want[2])
    # every framed record replays; replay ends at the never-written zero tail, which the
    # reference reports as "Corrupt record" (size-0 quirk), i.e. the writer resumes at the cursor
    assert got[0] == list(rec) and got[1] == cur and got[2] == wal_model.CORRUPT
    # same through a device copy of the image, with and without the host image
    d = torch.from_numpy(wal).cuda()
    assert _replay(lib, wal, d_wal=d) == got
    assert _replay(lib, wal, d_wal=d, host=False) == got


@pytest.mark.parametrize("what", ["payload_bit", "crc_field", "length_past_segment", "bad_type", "empty_record"])
def test_replay_stops_where_scan_record_does(lib, what):
    src, offs, lens = _payloads(7, 2500, 1, 2500)
    wal = np.zeros(48 * SEG, np.uint8)
    cur, rec = _append(lib, src, offs, lens, wal)
    k = 1234
    h = int(rec[k])
    if what == "payload_bit":
        wal[h + 8 + int(lens[k]) // 2] ^= 0x10
    elif what == "crc_field":
        wal[h] ^= 0x01
    elif what == "length_past_segment":
        wal[h + 4: h + 8] = np.frombuffer(np.uint32(((SEG) << 8) | 0).tobytes(), np.uint8)
    elif what == "bad_type":
        wal[h + 4] = 7
    else:  # an empty record as append_record writes it: crc Value("") = 0, len/type 0
        wal[h: h + 8] = 0
    got = _replay(lib, wal)
    want = wal_model.replay(wal.tobytes(), SEG)
    assert got == (list(want[0]), want[1], want[2])
    assert got[1] == h and len(got[0]) == k
    assert got[2] == (wal_model.BAD_TYPE if what == "bad_type" else wal_model.CORRUPT)


def test_replay_from_checkpoint_and_short_segment_tails(lib):
    # records sized so segments end with < 8 spare bytes (footer = '0' bytes only) and with padding records
    lens = np.array(([SEG // 2 - 8, SEG // 2 - 12] * 8) + [100] * 50, dtype=np.uint32)
    offs = np.concatenate([[0], np.cumsum(lens, dtype=np.uint64)[:-1]]).astype(np.uint64)
    src = synth.splitmix_np(11, 0, int(lens.sum()) + 16).copy()
    wal = np.zeros(16 * SEG, np.uint8)
    cur, rec = _append(lib, src, offs, lens, wal)
    for start in [0, int(rec[3]), int(rec[10])]:
        got = _replay(lib, wal, start=start)
        want = wal_model.replay(wal.tobytes(), SEG, start)
        assert got == (list(want[0]), want[1], want[2])


@pytest.mark.parametrize("walk", list(WALKS))
@pytest.mark.parametrize("seg", [(1 << 20), (64 << 10) + 12, 4096 + 4])
def test_replay_segment_sizes_tiles_and_misaligned_segments(lib, seg, walk, monkeypatch):
    """1 MiB segments (many LDS tiles of the device walk), and segment sizes that are not a
    multiple of 16 (every segment but the first is misaligned in the image: byte-wise tile loads);
    every walk kernel and sub-range split."""
    _walk_env(monkeypatch, walk)
    n = 6000 if seg >= (64 << 10) else 600
    src, offs, lens = _payloads(13, n, 1, min(3000, seg - 8))
    nseg = int((lens.astype(np.int64) + 8).sum() // seg) + 3
    wal = np.zeros(nseg * seg, np.uint8)
    cur, rec = _append(lib, src, offs, lens, wal, seg=seg)
    want = wal_model.replay(wal.tobytes(), seg)
    d = torch.from_numpy(wal).cuda()
    for kw in ({}, {"d_wal": d, "host": False}):
        got = _replay(lib, wal, seg=seg, **kw)
        assert got == (list(want[0]), want[1], want[2])
    assert want[0] == list(rec)
    # replay from checkpoints that fall in different sub-ranges of a segment
    for k in (1, len(rec) // 3, len(rec) // 2 + 7):
        got = _replay(lib, wal, start=int(rec[k]), seg=seg)
        w = wal_model.replay(wal.tobytes(), seg, int(rec[k]))
        assert got == (list(w[0]), w[1], w[2])
    # a flipped payload byte deep in the image: replay stops at that record
    k = len(rec) * 3 // 4
    wal[int(rec[k]) + 8] ^= 0x40
    got = _replay(lib, wal, seg=seg)
    assert got[2] == wal_model.CORRUPT and got[1] == int(rec[k]) and len(got[0]) == k
    # a broken length field: a structural stop inside a later sub-range
    wal[int(rec[k]) + 8] ^= 0x40
    j = len(rec) * 5 // 6
    wal[int(rec[j]) + 7] = 0x7F
    got = _replay(lib, wal, seg=seg)
    w = wal_model.replay(wal.tobytes(), seg)
    assert got == (list(w[0]), w[1], w[2])


@pytest.mark.parametrize("walk", list(WALKS))
@pytest.mark.parametrize("seg", [(1 << 20), (256 << 10) + 4])
def test_replay_large_records_jumps(lib, seg, walk, monkeypatch):
    """configs[2]-like payloads (log-uniform 1 B-60 KiB): the walk jumps past its prefetched
    tile and reads 1 KiB windows at the headers (byte-wise in misaligned segments), and goes
    back to tiles where records are short."""
    _walk_env(monkeypatch, walk)
    lens = synth.loguniform_lengths(17, 900, 1, 60000)
    offs = np.concatenate([[0], np.cumsum(lens, dtype=np.uint64)[:-1]]).astype(np.uint64)
    src = synth.splitmix_np(18, 0, int(lens.sum()) + 16).copy()
    nseg = int((lens.astype(np.int64) + 8).sum() // seg) + 3
    wal = np.zeros(nseg * seg, np.uint8)
    cur, rec = _append(lib, src, offs, lens, wal, seg=seg)
    want = wal_model.replay(wal.tobytes(), seg)
    assert want[0] == list(rec)
    d = torch.from_numpy(wal).cuda()
    for kw in ({}, {"d_wal": d, "host": False}):
        got = _replay(lib, wal, seg=seg, **kw)
        assert got == (list(want[0]), want[1], want[2])
    for k in (3, len(rec) // 2):
        got = _replay(lib, wal, start=int(rec[k]), seg=seg)
        w = wal_model.replay(wal.tobytes(), seg, int(rec[k]))
        assert got == (list(w[0]), w[1], w[2])


@pytest.mark.parametrize("walk", ["split", "split4k", "sep", "inline", "inline4k", "listcrc", "listcrc4k", "rg0"])
def test_replay_payloads_that_look_like_wal_records(lib, walk, monkeypatch):
    """Payloads that are themselves WAL images (valid header chains inside records): a sub-range
    walker can start on a header inside a payload, and the resolver must then walk the sub-range
    itself.  The result must still be scan_record's."""
    _walk_env(monkeypatch, walk)
    seg = 256 << 10
    inner_src, inner_offs, inner_lens = _payloads(31, 400, 1, 200)
    inner = np.zeros(64 << 10, np.uint8)
    _append(lib, inner_src, inner_offs, inner_lens, inner, seg=64 << 10)
    rng = np.random.default_rng(3)
    chunks, lens = [], []
    for i in range(300):  # alternate fake-WAL payloads (slices of the inner image) and random ones
        if i % 2 == 0:
            a = int(rng.integers(0, 4096))
            n = int(rng.integers(2000, 12000))
            chunks.append(inner[a: a + n])
        else:
            n = int(rng.integers(1, 3000))
            chunks.append(rng.integers(0, 256, n, dtype=np.uint8))
        lens.append(n)
    lens = np.array(lens, np.uint32)
    src = np.concatenate(chunks + [np.zeros(16, np.uint8)])
    offs = np.concatenate([[0], np.cumsum(lens, dtype=np.uint64)[:-1]]).astype(np.uint64)
    nseg = int((lens.astype(np.int64) + 8).sum() // seg) + 2
    wal = np.zeros(nseg * seg, np.uint8)
    cur, rec = _append(lib, src, offs, lens, wal, seg=seg)
    want = wal_model.replay(wal.tobytes(), seg)
    assert want[0] == list(rec)
    d = torch.from_numpy(wal).cuda()
    for kw in ({}, {"d_wal": d, "host": False}):
        got = _replay(lib, wal, seg=seg, **kw)
        assert got == (list(want[0]), want[1], want[2])
    for k in (5, 101, 222):
        got = _replay(lib, wal, start=int(rec[k]), seg=seg)
        w = wal_model.replay(wal.tobytes(), seg, int(rec[k]))
        assert got == (list(w[0]), w[1], w[2])


def test_replay_empty_and_start_at_end(lib):
    wal = np.zeros(4 * SEG, np.uint8)
    got = _replay(lib, wal)
    want = wal_model.replay(wal.tobytes(), SEG)
    assert got == (list(want[0]), want[1], want[2])
    assert _replay(lib, wal, start=wal.nbytes) == ([], wal.nbytes, wal_model.END)


def test_replay_dir_matches_image_replay(lib, tmp_path):
    """Segment files on disk, named by their WAL offsets (wal::load_from_path): replay of the
    directory equals replay of the image, with WAL offsets shifted by the first segment's."""
    seg = 64 << 10
    src, offs, lens = _payloads(41, 3000, 1, 2000)
    nseg = int((lens.astype(np.int64) + 8).sum() // seg) + 2
    wal = np.zeros(nseg * seg, np.uint8)
    cur, rec = _append(lib, src, offs, lens, wal, seg=seg)
    first = 7 * seg  # the directory's WAL starts at offset 7 segments (older segments deleted)
    for i in range(nseg):
        (tmp_path / str(first + i * seg)).write_bytes(wal[i * seg:(i + 1) * seg].tobytes())
    (tmp_path / "LOCK").write_bytes(b"")  # not a segment
    want = wal_model.replay(wal.tobytes(), seg)
    for start in (0, int(rec[100]), int(rec[2000])):
        w = wal_model.replay(wal.tobytes(), seg, start)
        base, n, stop, status = ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_int()
        got = np.zeros(wal.nbytes // 8, np.uint64)
        _lib.check("karma_wal_replay_dir",
                   lib.karma_wal_replay_dir(str(tmp_path).encode(), 0, first + start, ctypes.byref(base),
                                            ctypes.byref(n), ctypes.byref(stop), ctypes.byref(status), got.ctypes.data,
                                            got.size, 0))
        assert base.value == first
        assert [int(x) - first for x in got[: n.value]] == list(w[0])
        assert (stop.value - first, status.value) == (w[1], w[2])
    assert want[0] == list(rec)


@pytest.mark.parametrize("walk", ["split", "whole"])
def test_replay_exact_fills_tiny_tails_and_max_records(lib, walk, monkeypatch):
    """Records that fill a segment exactly, segment tails of 0-9 bytes (shorter than a header:
    '0' bytes, no footer), and a payload of 2^24 - 1 bytes (the 3-byte size field's maximum) in
    32 MiB segments.  (A size-0 record ends replay: the reference's stale-word quirk, tested in
    test_replay_stops_where_scan_record_does.)"""
    _walk_env(monkeypatch, walk)
    seg = 4096
    lens = []
    for tail in range(10):  # first record leaves `tail` bytes after a second one
        a = 2000
        lens += [a, seg - 8 - a - 8 - tail]
    lens += [seg - 8, 1, 7, seg - 8]
    lens = np.array(lens, np.uint32)
    offs = np.concatenate([[0], np.cumsum(lens, dtype=np.uint64)[:-1]]).astype(np.uint64)
    src = synth.splitmix_np(61, 0, int(lens.sum()) + 16).copy()
    wal = np.zeros(40 * seg, np.uint8)
    cur, rec = _append(lib, src, offs, lens, wal, seg=seg)
    want = wal_model.replay(wal.tobytes(), seg)
    assert want[0] == list(rec)
    assert _replay(lib, wal, seg=seg) == (list(want[0]), want[1], want[2])
    # the largest record the format can hold
    seg = 32 << 20
    lens = np.array([(1 << 24) - 1, 5, 1, 100000], np.uint32)
    offs = np.concatenate([[0], np.cumsum(lens, dtype=np.uint64)[:-1]]).astype(np.uint64)
    src = synth.splitmix_np(62, 0, int(lens.sum()) + 16).copy()
    wal = np.zeros(2 * seg, np.uint8)
    cur, rec = _append(lib, src, offs, lens, wal, seg=seg)
    want = wal_model.replay(wal.tobytes(), seg)
    assert want[0] == list(rec) and len(rec) == 4
    assert _replay(lib, wal, seg=seg) == (list(want[0]), want[1], want[2])


def test_replay_randomized_against_model(lib, monkeypatch):
    """Random images: segment sizes, record-size mixes (tiny, medium, large, WAL-looking payloads),
    a random corruption, a random start; every walk kernel and sub-range size against the model."""
    rng = np.random.default_rng(2024)
    inner = np.zeros(64 << 10, np.uint8)
    isrc, ioffs, ilens = _payloads(71, 600, 1, 100)
    _append(lib, isrc, ioffs, ilens, inner, seg=64 << 10)
    for case in range(12):
        seg = int(rng.choice([4096, 16384 + 4, 65536, 262144, 1 << 20]))
        mix = case % 4
        n = int(rng.integers(200, 3000))
        if mix == 0:
            lens = rng.integers(1, 64, n)
        elif mix == 1:
            lens = rng.integers(1, min(4000, seg - 8), n)
        elif mix == 2:
            lens = np.minimum(synth.loguniform_lengths(case, n, 1, 60000), seg - 8)
        else:
            lens = rng.integers(100, min(6000, seg - 8), n)
        lens = lens.astype(np.uint32)
        if mix == 3:  # payloads cut from a WAL image: header chains inside records
            src = np.concatenate([inner[int(rng.integers(0, 2048)):][: int(x)] if x <= inner.size - 2048 else
                                  rng.integers(0, 256, int(x), dtype=np.uint8) for x in lens] + [np.zeros(16, np.uint8)])
        else:
            src = rng.integers(0, 256, int(lens.sum()) + 16, dtype=np.uint8)
        offs = np.concatenate([[0], np.cumsum(lens, dtype=np.uint64)[:-1]]).astype(np.uint64)
        nseg = int((lens.astype(np.int64) + 8).sum() // seg) + 3
        wal = np.zeros(nseg * seg, np.uint8)
        cur, rec = _append(lib, src, offs, lens, wal, seg=seg)
        if case % 3 == 1 and len(rec) > 10:  # a flipped payload or length byte somewhere
            k = int(rng.integers(1, len(rec)))
            wal[int(rec[k]) + int(rng.choice([5, 8]))] ^= 0x10
        start = int(rec[int(rng.integers(0, len(rec)))]) if case % 2 and len(rec) else 0
        want = wal_model.replay(wal.tobytes(), seg, start)
        for walk in ("whole", "split", "split4k", "inline", "inline4k", "listcrc4k"):
            _walk_env(monkeypatch, walk)
            got = _replay(lib, wal, start=start, seg=seg)
            assert got == (list(want[0]), want[1], want[2]), (case, walk, seg, mix)


@pytest.mark.parametrize("walk", ["whole", "split", "split4k", "inline", "listcrc", "r8", "sliced", "sliced_r8", "rg0",
                                  "spec", "spec0", "specnarrow", "narrow", "specnoal"])
@pytest.mark.parametrize("seg", [4096 + 4, 65536, 1 << 20])
def test_replay_uniform_runs_speculative_walk(lib, seg, walk, monkeypatch):
    """Runs of one record size (the walker reads a round of headers at the last stride, lane j at
    pos + j * stride, and takes every header up to the first size change): run lengths 1..300,
    sizes from 1 B to a tile and beyond, runs that cross tiles, windows and segments; then a bad
    type, a length bit and an empty record in the middle of a run, where the round must stop at
    exactly that header."""
    _walk_env(monkeypatch, walk)
    rng = np.random.default_rng(seg + len(walk))
    sizes = [1, 7, 8, 24, 180, 1000, 4088, 5000]
    lens = []
    while len(lens) < 12000:
        size = int(rng.choice(sizes))
        lens += [min(size, seg - 8)] * int(rng.integers(1, 301 if size < 1000 else 20))
    lens = np.array(lens, np.uint32)
    offs = np.concatenate([[0], np.cumsum(lens, dtype=np.uint64)[:-1]]).astype(np.uint64)
    src = synth.splitmix_np(seg, 0, int(lens.sum()) + 16).copy()
    nseg = int((lens.astype(np.int64) + 8).sum() // (seg - 4096) + 3)
    wal = np.zeros(nseg * seg, np.uint8)
    cur, rec = _append(lib, src, offs, lens, wal, seg=seg)
    want = wal_model.replay(wal.tobytes(), seg)
    assert want[0] == list(rec)
    assert _replay(lib, wal, seg=seg) == (list(want[0]), want[1], want[2])
    runs = np.nonzero((lens[1:-1] == lens[:-2]) & (lens[1:-1] == lens[2:]))[0] + 1  # inside a run
    for what in ("bad_type", "length_bit", "empty"):
        bad = wal.copy()
        k = int(runs[int(rng.integers(0, runs.size))])
        h = int(rec[k])
        if what == "bad_type":
            bad[h + 4] = 3
        elif what == "length_bit":
            bad[h + 5] ^= 0x01
        else:
            bad[h: h + 8] = 0
        w = wal_model.replay(bad.tobytes(), seg)
        assert len(w[0]) == k
        assert _replay(lib, bad, seg=seg) == (list(w[0]), w[1], w[2]), what


@pytest.mark.parametrize("nseg", [1000, 1024, 1025, 3000])
def test_replay_segment_counts_around_the_fused_plan(lib, nseg):
    """Up to 1024 segments the device-planned gather reduces the segments' metas itself; above, a
    separate k_wal_plan launch does (wal.cc).  Both must give scan_record's result, from the start,
    from a checkpoint, and with a corrupted record."""
    seg = 4096
    src, offs, lens = _payloads(nseg, nseg * 14, 1, 300)
    wal = np.zeros(nseg * seg, np.uint8)
    cur, rec = _append(lib, src, offs, lens, wal, seg=seg)
    for start in (0, int(rec[len(rec) // 3])):
        got = _replay(lib, wal, start=start, seg=seg)
        w = wal_model.replay(wal.tobytes(), seg, start)
        assert got == (list(w[0]), w[1], w[2])
    k = len(rec) * 2 // 3
    wal[int(rec[k]) + 8] ^= 1  # a payload bit: replay stops at record k ("Corrupt record")
    got = _replay(lib, wal, seg=seg)
    w = wal_model.replay(wal.tobytes(), seg)
    assert got == (list(w[0]), w[1], w[2]) and len(got[0]) == k


@pytest.mark.parametrize("walk", list(WALKS))
@pytest.mark.parametrize("seg", [65536, 16384 + 4, 1 << 20])
def test_replay_accepted_size0_records_advance_12(lib, seg, walk, monkeypatch):
    """An empty record whose stored CRC is Value("\\0\\0\\0\\0") = 0x48674BC7 passes scan_record's
    stale-word check (wal.cc:47-60) and is returned 12 bytes long (wal.cc:66); sivir::open then
    reads the next header 12 bytes on (sivir.cc:38), into the next segment when the record sits in
    a segment's last 11 bytes, and past the image end at the last segment (tests/wal_images.py
    stale_empty: such records mid-run, around every tile / sub-range edge, at seg-8..seg-13 and at
    the image end).  Every walk plan must give scan_record's result, from the start and from
    checkpoints on such records, over the host image and the device copy alone."""
    import wal_images
    _walk_env(monkeypatch, walk)
    nseg = 3 if seg == (1 << 20) else 6
    spills = 0
    for seed in range(3):
        wal, heads = wal_images.stale_empty(seg, nseg, seed * 7 + (seg & 0xFF) + len(walk))
        w = wal_model.replay(wal.tobytes(), seg)
        assert w[0] == heads[: len(w[0])]
        zs = [h for h in w[0] if int.from_bytes(wal[h + 4: h + 8].tobytes(), "little") == 0]
        assert zs, "the image must hold accepted size-0 records"
        spills += sum(1 for h in zs if h % seg + 12 > seg)
        assert _replay(lib, wal, seg=seg) == (list(w[0]), w[1], w[2])
        d = torch.from_numpy(wal).cuda()
        assert _replay(lib, wal, d_wal=d, host=False, seg=seg) == (list(w[0]), w[1], w[2])
        for start in (zs[len(zs) // 2], zs[-1], zs[-1] + 12 if zs[-1] + 12 <= wal.size else zs[-1]):
            ws = wal_model.replay(wal.tobytes(), seg, start)
            assert _replay(lib, wal, start=start, seg=seg) == (list(ws[0]), ws[1], ws[2]), start
        # a stop past the image end (a size-0 record in the last 11 bytes) is a valid start:
        # replaying from it finds nothing (sivir::open's next scan_record returns false)
        for past in range(1, 5):
            assert _replay(lib, wal, start=wal.size + past, seg=seg) == ([], wal.size + past, 0)
    assert spills > 0, "some size-0 record must carry the chain into the next segment"


@pytest.mark.parametrize("walk", ["split", "sep", "split4k", "r8", "sliced", "rg0", "spec", "spec0", "narrow"])
def test_replay_size_class_changes_between_calls(lib, walk, monkeypatch):
    """The device-planned replay launches one small-record kernel, chosen by the largest payload of
    the previous call on the same device (the staged kernel up to 183 B, the 4-lane kernel up to
    1 KiB); a call whose payloads that kernel does not cover runs the batch again.  Every
    transition between the classes (<= 183 B, 184 B-1 KiB, larger, and a WAL with no record), with
    and without a corrupt payload, must give scan_record's result."""
    _walk_env(monkeypatch, walk)
    seg = 64 << 10
    wals = {}
    for name, lo, hi, seed in (("small", 1, 183, 81), ("edge", 170, 200, 82), ("mid", 184, 1024, 83),
                               ("large", 100, 6000, 84)):
        src, offs, lens = _payloads(seed, 1500, lo, hi)
        nseg = int((lens.astype(np.int64) + 8).sum() // (seg - 6100)) + 2
        wal = np.zeros(nseg * seg, np.uint8)
        cur, rec = _append(lib, src, offs, lens, wal, seg=seg)
        assert len(rec) == lens.size
        bad = wal.copy()
        k = 1000
        bad[int(rec[k]) + 8 + int(lens[k]) // 2] ^= 0x40
        wals[name] = wal
        wals[name + "_bad"] = bad
    wals["empty"] = np.zeros(4 * seg, np.uint8)
    want = {k: wal_model.replay(w.tobytes(), seg) for k, w in wals.items()}
    order = ["small", "small_bad", "mid", "mid_bad", "small", "mid", "large", "small_bad", "edge", "edge_bad",
             "mid", "large_bad", "mid_bad", "empty", "small", "edge", "small", "mid", "small"]
    dev = {k: torch.from_numpy(w).cuda() for k, w in wals.items()}
    for i, name in enumerate(order):
        w = want[name]
        got = _replay(lib, wals[name], d_wal=dev[name], seg=seg, host=bool(i % 2))
        assert got == (list(w[0]), w[1], w[2]), (i, name, walk)


@pytest.mark.parametrize("walk", ["split", "sep", "r8", "sliced", "rg0", "spec", "spec0"])
def test_replay_stage_skew_hint_between_calls(lib, walk, monkeypatch):
    """The staged small-record kernel comes in two forms, with the bank-skewed stage (records on
    few LDS banks: strides that are multiples of 32 bytes) and without it; a call takes the form
    the previous call's records asked for, and a plain stage over bank-poor records is slower but
    exact.  Uniform 120-B payloads (128-B stride: every record on one bank), 180-B (188-B stride)
    and 56-B (64-B stride) WALs in every order, with a corrupt payload, against the model."""
    _walk_env(monkeypatch, walk)
    seg = 64 << 10
    wals, want = {}, {}
    for size in (120, 180, 56):
        n = 4000
        lens = np.full(n, size, np.uint32)
        offs = (np.arange(n, dtype=np.uint64) * size).astype(np.uint64)
        src = synth.splitmix_np(size, 0, n * size + 16).copy()
        nseg = n * (size + 8) // (seg - 256) + 2
        wal = np.zeros(nseg * seg, np.uint8)
        cur, rec = _append(lib, src, offs, lens, wal, seg=seg)
        assert len(rec) == n
        bad = wal.copy()
        bad[int(rec[2345]) + 8 + size // 3] ^= 0x08
        for name, img in ((f"{size}", wal), (f"{size}_bad", bad)):
            wals[name] = img
            want[name] = wal_model.replay(img.tobytes(), seg)
    dev = {k: torch.from_numpy(w).cuda() for k, w in wals.items()}
    order = ["180", "120", "120", "180", "120_bad", "56", "180_bad", "120", "56_bad", "180", "180", "120"]
    for i, name in enumerate(order):
        w = want[name]
        assert _replay(lib, wals[name], d_wal=dev[name], seg=seg, host=False) == (list(w[0]), w[1], w[2]), (i, name)


@pytest.mark.parametrize("walk", ["sliced", "sliced_r8", "rg0"])
@pytest.mark.parametrize("nseg", [2, 7, 40])
def test_replay_sliced_pass_every_stop(lib, walk, nseg, monkeypatch):
    """The tools build's sliced pass (wal.cc sliced_pass: slice 1's walk beside slice 0's staged
    CRCs): small payloads (<= 180 B, so the previous call's hint takes the sliced path), replayed
    twice each, from the start and from checkpoints in either slice, with every kind of stop in
    either slice -- a corrupt payload, a bad type, a zero tail (the never-written rest) ending
    slice 0 early (slice 1's work is then speculative and must not count) -- against the model."""
    _walk_env(monkeypatch, walk)
    seg = 16 << 10
    n = nseg * seg // 100
    src, offs, lens = _payloads(nseg + len(walk), n, 1, 180)
    wal = np.zeros(nseg * seg, np.uint8)
    cur, rec = _append(lib, src, offs, lens, wal, seg=seg)
    h = [int(x) for x in rec]
    half = (nseg + 1) // 2 * seg  # slice 1's first byte
    in0 = [i for i, x in enumerate(h) if x < half]
    in1 = [i for i, x in enumerate(h) if x >= half]
    images = {"clean": wal}
    for name, k in (("bad0", in0[len(in0) // 2]), ("bad1", in1[len(in1) // 3] if in1 else None)):
        if k is None:
            continue
        img = wal.copy()
        img[h[k] + 8 + int(lens[k]) // 2] ^= 0x20
        images[name] = img
    img = wal.copy()
    img[h[in0[len(in0) // 3]] + 4] = 9
    images["badtype0"] = img
    img = wal.copy()
    img[h[in0[-5]]:half] = 0  # the WAL ends inside slice 0
    images["tail0"] = img
    d = {k: torch.from_numpy(v).cuda() for k, v in images.items()}
    for name, img in images.items():
        starts = [0, h[in0[len(in0) // 4]]] + ([h[in1[len(in1) // 2]]] if in1 else [])
        for start in starts:
            w = wal_model.replay(img.tobytes(), seg, start)
            for _ in range(2):  # (the first call may take the unsliced path: the previous call's hint)
                got = _replay(lib, img, start=start, seg=seg, d_wal=d[name], host=False)
                assert got == (list(w[0]), w[1], w[2]), (name, start)


@pytest.mark.parametrize("walk", ["split", "rg0"])
@pytest.mark.parametrize("nseg", [1, 2, 300, 1024])
def test_replay_resolve_gather_fused_many_segments(lib, nseg, walk, monkeypatch):
    """The one-launch resolve + gather (k_wal_resolve_gather, the plan's default; rg0: the tools
    build's two launches) over 1 to 1024 segments of 64 KiB (4 sub-range walkers each, so the
    resolve runs): every block's list offset comes from the earlier segments' tagged counts.  From
    the start, from a checkpoint, with a corrupted payload, with a bad type that stops replay in the
    first third (later blocks must gather nothing), and repeated calls (the call tag changes),
    against the model."""
    _walk_env(monkeypatch, walk)
    seg = 64 << 10
    src, offs, lens = _payloads(nseg + 3, nseg * 420, 1, 300)
    wal = np.zeros(nseg * seg, np.uint8)
    cur, rec = _append(lib, src, offs, lens, wal, seg=seg)
    d = torch.from_numpy(wal).cuda()
    for start in (0, int(rec[len(rec) // 3])):
        w = wal_model.replay(wal.tobytes(), seg, start)
        for _ in range(2):
            assert _replay(lib, wal, start=start, seg=seg, d_wal=d, host=False) == (list(w[0]), w[1], w[2])
    for what in ("payload", "type"):
        bad = wal.copy()
        k = len(rec) * 2 // 3 if what == "payload" else len(rec) // 3
        if what == "payload":
            bad[int(rec[k]) + 8] ^= 1
        else:
            bad[int(rec[k]) + 4] = 5
        w = wal_model.replay(bad.tobytes(), seg)
        assert len(w[0]) == k
        assert _replay(lib, bad, seg=seg) == (list(w[0]), w[1], w[2]), what


def _uniform_wal(lib, size, seg, n, seed):
    """n records of one payload size framed into segments (footers as append writes them), one
    never-written segment after them."""
    lens = np.full(n, size, np.uint32)
    offs = (np.arange(n, dtype=np.uint64) * size).astype(np.uint64)
    src = synth.splitmix_np(seed, 0, n * size + 16).copy()
    per = seg // (size + 8)
    wal = np.zeros(((n + per - 1) // per + 1) * seg, np.uint8)
    cur, rec = _append(lib, src, offs, lens, wal, seg=seg)
    assert len(rec) == n
    return wal, [int(x) for x in rec]


_SPEC_CASES = ([(4096 + 4, s) for s in (1, 3, 4, 5, 15, 16, 17, 56, 120, 180, 182, 183)] +
               [(65536, s) for s in (4, 17, 120, 180, 183)] + [(1 << 20, s) for s in (100, 180)] +
               # payloads over the staged kernel's gate: the 4-lane form (kSpecDirectMax)
               [(4096 + 4, s) for s in (184, 300)] + [(65536, s) for s in (500, 1000, 1024)] + [(1 << 20, 700)])


# (specnarrow: the staged kernel's sizes only, <= 183 B)
@pytest.mark.parametrize("seg,size,walk", [(g, z, "spec") for g, z in _SPEC_CASES] +
                         [(g, z, w) for g, z in _SPEC_CASES if z <= 183 for w in ("specnarrow", "specnoal")])
def test_replay_uniform_stride_pass(lib, seg, size, walk, monkeypatch):
    """The uniform-stride pass (engine.h WalSpec; tools build, KARMA_WAL_SPEC=2: tried on every call)
    over WALs of one payload size, up to 183 B (the staged kernel) and up to 1 KiB (the 4-lane one).  Its result is taken (karma_ab_wal_spec_last 1) for the zero tail
    after the last record (CORRUPT at the first unwritten header), segments filled to the image end
    (END), a corrupt payload or CRC field at a segment's first, middle or last slot, an empty record
    (all-zero header) and a zeroed padding header; it declines (2) and the walk decides for a changed
    length, a bad type, padding mid-segment, a size-0 record with the stale-word CRC (accepted, 12
    bytes), a length past the segment and a smaller record in a segment's tail; from checkpoints
    (records in segments 0-2) it is taken too.  Every result against the model, over the host image
    and the device copy.  specnarrow: the staged kernel without its phased window loop (KARMA_SPEC_WIDE=0)."""
    _walk_env(monkeypatch, walk)
    ab = _lib.load(_lib.AB_LIB_PATH)
    sig = size + 8
    per = seg // sig
    tail = seg - per * sig
    n = per * 3 + per // 2
    wal, h = _uniform_wal(lib, size, seg, n, seed=size * 7 + seg)
    # (a first call leaves this size class's hint: a pass whose kernel is the other class's reports 3)
    _replay(lib, wal, seg=seg)
    assert ab.karma_ab_wal_spec_last() in (1, 3)

    def check(img, spec, start=0, device=False):
        w = wal_model.replay(img.tobytes(), seg, start)
        got = _replay(lib, img, start=start, seg=seg)
        assert got == (list(w[0]), w[1], w[2]), (spec, start)
        assert ab.karma_ab_wal_spec_last() == spec
        if device:
            d = torch.from_numpy(img).cuda()
            assert _replay(lib, img, d_wal=d, host=False, seg=seg) == (list(w[0]), w[1], w[2])
            assert ab.karma_ab_wal_spec_last() == spec
        return w

    w = check(wal, 1, device=True)
    assert w[2] == wal_model.CORRUPT and len(w[0]) == n and w[1] == h[-1] + sig
    full = wal[: 3 * seg].copy()  # three full segments: END
    w = check(full, 1, device=True)
    assert w[2] == wal_model.END and len(w[0]) == 3 * per
    img = full.copy()  # ... with a corrupt payload and no other stop: every slot was checked
    img[h[per + 3] + 8] ^= 0x01
    w = check(img, 1)
    assert w[2] == wal_model.CORRUPT and len(w[0]) == per + 3
    img = full.copy()  # ... with a changed length and no stop: declined
    img[h[2 * per + 1] + 5] ^= 0x01
    check(img, 2)
    taken = {"payload_mid": (2 * per + per // 3, "payload"), "crc_first": (per, "crc"),
             "crc_last": (2 * per - 1, "crc"), "payload_first": (0, "payload"), "empty": (per + 7, "zero")}
    for name, (k, what) in taken.items():
        img = wal.copy()
        if what == "payload":
            img[h[k] + 8 + size // 2] ^= 0x20
        elif what == "crc":
            img[h[k]] ^= 0x01
        else:
            img[h[k]: h[k] + 8] = 0
        w = check(img, 1)
        assert w[2] == wal_model.CORRUPT and len(w[0]) == k, name
    if tail >= 8:  # segment 1's padding header zeroed: "Corrupt record" there
        img = wal.copy()
        img[seg + per * sig: seg + per * sig + 8] = 0
        w = check(img, 1)
        assert w[2] == wal_model.CORRUPT and w[1] == seg + per * sig and len(w[0]) == 2 * per
    k = per + per // 2
    declined = {"length": lambda img: img.__setitem__(h[k] + 5, img[h[k] + 5] ^ 0x01),
                "bad_type": lambda img: img.__setitem__(h[k] + 4, 3),
                "padding": lambda img: img.__setitem__(h[k] + 4, 1),
                "past_segment": lambda img: img.__setitem__(slice(h[k] + 4, h[k] + 8),
                                                            np.frombuffer(np.uint32(seg << 8).tobytes(), np.uint8)),
                "stale_empty": lambda img: img.__setitem__(slice(h[k], h[k] + 8),
                                                           np.frombuffer(np.array([0x48674BC7, 0], np.uint32).tobytes(),
                                                                         np.uint8))}
    for name, edit in declined.items():
        img = wal.copy()
        edit(img)
        check(img, 2)
    if tail >= 9:  # a record of tail - 8 bytes fills segment 1's tail instead of the padding
        img = wal.copy()
        t = seg + per * sig
        body = synth.splitmix_np(5, 0, tail - 8).copy()
        import oracle_lib
        img[t: t + 8] = np.frombuffer(np.array([oracle_lib.extend(0, body.tobytes()), (tail - 8) << 8], np.uint32)
                                      .tobytes(), np.uint8)
        img[t + 8: t + tail] = body
        w = check(img, 2)
        assert t in w[0]
    # from checkpoints (sivir::open starts at the WAL's checkpoint, sivir.cc:31): a record in
    # segment 0, segment 0's last record, a record in segment 2, segment 1's first; a corrupt
    # payload after the checkpoint; a start inside a payload (decided either way, always exact)
    for k in (5, per - 1, 2 * per + per // 2, per):
        w = check(wal, 1, start=h[k])
        assert w[2] == wal_model.CORRUPT and len(w[0]) == n - k
    img = wal.copy()
    img[h[per + 9] + 8] ^= 0x04
    w = check(img, 1, start=h[per // 2])
    assert w[2] == wal_model.CORRUPT and w[1] == h[per + 9]
    for start in (h[7] + 3, h[per + 2] + 8):
        w = wal_model.replay(wal.tobytes(), seg, start)
        assert _replay(lib, wal, start=start, seg=seg) == (list(w[0]), w[1], w[2])
    check(wal, 1)  # and from the start again


@pytest.mark.parametrize("walk", ["split", "spec", "spec0"])
def test_replay_tiny_segments(lib, walk, monkeypatch):
    """Segments of 8-40 bytes (a header and a few payload bytes, or less): one record per segment
    or none, short rests, from the start and from every record; whatever path replay takes (the
    uniform-stride pass needs a header and a byte after the start), scan_record's result."""
    _walk_env(monkeypatch, walk)
    for seg in (8, 9, 10, 16, 17, 24, 40):
        for size in (1, 2, 7, 8, 16, 32):
            if size + 8 > seg:
                continue
            n = 12
            lens = np.full(n, size, np.uint32)
            offs = (np.arange(n, dtype=np.uint64) * size).astype(np.uint64)
            src = synth.splitmix_np(seg * 100 + size, 0, n * size + 16).copy()
            wal = np.zeros((n // max(1, seg // (size + 8)) + 2) * seg, np.uint8)
            cur, rec = _append(lib, src, offs, lens, wal, seg=seg)
            for start in [0] + [int(x) for x in rec[:4]]:
                w = wal_model.replay(wal.tobytes(), seg, start)
                assert _replay(lib, wal, start=start, seg=seg) == (list(w[0]), w[1], w[2]), (seg, size, start)
