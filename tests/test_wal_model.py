"""The WAL restatement itself (CPU): framing round-trips through replay, and the reference's
own end-of-log behaviour (zero tail -> "Corrupt record") holds."""
import struct

import numpy as np

import synth
import wal_model

SEG = 16 << 10


def test_model_round_trip():
    lens = synth.uniform_lengths(1, 400, 1, 1500)
    data = synth.splitmix(2, 0, int(lens.sum()))
    pos = np.concatenate([[0], np.cumsum(lens)[:-1]])
    payloads = [data[int(p): int(p) + int(n)] for p, n in zip(pos, lens)]
    wal = bytearray(64 * SEG)
    cur, offs = wal_model.append(payloads, wal, SEG, 0)
    recs, stop, status = wal_model.replay(bytes(wal), SEG)
    assert recs == offs and stop == cur and status == wal_model.CORRUPT


def test_model_empty_record_is_corrupt_on_replay():
    wal = bytearray(4 * SEG)
    cur, offs = wal_model.append([b"abc", b"", b"xyz"], wal, SEG, 0)
    recs, stop, status = wal_model.replay(bytes(wal), SEG)
    assert recs == offs[:1] and stop == offs[1] and status == wal_model.CORRUPT


def test_model_footer_kinds():
    wal = bytearray(2 * SEG)
    cur, offs = wal_model.append([b"a" * (SEG - 8 - 5), b"b" * 10], wal, SEG, 0)
    assert offs == [0, SEG] and wal[SEG - 5:SEG] == b"00000"  # < 8 spare bytes: '0' padding only
    wal = bytearray(2 * SEG)
    cur, offs = wal_model.append([b"a" * 100, b"b" * (SEG - 50)], wal, SEG, 0)
    assert offs == [0, SEG] and wal[108] == 0 and wal[112] == 1  # padding record: crc 0, type 1


def test_reference_append_harness_matches_model():
    """The config-1 CPU harness (oracle/ref_shim.cc, reference crc32c::Value) frames byte-for-byte
    what the model frames; bench.py times it as the wal_append cpu_baseline."""
    import oracle_lib
    ref = oracle_lib.ref()
    if ref is None:
        import pytest
        pytest.skip("oracle/_ref not built")
    lens = synth.uniform_lengths(3, 500, 1, 3000).astype(np.uint32)
    offs = np.concatenate([[0], np.cumsum(lens, dtype=np.uint64)[:-1]]).astype(np.uint64)
    src = synth.splitmix_np(4, 0, int(lens.sum()) + 8).copy()
    wal = np.zeros(64 * SEG, np.uint8)
    n = ref.ref_wal_append_mt(src.ctypes.data, offs.ctypes.data, lens.ctypes.data, lens.size, wal.ctypes.data,
                              wal.nbytes, SEG, 1)
    model = bytearray(64 * SEG)
    _, moffs = wal_model.append([src[int(o): int(o) + int(k)] for o, k in zip(offs, lens)], model, SEG, 0)
    assert n == len(moffs) and wal.tobytes() == bytes(model)
    # and the replay harness accepts exactly the records the model replays
    recs, _, _ = wal_model.replay(bytes(model), SEG)
    assert ref.ref_wal_replay_mt(wal.ctypes.data, wal.nbytes, SEG, 1, 1) == len(recs) == n


def test_spec_replay_is_scan_record_whenever_it_decides():
    """The uniform-stride pass's decision rule (wal_model.spec_replay, the CPU restatement of the
    SPEC form of k_ragged_staged_pipe and k_wal_spec_finish): over uniform WALs with random
    edits (flipped bytes, zeroed / retyped / resized headers, accepted size-0 records, zeroed
    rests, padding headers), WALs of mixed sizes and sizes past the stage gate, from the start, a
    record and an arbitrary byte, every result it takes equals the model's replay, and it takes the
    clean and the simply-corrupted ones."""
    rng = np.random.default_rng(77)
    taken = declined = 0
    taken_mid = [0]
    for case in range(400):
        seg = int(rng.choice([64, 100, 256, 1000, 4096]))
        size = int(rng.choice([1, 2, 5, 16, 20, 56, 100, 120, 183, 184, 300])) if case % 5 else 0
        if size + 8 > seg:
            continue
        nseg = int(rng.integers(1, 7))
        if size:
            per = seg // (size + 8)
            count = int(rng.integers(1, nseg * per + 1))
            lens = [size] * count
        else:  # mixed sizes
            lens = [int(x) for x in rng.integers(1, min(300, seg - 8) + 1, int(rng.integers(1, 200)))]
        data = synth.splitmix(case, 0, sum(lens) + 16)
        pos = np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.int64)
        wal = bytearray(nseg * seg)
        cur, offs = wal_model.append([data[int(p): int(p) + n] for p, n in zip(pos, lens)], wal, seg, 0)
        if case % 3 and offs:
            for _ in range(int(rng.integers(1, 3))):
                k = int(offs[int(rng.integers(0, len(offs)))])
                kind = int(rng.integers(0, 7))
                if kind == 0:
                    wal[int(rng.integers(0, max(cur, 1)))] ^= 1 << int(rng.integers(0, 8))
                elif kind == 1:
                    wal[k: k + 8] = bytes(8)
                elif kind == 2:
                    wal[k + 4] = int(rng.choice([1, 2, 9]))
                elif kind == 3:
                    wal[k + 5] ^= 1
                elif kind == 4:
                    wal[k: k + 8] = struct.pack("<II", 0x48674BC7, 0)
                elif kind == 5:
                    wal[k:] = bytes(len(wal) - k)
                else:
                    s = k // seg * seg
                    wal[s + seg - 8: s + seg] = bytes(8) if rng.integers(0, 2) else struct.pack("<II", 0, (0 << 8) | 1)
        # from the start, from a record (a checkpoint) and from an arbitrary byte
        starts = [0]
        if offs:
            starts += [int(offs[int(rng.integers(0, len(offs)))]), int(rng.integers(0, len(wal)))]
        for start in starts:
            got = wal_model.spec_replay(bytes(wal), seg, start)
            if got is None:
                declined += 1
                continue
            taken += 1
            if start:
                taken_mid[0] += 1
            assert got == wal_model.replay(bytes(wal), seg, start), (case, seg, size, start)
    assert taken > 200 and declined > 100 and taken_mid[0] > 50, (taken, declined, taken_mid)
