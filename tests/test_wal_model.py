"""The WAL restatement itself (CPU): framing round-trips through replay, and the reference's
own end-of-log behaviour (zero tail -> "Corrupt record") holds."""
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
