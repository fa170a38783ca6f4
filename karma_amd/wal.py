"""WAL and KFP batch calls on numpy buffers (the C ABI of include/karma_crc32c.h).

Python mirror of the reference's loops that checksum through crc32c::Value / Extend:

* ``append``      -- sivir::build_sqe framing (segment_file::append_record / append_footer,
                     karma-store/segment_file.cc:21-49), CRCs of the batch in one GPU batch;
* ``replay``      -- sivir::open's wal::scan_record loop (karma-store/wal.cc:34-87) over an
                     image in host memory or in HBM;
* ``replay_dir``  -- the same over the directory wal::load_from_path opens (wal.cc:9-27);
* ``kfp_encode`` / ``kfp_parse`` -- transport::frame::encode / connection::read_frame's
                     frame::parse loop (karma-transport/frame.cc:41-130, connection.cc:20-27).

Every call needs the MI355X: without it the library returns KARMA_E_NO_DEVICE and these raise
(no CPU fallback).  Status codes: ``END`` / ``CORRUPT`` / ``BAD_TYPE`` for replay, the
``KFP_*`` constants for parsing.
"""
from __future__ import annotations

import ctypes
import os
from typing import NamedTuple, Optional

import numpy as np

from . import _lib

END, CORRUPT, BAD_TYPE = 0, 1, 2
KFP_OK, KFP_BAD_SIZE, KFP_BAD_MAGIC, KFP_BAD_HEADER_LEN, KFP_BAD_CRC, KFP_BAD_LENGTH = 0, 1, 2, 3, 4, 5


class Replay(NamedTuple):
    records: np.ndarray  # header offsets (WAL offsets) of the records sivir::open applies, in order
    stop: int            # where scan_record returned false: the writer resumes here
    status: int          # END / CORRUPT / BAD_TYPE


class Appended(NamedTuple):
    cursor: int          # the WAL offset after the last framed record
    records: np.ndarray  # header offset of each framed record
    framed: int          # records framed (the rest did not fit the image)


def _u8(a) -> np.ndarray:
    a = np.asarray(a)
    if not a.flags.c_contiguous:
        raise ValueError("buffers must be C-contiguous")
    return a.view(np.uint8).reshape(-1)


def _extents(payloads):
    lens = np.array([len(p) for p in payloads], dtype=np.uint32)
    offs = np.concatenate([[0], np.cumsum(lens, dtype=np.uint64)[:-1]]).astype(np.uint64) if len(payloads) else \
        np.zeros(0, np.uint64)
    src = np.frombuffer(b"".join(bytes(p) for p in payloads) + bytes(16), dtype=np.uint8)
    return src, offs, lens


def append(payloads, wal: np.ndarray, seg_bytes: int, cursor: int = 0, device: int = -1) -> Appended:
    """Frame ``payloads`` (a sequence of bytes-like) into ``wal`` (uint8, a whole number of
    segments) from ``cursor``; the image is updated in place."""
    w = _u8(wal)
    src, offs, lens = _extents(payloads)
    cur, nf = ctypes.c_uint64(cursor), ctypes.c_size_t()
    rec = np.zeros(lens.size, np.uint64)
    _lib.check("karma_wal_append_batch",
               _lib.lib().karma_wal_append_batch(src.ctypes.data, offs.ctypes.data, lens.ctypes.data, lens.size,
                                                 w.ctypes.data, w.nbytes, seg_bytes, ctypes.byref(cur),
                                                 rec.ctypes.data, ctypes.byref(nf), device))
    return Appended(cur.value, rec[: nf.value], nf.value)


def replay(wal=None, seg_bytes: int = 1 << 20, start: int = 0, d_wal=None, wal_bytes: Optional[int] = None,
           device: int = -1, walk_sub_bytes: int = 0, crc_batch: int = _lib.KARMA_WAL_CRC_PLAN) -> Replay:
    """sivir::open over an image: ``wal`` in host memory (numpy), or ``d_wal`` (a CUDA tensor)
    already in HBM.  ``walk_sub_bytes`` / ``crc_batch`` override the plan (karma_wal_tuning;
    the result is the same whatever the plan)."""
    h = _u8(wal) if wal is not None else None
    if wal_bytes is None:
        wal_bytes = h.nbytes if h is not None else d_wal.numel() * d_wal.element_size()
    n, stop, status = ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_int()
    rec = np.zeros(wal_bytes // 8 + 1, np.uint64)
    tuning = _lib.WalTuning(walk_sub_bytes, crc_batch, 0)
    _lib.check("karma_wal_replay",
               _lib.lib().karma_wal_replay_tuned(h.ctypes.data if h is not None else None,
                                                 d_wal.data_ptr() if d_wal is not None else None, wal_bytes,
                                                 seg_bytes, start, ctypes.byref(n), ctypes.byref(stop),
                                                 ctypes.byref(status), rec.ctypes.data, rec.size, device,
                                                 ctypes.byref(tuning)))
    return Replay(rec[: n.value].copy(), stop.value, status.value)


def replay_dir(path: str, seg_bytes: int = 0, start: Optional[int] = None, max_records: int = 1 << 24,
               device: int = -1) -> Replay:
    """sivir::open over a WAL directory: regular files named by the decimal WAL offset of their
    first byte (wal::load_from_path).  ``start`` defaults to the first segment's offset."""
    base, n, stop, status = ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_int()
    if start is None:
        names = [int(f) for f in os.listdir(path) if f.isdigit()]
        start = min(names) if names else 0
    rec = np.zeros(max_records, np.uint64)
    _lib.check("karma_wal_replay_dir",
               _lib.lib().karma_wal_replay_dir(str(path).encode(), seg_bytes, start, ctypes.byref(base),
                                               ctypes.byref(n), ctypes.byref(stop), ctypes.byref(status),
                                               rec.ctypes.data, rec.size, device))
    return Replay(rec[: min(n.value, rec.size)].copy(), stop.value, status.value)


class Encoded(NamedTuple):
    data: np.ndarray     # the encoded frames, back to back
    offsets: np.ndarray  # offset of each encoded frame
    n: int               # frames encoded (the rest did not fit)


class Parsed(NamedTuple):
    offsets: np.ndarray  # offsets of the accepted frames
    consumed: int        # bytes they occupy: where parsing stopped
    status: int          # KFP_*


def kfp_encode(frames, out_bytes: Optional[int] = None, device: int = -1) -> Encoded:
    """frame::encode for each (operation_code, flag, seq, header, payload) in ``frames``."""
    ops = np.array([f[0] for f in frames], np.int16)
    flags = np.array([f[1] for f in frames], np.uint8)
    seqs = np.array([f[2] for f in frames], np.uint32)
    hsrc, hoff, hlen = _extents([f[3] for f in frames])
    psrc, poff, plen = _extents([f[4] for f in frames])
    if out_bytes is None:
        out_bytes = int(hlen.sum()) + int(plen.sum()) + 20 * len(frames)
    out = np.zeros(out_bytes, np.uint8)
    foff = np.zeros(len(frames), np.uint64)
    ne, nb = ctypes.c_size_t(), ctypes.c_uint64()
    _lib.check("karma_kfp_encode_batch",
               _lib.lib().karma_kfp_encode_batch(hsrc.ctypes.data, hoff.ctypes.data, hlen.ctypes.data,
                                                 psrc.ctypes.data, poff.ctypes.data, plen.ctypes.data,
                                                 ops.ctypes.data, flags.ctypes.data, seqs.ctypes.data, len(frames),
                                                 out.ctypes.data, out.nbytes, foff.ctypes.data, ctypes.byref(ne),
                                                 ctypes.byref(nb), device))
    return Encoded(out[: nb.value], foff[: ne.value], ne.value)


def kfp_parse(buf, max_frames: int = 1 << 20, device: int = -1) -> Parsed:
    """connection::read_frame's loop over a receive buffer: frame::parse, advance, repeat."""
    b = _u8(buf)
    foff = np.zeros(max_frames, np.uint64)
    n, used, status = ctypes.c_size_t(), ctypes.c_uint64(), ctypes.c_int()
    _lib.check("karma_kfp_parse_batch",
               _lib.lib().karma_kfp_parse_batch(b.ctypes.data, None, b.nbytes, max_frames, foff.ctypes.data,
                                                ctypes.byref(n), ctypes.byref(used), ctypes.byref(status), device))
    return Parsed(foff[: n.value].copy(), used.value, status.value)
