"""ctypes access to the CPU oracle (oracle/crc32c_port.c) -- test infrastructure only.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use this module.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PORT_SO = os.path.join(ROOT, "oracle", "_build", "libkarma_oracle.so")
REF_SO = os.path.join(ROOT, "oracle", "_ref", "libkarma_ref_crc32c.so")

_c = ctypes
_PORT = None
_REF = None


def _build():
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "port"], check=True)


def port():
    """The C restatement of karma-util/crc32c.cc (always buildable with gcc)."""
    global _PORT
    if _PORT is None:
        if not os.path.exists(PORT_SO):
            _build()
        L = ctypes.CDLL(PORT_SO)
        L.oracle_crc32c_extend.restype = _c.c_uint32
        L.oracle_crc32c_extend.argtypes = [_c.c_uint32, _c.c_void_p, _c.c_size_t]
        L.oracle_splitmix_fixed_crcs.restype = _c.c_int
        L.oracle_splitmix_fixed_crcs.argtypes = [_c.c_uint64, _c.c_uint64, _c.c_uint64, _c.c_uint64, _c.c_uint32,
                                                 _c.c_void_p, _c.c_int]
        L.oracle_ragged_crcs.restype = _c.c_int
        L.oracle_ragged_crcs.argtypes = [_c.c_void_p, _c.c_void_p, _c.c_void_p, _c.c_void_p, _c.c_uint64,
                                         _c.c_void_p, _c.c_int]
        L.oracle_fixed_crcs.restype = _c.c_int
        L.oracle_fixed_crcs.argtypes = [_c.c_void_p, _c.c_uint64, _c.c_uint64, _c.c_void_p, _c.c_int]
        L.oracle_splitmix_bytes.restype = None
        L.oracle_splitmix_bytes.argtypes = [_c.c_uint64, _c.c_uint64, _c.c_void_p, _c.c_size_t]
        _PORT = L
    return _PORT


def ref():
    """The reference's own crc32c.cc built by oracle/Makefile, or None when not shipped."""
    global _REF
    if _REF is None and os.path.exists(REF_SO):
        L = ctypes.CDLL(REF_SO)
        L.ref_crc32c_extend.restype = _c.c_uint32
        L.ref_crc32c_extend.argtypes = [_c.c_uint32, _c.c_void_p, _c.c_size_t]
        L.ref_crc32c_fixed_mt.restype = _c.c_int
        L.ref_crc32c_fixed_mt.argtypes = [_c.c_void_p, _c.c_uint64, _c.c_uint64, _c.c_void_p, _c.c_int]
        L.ref_wal_append_mt.restype = _c.c_uint64
        L.ref_wal_append_mt.argtypes = [_c.c_void_p, _c.c_void_p, _c.c_void_p, _c.c_uint64, _c.c_void_p, _c.c_uint64,
                                        _c.c_uint64, _c.c_int]
        L.ref_wal_replay_mt.restype = _c.c_uint64
        L.ref_wal_replay_mt.argtypes = [_c.c_void_p, _c.c_uint64, _c.c_uint64, _c.c_int, _c.c_int]
        L.ref_crc32c_ragged_mt.restype = _c.c_int
        L.ref_crc32c_ragged_mt.argtypes = [_c.c_void_p, _c.c_void_p, _c.c_void_p, _c.c_void_p, _c.c_uint64,
                                           _c.c_void_p, _c.c_int]
        _REF = L
    return _REF


def extend(init: int, data: bytes) -> int:
    buf = ctypes.create_string_buffer(data, len(data) + 1)
    return int(port().oracle_crc32c_extend(init & 0xFFFFFFFF, buf, len(data)))


def splitmix_fixed_crcs(seed: int, rec_bytes: int, first: int, n_rec: int, init: int = 0, threads: int = 8):
    out = np.empty(n_rec, dtype=np.uint32)
    port().oracle_splitmix_fixed_crcs(seed, rec_bytes, first, n_rec, init & 0xFFFFFFFF, out.ctypes.data, threads)
    return out


def ragged_crcs(arena: np.ndarray, off: np.ndarray, lens: np.ndarray, init=None, threads: int = 8):
    arena = np.ascontiguousarray(arena, dtype=np.uint8)
    off = np.ascontiguousarray(off, dtype=np.uint64)
    lens = np.ascontiguousarray(lens, dtype=np.uint32)
    ini = None if init is None else np.ascontiguousarray(init, dtype=np.uint32)
    out = np.empty(off.size, dtype=np.uint32)
    port().oracle_ragged_crcs(arena.ctypes.data, off.ctypes.data, lens.ctypes.data,
                              None if ini is None else ini.ctypes.data, off.size, out.ctypes.data, threads)
    return out


def fixed_crcs(buf: np.ndarray, rec_bytes: int, threads: int = 8):
    buf = np.ascontiguousarray(buf, dtype=np.uint8)
    n = buf.nbytes // rec_bytes
    out = np.empty(n, dtype=np.uint32)
    port().oracle_fixed_crcs(buf.ctypes.data, rec_bytes, n, out.ctypes.data, threads)
    return out
