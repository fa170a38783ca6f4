"""ctypes binding of libkarma_crc32c.so (the C ABI in include/karma_crc32c.h).

The shared library is built in-tree (``karma_amd/lib/``, see ``__graft_entry__.build``)
so it travels with the repository snapshot.  There is no fallback: if the library is
missing, importing the device entry points raises ``KarmaUnavailable``.
"""
from __future__ import annotations

import contextlib
import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "lib", "libkarma_crc32c.so")
# The tools build (karma_amd/csrc/ab.h): the same C ABI plus the A/B kernel variants of
# DESIGN.md §4, chosen by KARMA_* environment variables.  Only tools/ and the variant
# tests load it (through `using`); the package always runs LIB_PATH.
AB_LIB_PATH = os.path.join(os.path.dirname(_HERE), "tools", "lib", "libkarma_crc32c_ab.so")
# The bounds-checked debug build (karma_amd/csrc/bounds.h): the same C ABI plus
# karma_debug_bounds_report; the GPU suite runs on it under `pytest --karma-lib bounds`.
BOUNDS_LIB_PATH = os.path.join(os.path.dirname(_HERE), "tools", "lib", "libkarma_crc32c_bounds.so")
# The tools build with the bounds checks (`make abbounds`): `pytest --karma-lib abbounds` runs the
# variant tests on it (and the rest of the suite on BOUNDS_LIB_PATH).
ABBOUNDS_LIB_PATH = os.path.join(os.path.dirname(_HERE), "tools", "lib", "libkarma_crc32c_abbounds.so")
KB_SITES = {1: "WAL image byte outside the image", 2: "WAL image byte outside the walker's segment",
            3: "candidate slot outside the segment's lists", 4: "candidate write dropped by the cap guard",
            5: "sub-range report index", 6: "span index", 7: "segment meta index", 8: "gathered list index",
            9: "gathered slot outside its sub-range", 10: "record byte outside the arena allocation",
            11: "ragged unit slot >= unit_cap"}

KARMA_OK = 0
KARMA_E_INVALID = -1
KARMA_E_NO_DEVICE = -2
KARMA_E_HIP = -3
KARMA_E_NOMEM = -4
KARMA_E_RCCL = -5
KARMA_E_IO = -6
UNIQUE_ID_BYTES = 128

_c = ctypes
_vp, _sz, _u32, _u64, _i = _c.c_void_p, _c.c_size_t, _c.c_uint32, _c.c_uint64, _c.c_int

# name -> (restype, argtypes); mirrors include/karma_crc32c.h one to one
SIGNATURES = {
    "karma_crc32c_abi_version": (_i, []),
    "karma_crc32c_strerror": (_c.c_char_p, [_i]),
    "karma_crc32c_last_error": (_c.c_char_p, []),
    "karma_crc32c_extend_host": (_u32, [_u32, _vp, _sz]),
    "karma_crc32c_extend_host_portable": (_u32, [_u32, _vp, _sz]),
    "karma_crc32c_combine": (_u32, [_u32, _u32, _u64]),
    "karma_crc32c_batch_fixed": (_i, [_vp, _sz, _sz, _vp, _u32, _vp, _vp]),
    "karma_crc32c_batch_ragged": (_i, [_vp, _vp, _vp, _sz, _sz, _vp, _u32, _vp, _vp]),
    "karma_crc32c_batch_ragged_bounded": (_i, [_vp, _vp, _vp, _sz, _sz, _u32, _vp, _u32, _vp, _vp]),
    "karma_crc32c_stream": (_i, [_u32, _vp, _sz, _vp, _vp]),
    "karma_crc32c_release_stream": (_i, [_i, _vp]),
    "karma_crc32c_trim": (_i, [_i]),
    "karma_crc32c_graph_hold": (_i, [_i, _i]),
    "karma_crc32c_stream_states": (_i, []),
    "karma_crc32c_batch_fixed_host": (_i, [_vp, _sz, _sz, _u32, _vp, _i]),
    "karma_crc32c_batch_ragged_host": (_i, [_vp, _sz, _vp, _vp, _sz, _u32, _vp, _i]),
    "karma_crc32c_batch_fixed_host_multi": (_i, [_vp, _sz, _sz, _u32, _vp, _vp, _i]),
    "karma_crc32c_batch_ragged_host_multi": (_i, [_vp, _sz, _vp, _vp, _sz, _u32, _vp, _vp, _i]),
    "karma_wal_replay_multi": (_i, [_vp, _sz, _sz, _u64, _c.POINTER(_u64), _c.POINTER(_u64), _c.POINTER(_i), _vp, _sz,
                                    _vp, _i]),
    "karma_crc32c_get_unique_id": (_i, [_vp, _sz]),
    "karma_crc32c_comm_init": (_i, [_c.POINTER(_vp), _i, _vp, _i]),
    "karma_crc32c_comm_destroy": (_i, [_vp]),
    "karma_crc32c_comm_count": (_i, [_vp, _c.POINTER(_i)]),
    "karma_crc32c_gather_u32": (_i, [_vp, _vp, _sz, _vp, _i, _vp]),
    "karma_crc32c_batch_fixed_sharded": (_i, [_vp, _vp, _sz, _sz, _u32, _vp, _vp, _i, _vp]),
    "karma_wal_append_batch": (_i, [_vp, _vp, _vp, _sz, _vp, _sz, _sz, _c.POINTER(_u64), _vp, _c.POINTER(_sz), _i]),
    "karma_wal_replay": (_i, [_vp, _vp, _sz, _sz, _u64, _c.POINTER(_u64), _c.POINTER(_u64), _c.POINTER(_i), _vp, _sz,
                              _i]),
    "karma_wal_replay_tuned": (_i, [_vp, _vp, _sz, _sz, _u64, _c.POINTER(_u64), _c.POINTER(_u64), _c.POINTER(_i), _vp,
                                    _sz, _i, _vp]),
    "karma_wal_replay_dir": (_i, [_c.c_char_p, _sz, _u64, _c.POINTER(_u64), _c.POINTER(_u64), _c.POINTER(_u64),
                                  _c.POINTER(_i), _vp, _sz, _i]),
    "karma_kfp_encode_batch": (_i, [_vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _sz, _vp, _sz, _vp, _c.POINTER(_sz),
                                    _c.POINTER(_u64), _i]),
    "karma_kfp_parse_batch": (_i, [_vp, _vp, _sz, _sz, _vp, _c.POINTER(_sz), _c.POINTER(_u64), _c.POINTER(_i), _i]),
    "karma_fill_splitmix64": (_i, [_vp, _sz, _u64, _u64, _vp]),
    "karma_stream_probe": (_i, [_vp, _sz, _vp, _vp]),
    "karma_device_cu_count": (_i, []),
    "karma_crc32c_time_next_units": (_i, [_vp, _vp]),
}


KARMA_WAL_CRC_PLAN, KARMA_WAL_CRC_DIRECT, KARMA_WAL_CRC_UNITS, KARMA_WAL_CRC_SEPARATE, KARMA_WAL_CRC_INLINE = 0, 1, 2, 3, 4


class WalTuning(ctypes.Structure):
    """karma_wal_tuning (include/karma_crc32c.h): plan overrides of karma_wal_replay_tuned."""
    _fields_ = [("walk_sub_bytes", _u64), ("crc_batch", _c.c_int32), ("reserved", _c.c_int32)]


class KarmaUnavailable(ImportError):
    """libkarma_crc32c.so is not built / not loadable."""


class KarmaError(RuntimeError):
    """A C ABI call returned a non-zero status."""

    def __init__(self, fn: str, status: int, detail: str):
        super().__init__(f"{fn} failed: status {status} ({detail})")
        self.fn = fn
        self.status = status


_LIB = None
_LOADED = {}


def load(path: str) -> ctypes.CDLL:
    """A build of the C ABI at `path` with its signatures bound (loaded once per path)."""
    if path not in _LOADED:
        if not os.path.exists(path):
            raise KarmaUnavailable(f"{path} not built: run `python -c 'import __graft_entry__ as g; g.build()'`")
        try:
            handle = ctypes.CDLL(path)
        except OSError as e:  # pragma: no cover - depends on the host
            raise KarmaUnavailable(f"cannot load {path}: {e}") from e
        for name, (res, args) in SIGNATURES.items():
            if not hasattr(handle, name) and path != LIB_PATH:
                continue  # an older build compared side by side (tools/): an entry point it predates
            fn = getattr(handle, name)
            fn.restype = res
            fn.argtypes = args
        if hasattr(handle, "karma_debug_bounds_report"):  # the bounds build only
            handle.karma_debug_bounds_report.restype = _i
            handle.karma_debug_bounds_report.argtypes = [_vp, _i]
        _LOADED[path] = handle
    return _LOADED[path]


def is_loaded(path: str) -> bool:
    return path in _LOADED


def lib() -> ctypes.CDLL:
    """The loaded library (loaded once).  Raises KarmaUnavailable when it is missing."""
    global _LIB
    if _LIB is None:
        _LIB = load(LIB_PATH)
    return _LIB


def select(path: str) -> None:
    """Make the build at `path` the package's library for the rest of the process (the test
    suite's --karma-lib option)."""
    global _LIB
    _LIB = load(path)


@contextlib.contextmanager
def using(path: str):
    """Run the package's wrappers on another build of the C ABI (the tools build) meanwhile."""
    global _LIB
    prev = lib()
    _LIB = load(path)
    try:
        yield _LIB
    finally:
        _LIB = prev


def check(fn: str, status: int) -> None:
    if status != KARMA_OK:
        L = lib()  # (a failure inside `using` reads the error text of the build in use)
        detail = L.karma_crc32c_strerror(status).decode()
        extra = L.karma_crc32c_last_error().decode()
        raise KarmaError(fn, status, f"{detail}: {extra}" if extra else detail)
