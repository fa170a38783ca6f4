#!/usr/bin/env python3
"""Which calls leave device memory behind per stream?  (tests/test_gpu_lifetime.py's 1,000-stream
test.)  Per phase: N streams created with hipStreamCreate, one kind of call on each, the stream
released (karma_crc32c_release_stream) and destroyed, then karma_crc32c_trim; device free memory
before and after the phase (torch.cuda.mem_get_info).  Run on the GPU box from the repo root."""
import ctypes
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import karma_amd as K  # noqa: E402
from karma_amd import _lib  # noqa: E402

MIB = 1 << 20


def main():
    N = int(sys.argv[1]) if len(sys.argv) > 1 else 300
    L = _lib.lib()
    hip = ctypes.CDLL("libamdhip64.so")
    hip.hipStreamCreate.argtypes = [ctypes.POINTER(ctypes.c_void_p)]
    hip.hipStreamDestroy.argtypes = [ctypes.c_void_p]
    dev = torch.device("cuda:0")
    rng = np.random.default_rng(2)
    n = 20000
    lens = rng.integers(0, 3000, n).astype(np.uint32)
    offs = np.concatenate([[0], np.cumsum(lens[:-1].astype(np.uint64) + 8)]).astype(np.uint64)
    arena = torch.empty(64 * MIB, dtype=torch.uint8, device=dev)
    K.fill_splitmix64(arena, 17)
    perm = rng.permutation(n)
    d_off = torch.from_numpy(offs.astype(np.int64)).to(dev)
    d_len = torch.from_numpy(lens.astype(np.int32)).to(dev)
    d_off_p = torch.from_numpy(offs[perm].astype(np.int64)).to(dev)
    d_len_p = torch.from_numpy(lens[perm].astype(np.int32)).to(dev)
    out = torch.empty(n, dtype=torch.int32, device=dev)
    total = int(lens.sum())
    calls = {
        "none": lambda sh: None,
        "ragged_sorted": lambda sh: L.karma_crc32c_batch_ragged(arena.data_ptr(), d_off.data_ptr(), d_len.data_ptr(), n,
                                                                total, None, 0, out.data_ptr(), sh),
        "ragged_unsorted": lambda sh: L.karma_crc32c_batch_ragged(arena.data_ptr(), d_off_p.data_ptr(),
                                                                  d_len_p.data_ptr(), n, total, None, 0,
                                                                  out.data_ptr(), sh),
        "segment": lambda sh: L.karma_crc32c_stream(0, arena.data_ptr(), 64 * MIB, out.data_ptr(), sh),
        "fixed": lambda sh: L.karma_crc32c_batch_fixed(arena.data_ptr(), 4096, 4096, None, 0, out.data_ptr(), sh),
    }

    # the per-device host-path contexts (replay / append from host memory), as the lifetime test
    seg = 1 << 16
    plens = rng.integers(1, 500, 3000).astype(np.uint32)
    poffs = np.concatenate([[0], np.cumsum(plens[:-1], dtype=np.uint64)]).astype(np.uint64)
    src = rng.integers(0, 256, int(plens.sum()) + 16, dtype=np.uint8)
    wal = np.zeros(64 * seg, np.uint8)
    cur, nf = ctypes.c_uint64(0), ctypes.c_size_t()
    nrec, stop, status = ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_int()
    hbuf = rng.integers(0, 256, 4096 * 64, dtype=np.uint8)
    hout = np.zeros(4096, np.uint32)

    def wal_host(sh):
        cur.value = 0
        st = L.karma_wal_append_batch(src.ctypes.data, poffs.ctypes.data, plens.ctypes.data, plens.size, wal.ctypes.data,
                                      wal.nbytes, seg, ctypes.byref(cur), None, ctypes.byref(nf), 0)
        st = st or L.karma_wal_replay(wal.ctypes.data, None, wal.nbytes, seg, 0, ctypes.byref(nrec), ctypes.byref(stop),
                                      ctypes.byref(status), None, 0, 0)
        return st

    def host_batch(sh):
        return L.karma_crc32c_batch_fixed_host(hbuf.ctypes.data, 64, 4096, 0, hout.ctypes.data, 0)

    calls["wal_host"] = wal_host
    calls["host_batch"] = host_batch

    def free():
        torch.cuda.synchronize()
        return torch.cuda.mem_get_info()[0]

    for name, f in calls.items():  # warm-up: per-device tables exist before any baseline
        s = ctypes.c_void_p()
        assert hip.hipStreamCreate(ctypes.byref(s)) == 0
        st = f(s)
        assert not st, (name, st)
        assert L.karma_crc32c_release_stream(-1, s) == 0
        assert hip.hipStreamDestroy(s) == 0
    assert L.karma_crc32c_trim(-1) == 0
    report = {}
    for name, f in calls.items():
        base = free()
        for i in range(N):
            s = ctypes.c_void_p()
            assert hip.hipStreamCreate(ctypes.byref(s)) == 0
            st = f(s)
            assert not st, (name, st)
            assert L.karma_crc32c_release_stream(-1, s) == 0
            assert hip.hipStreamDestroy(s) == 0
        mid = free()
        assert L.karma_crc32c_trim(-1) == 0
        after = free()
        report[name] = {"before_trim_mib": round((base - mid) / MIB, 2), "after_trim_mib": round((base - after) / MIB, 2)}
        print(name, json.dumps(report[name]), flush=True)
    # tests/test_gpu_lifetime.py's loop as it is (every call on each stream, the host paths every
    # 250 streams), free memory every 100 streams
    base = free()
    for i in range(1000):
        s = ctypes.c_void_p()
        assert hip.hipStreamCreate(ctypes.byref(s)) == 0
        for name in ("ragged_sorted", "ragged_unsorted", "segment", "fixed"):
            assert not calls[name](s), name
        if i % 250 == 0:
            assert hip.hipStreamSynchronize(s) == 0
            assert not wal_host(s)
        assert L.karma_crc32c_release_stream(-1, s) == 0
        assert hip.hipStreamDestroy(s) == 0
        if i % 100 == 99:
            print("replica", i + 1, "streams:", round((base - free()) / MIB, 2), "MiB", flush=True)
    assert L.karma_crc32c_trim(-1) == 0
    print("replica after trim:", round((base - free()) / MIB, 2), "MiB", flush=True)
    # the same with streams kept (not destroyed) until the end: does the HIP runtime hold memory per stream?
    base = free()
    keep = []
    for i in range(N):
        s = ctypes.c_void_p()
        assert hip.hipStreamCreate(ctypes.byref(s)) == 0
        keep.append(s)
    mid = free()
    for s in keep:
        assert hip.hipStreamDestroy(s) == 0
    after = free()
    print("streams_alive", json.dumps({"alive_mib": round((base - mid) / MIB, 2),
                                       "destroyed_mib": round((base - after) / MIB, 2)}), flush=True)


if __name__ == "__main__":
    main()
