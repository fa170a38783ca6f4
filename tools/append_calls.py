"""tools/append_calls.py -- per-call wall time of karma_wal_append_batch (bench.py's wal_append
workload: 1M x 180 B records, 1 MiB segments) measured around the ctypes call alone, for a pinned
and a pageable image, to separate the library's time from the caller's."""
import ctypes
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import synth  # noqa: E402
from karma_amd import _lib  # noqa: E402


def main():
    L = _lib.lib()
    n, size, seg = 1 << 20, int(sys.argv[1]) if len(sys.argv) > 1 else 180, 1 << 20
    lens = np.full(n, size, dtype=np.uint32)
    offs = (np.arange(n, dtype=np.uint64) * np.uint64(size)).astype(np.uint64)
    src = synth.splitmix_np(1, 0, n * size + 16).copy()
    per_seg = seg // (size + 8)
    wal_bytes = ((n + per_seg - 1) // per_seg + 1) * seg
    cur, nf = ctypes.c_uint64(0), ctypes.c_size_t()
    for kind, wal in (("pinned", torch.zeros(wal_bytes, dtype=torch.uint8).pin_memory().numpy()),
                      ("pageable", np.zeros(wal_bytes, dtype=np.uint8))):
        ts = []
        for i in range(40):
            cur.value = 0
            t0 = time.perf_counter()
            st = L.karma_wal_append_batch(src.ctypes.data, offs.ctypes.data, lens.ctypes.data, n, wal.ctypes.data,
                                          wal_bytes, seg, ctypes.byref(cur), None, ctypes.byref(nf), 0)
            ts.append(time.perf_counter() - t0)
            _lib.check("wal_append", st)
        t = np.array(ts[10:]) * 1e3
        pay = n * size / 2**30
        print(f"{kind:8s} {size} B: call ms min {t.min():.3f} median {np.median(t):.3f} max {t.max():.3f}  "
              f"-> {pay / (np.median(t) / 1e3):.1f} GiB/s median", flush=True)


if __name__ == "__main__":
    main()
