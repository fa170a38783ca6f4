#!/usr/bin/env python3
"""WAL append A/B (run on the GPU box from the repo root):

    KARMA_TRACE_HOST=1 python tools/append_study.py [--record 180] [--calls 10]

Frames 1M records of --record bytes (1 MiB segments) with karma_wal_append_batch into a pageable
and a page-locked image, alternating, and prints ms per call and GiB/s of payload for each
(median over rounds).  With KARMA_TRACE_HOST set the library prints its phase marks (stderr).
"""
import argparse
import ctypes
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--record", type=int, default=180)
    p.add_argument("--n", type=int, default=1 << 20)
    p.add_argument("--calls", type=int, default=10)
    p.add_argument("--rounds", type=int, default=3)
    p.add_argument("--ab", action="store_true", help="the tools build")
    p.add_argument("--only", default="", help="pageable or pinned: that image only")
    a = p.parse_args()
    import torch
    import synth
    from karma_amd import _lib
    seg, n, size = 1 << 20, a.n, a.record
    lens = np.full(n, size, dtype=np.uint32)
    offs = (np.arange(n, dtype=np.uint64) * np.uint64(size)).astype(np.uint64)
    src = synth.splitmix_np(1, 0, n * size + 16).copy()
    per_seg = seg // (size + 8)
    wal_bytes = ((n + per_seg - 1) // per_seg + 1) * seg
    images = {"pageable": np.zeros(wal_bytes, np.uint8),
              "pinned": torch.zeros(wal_bytes, dtype=torch.uint8).pin_memory().numpy()}
    L = _lib.load(_lib.AB_LIB_PATH) if a.ab else _lib.lib()
    if a.only:
        images = {a.only: images[a.only]}
    cur, nf = ctypes.c_uint64(0), ctypes.c_size_t()

    def call(w):
        cur.value = 0
        _lib.check("append", L.karma_wal_append_batch(src.ctypes.data, offs.ctypes.data, lens.ctypes.data, n,
                                                      w.ctypes.data, wal_bytes, seg, ctypes.byref(cur), None,
                                                      ctypes.byref(nf), 0))
        assert nf.value == n

    res = {k: [] for k in images}
    for r in range(a.rounds):
        for k, w in images.items():
            call(w)
            t0 = time.perf_counter()
            for _ in range(a.calls):
                call(w)
            res[k].append((time.perf_counter() - t0) / a.calls * 1e3)
        print(f"round {r}: " + "  ".join(f"{k} {v[-1]:.3f} ms" for k, v in res.items()), flush=True)
    if len(images) == 2:
        assert np.array_equal(images["pageable"], images["pinned"])
    for k, v in res.items():
        ms = float(np.median(v))
        print(f"{k:>9}: {ms:.3f} ms/call  {n * size / ms / 1e6 / 1.073741824:.1f} GiB/s payload", flush=True)


if __name__ == "__main__":
    main()
