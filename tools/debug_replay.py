#!/usr/bin/env python3
"""Debug: replay the 'small' mix of test_append_into_pinned_image_matches_pageable repeatedly
(pageable / pinned image, default plan / KARMA_WAL_CRC_SEPARATE) and compare with wal_model."""
import ctypes
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import synth  # noqa: E402
import wal_model  # noqa: E402
from karma_amd import _lib  # noqa: E402

L = _lib.lib()
SEG = 64 << 10


def payloads(seed, n, lo, hi):
    lens = synth.uniform_lengths(seed, n, lo, hi)
    offs = np.concatenate([[0], np.cumsum(lens, dtype=np.uint64)[:-1]]).astype(np.uint64)
    src = synth.splitmix_np(seed + 1, 0, int(lens.sum()) + 16).copy()
    return src, offs, lens


def append(src, offs, lens, wal, seg):
    cur = ctypes.c_uint64(0)
    nf = ctypes.c_size_t()
    rec = np.zeros(lens.size, np.uint64)
    _lib.check("append", L.karma_wal_append_batch(src.ctypes.data, offs.ctypes.data, lens.ctypes.data, lens.size,
                                                  wal.ctypes.data, wal.nbytes, seg, ctypes.byref(cur), rec.ctypes.data,
                                                  ctypes.byref(nf), 0))
    return cur.value, rec[: nf.value]


def replay(wal, start, seg, batch, sub=0, d=None):
    tuning = _lib.WalTuning(sub, batch, 0)
    n, stop, status = ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_int()
    rec = np.zeros(wal.nbytes // 8, np.uint64)
    _lib.check("replay", L.karma_wal_replay_tuned(wal.ctypes.data if d is None else None,
                                                  d.data_ptr() if d is not None else None, wal.nbytes, seg, start,
                                                  ctypes.byref(n), ctypes.byref(stop), ctypes.byref(status),
                                                  rec.ctypes.data, rec.size, 0, ctypes.byref(tuning)))
    return list(rec[: n.value]), stop.value, status.value


src, offs, lens = payloads(41, 30000, 1, 300)
nseg = int((lens.astype(np.int64) + 8).sum() // (SEG - int(lens.max()) - 8)) + 2
for cut in (0, nseg // 2):
    wal = np.zeros((nseg - cut) * SEG, np.uint8)
    cur, rec = append(src, offs, lens, wal, SEG)
    pinned = torch.zeros(wal.nbytes, dtype=torch.uint8).pin_memory()
    pw = pinned.numpy()
    pw[:] = wal
    d = torch.from_numpy(wal).cuda()
    for start in (0, int(rec[len(rec) // 3])):
        want = wal_model.replay(wal.tobytes(), SEG, start)
        print("cut", cut, "start", start, "model", len(want[0]), want[1], want[2], flush=True)
        for batch in (0, 3):
            for k in range(3):
                for kind in ("pageable", "pinned", "device"):
                    img = pw if kind == "pinned" else wal
                    got = replay(img, start, SEG, batch, d=d if kind == "device" else None)
                    ok = got == (list(want[0]), want[1], want[2])
                    if not ok:
                        a, b = got[0], list(want[0])
                        i = next((j for j in range(min(len(a), len(b))) if a[j] != b[j]), min(len(a), len(b)))
                        print(f"  MISMATCH batch={batch} rep={k} {kind}: n={len(a)} vs {len(b)} stop {got[1]} "
                              f"status {got[2]}; first diff at {i}: got {a[i:i+3]} want {b[i:i+3]}", flush=True)
                    else:
                        print(f"  ok batch={batch} rep={k} {kind}", flush=True)
