#!/usr/bin/env python3
"""Ragged finalize grid: blocks per CU (the tools build's KARMA_FINALIZE_PER_CU = 1, 2, 4) on
configs[2]'s layout, same process, interleaved, whole-call medians; CRCs compared.
Run on the GPU box from the repo root:  python tools/finalize_ab.py
"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import karma_amd as K  # noqa: E402
from karma_amd import _lib  # noqa: E402
import synth  # noqa: E402

L = _lib.load(_lib.AB_LIB_PATH)
dev = torch.device("cuda:0")
count = int((4 << 30) / (((65536 - 64) / np.log(1024)) + 8))
lens = synth.loguniform_lengths(7, count, 64, 65536)
offs, arena_bytes = synth.ragged_layout(lens, header=8)
arena = torch.empty(arena_bytes + 16, dtype=torch.uint8, device=dev)
K.fill_splitmix64(arena, 42)
d_off = torch.from_numpy(offs.astype(np.int64)).to(dev)
d_len = torch.from_numpy(lens.astype(np.int32)).to(dev)
total = int(lens.sum())
sh = torch.cuda.current_stream().cuda_stream
V = os.environ.get("PER_CU", "1 2 4").split()
outs = {v: torch.empty(count, dtype=torch.uint32, device=dev) for v in V}


def run(v):
    os.environ["KARMA_FINALIZE_PER_CU"] = v
    _lib.check("ragged", L.karma_crc32c_batch_ragged(arena.data_ptr(), d_off.data_ptr(), d_len.data_ptr(), count,
                                                      total, None, 0, outs[v].data_ptr(), sh))


res = {v: [] for v in V}
for rnd in range(6):
    for v in V if rnd % 2 == 0 else V[::-1]:
        for _ in range(3):
            run(v)
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(15)]
        for a, b in ev:
            a.record()
            run(v)
            b.record()
        torch.cuda.synchronize()
        res[v].append(np.median([a.elapsed_time(b) for a, b in ev]))
    assert all(torch.equal(outs[V[0]], outs[v]) for v in V), "variants differ"
for v in V:
    t = np.median(res[v])
    print(f"finalize {v} per CU: call {t:.4f} ms ({total / t / 8e9:.4f} of 8 TB/s payload)", flush=True)
