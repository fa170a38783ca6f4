#!/usr/bin/env python3
"""Fixed-record kernel, configs[1] (1M x 4 KiB): workgroups per CU (the tools build's
KARMA_FIXED_GRID_MULT = 1, 2, 4), same process, interleaved rounds, after a 400 ms pre-warm.
Every call's CRCs are compared with the first variant's.  Run on the GPU box from the repo root.
"""
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import karma_amd as K  # noqa: E402
from karma_amd import _lib  # noqa: E402

L = _lib.load(_lib.AB_LIB_PATH)
dev = torch.device("cuda:0")
n, rec = 1 << 20, 4096
buf = torch.empty(n * rec, dtype=torch.uint8, device=dev)
K.fill_splitmix64(buf, 42)
sh = torch.cuda.current_stream().cuda_stream
V = os.environ.get("GRID_MULTS", "1 2 4").split()
outs = {v: torch.empty(n, dtype=torch.uint32, device=dev) for v in V}


def run(v):
    os.environ["KARMA_FIXED_GRID_MULT"] = v
    _lib.check("fixed", L.karma_crc32c_batch_fixed(buf.data_ptr(), rec, n, None, 0, outs[v].data_ptr(), sh))


t0 = time.time()
while time.time() - t0 < 0.4:
    run(V[0])
torch.cuda.synchronize()
res = {v: [] for v in V}
for rnd in range(int(os.environ.get("ROUNDS", "6"))):
    for v in V if rnd % 2 == 0 else V[::-1]:
        for _ in range(3):
            run(v)
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(20)]
        for a, b in ev:
            a.record()
            run(v)
            b.record()
        torch.cuda.synchronize()
        res[v].append(np.median([a.elapsed_time(b) for a, b in ev]))
    assert all(torch.equal(outs[V[0]], outs[v]) for v in V), "variants differ"
for v in V:
    t = np.median(res[v])
    print(f"grid x{v}: {t:.4f} ms per call ({n * (rec + 4) / t / 1e9:.3f} TB/s, {n * (rec + 4) / t / 8e9:.4f} of 8 TB/s)", flush=True)
