#!/usr/bin/env python3
"""Builds of the library side by side on fixed batches, back to back as the bench runs them:
per round and build, 3 warm calls then 20 calls between two HIP events (ms per call), rounds
interleaved (order reversed every other round), after a 500 ms pre-warm; CRCs compared with the
first build's.  Run on the GPU box from the repo root:

    LIBS="shipped=karma_amd/lib/libkarma_crc32c.so,prev=tools/lib/libkarma_crc32c_prev.so" \\
        python tools/fixed_libs_ab.py
"""
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from karma_amd import _lib  # noqa: E402
import karma_amd as K  # noqa: E402

LIBS = {}
for item in os.environ.get("LIBS", f"shipped={_lib.LIB_PATH}").split(","):
    name, _, path = item.partition("=")
    LIBS[name] = _lib.load(path if os.path.isabs(path) else os.path.join(ROOT, path))
dev = torch.device("cuda:0")
arena = torch.empty(4 << 30, dtype=torch.uint8, device=dev)
K.fill_splitmix64(arena, 42)
sh = torch.cuda.current_stream().cuda_stream
cases = {"1M x 4 KiB": (4096, 1 << 20), "256K x 16 KiB": (16384, 1 << 18), "4M x 1 KiB": (1024, 1 << 22),
         "64 x 64 MiB": (64 << 20, 64)}  # (the last: configs[3], wave-folded units + k_combine_block)
if os.environ.get("CASES"):  # a subset, e.g. CASES="1M x 4 KiB,64 x 64 MiB"
    cases = {k: v for k, v in cases.items() if k in os.environ["CASES"].split(",")}
outs = {n: {v: torch.empty(c[1], dtype=torch.int32, device=dev) for v in LIBS} for n, c in cases.items()}


def run(lib, rec, n, out):
    assert lib.karma_crc32c_batch_fixed(arena.data_ptr(), rec, n, None, 0, out.data_ptr(), sh) == 0


first = next(iter(LIBS))
t_end = time.perf_counter() + 0.5
while time.perf_counter() < t_end:
    run(LIBS[first], 4096, 1 << 20, outs["1M x 4 KiB"][first])
    torch.cuda.synchronize()
res = {(n, v): [] for n in cases for v in LIBS}
for rnd in range(int(os.environ.get("ROUNDS", "8"))):
    order = list(LIBS.items()) if rnd % 2 == 0 else list(LIBS.items())[::-1]
    for n, (rec, cnt) in cases.items():
        for v, lib in order:
            for _ in range(3):
                run(lib, rec, cnt, outs[n][v])
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            for _ in range(20):
                run(lib, rec, cnt, outs[n][v])
            b.record()
            b.synchronize()
            res[(n, v)].append(a.elapsed_time(b) / 20)
        for v in LIBS:
            assert torch.equal(outs[n][first], outs[n][v]), (n, v)
    print(f"round {rnd}: " + "  ".join(f"{n}/{v} {res[(n, v)][-1]:.4f}" for n in cases for v in LIBS), flush=True)
for n, (rec, cnt) in cases.items():
    print(f"{n:14s} " + "  ".join(f"{v}: {np.median(res[(n, v)]):.4f} ms ({rec * cnt / np.median(res[(n, v)]) / 8e9:.3f})"
                                 for v in LIBS), flush=True)
