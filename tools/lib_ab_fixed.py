#!/usr/bin/env python3
"""Same-process A/B of two builds of the library on fixed batches (1M x 4 KiB, configs[1]) and a
64 MiB segment: build/head (a committed tree: git archive <rev> karma_amd/csrc include | tar -x -C
build/head && make -C build/head/karma_amd/csrc) against the working tree's.  Interleaved rounds,
median of 20 calls each (HIP events around the calls), CRCs compared between the builds.
Run on the GPU box from the repo root:  python tools/lib_ab_fixed.py"""
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from karma_amd import _lib  # noqa: E402
import karma_amd as K  # noqa: E402

LIBS = {"head": _lib.load(os.path.join(ROOT, "build", "head", "karma_amd", "lib", "libkarma_crc32c.so")),
        "new": _lib.load(_lib.LIB_PATH)}
dev = torch.device("cuda:0")
arena = torch.empty(4 << 30, dtype=torch.uint8, device=dev)
K.fill_splitmix64(arena, 42)
sh = torch.cuda.current_stream().cuda_stream
cases = {"fixed 1M x 4 KiB": (4096, 1 << 20), "segment 64 MiB": (64 << 20, 1)}
outs = {n: {v: torch.empty(c[1], dtype=torch.int32, device=dev) for v in LIBS} for n, c in cases.items()}


def run(lib, rec, n, out):
    assert lib.karma_crc32c_batch_fixed(arena.data_ptr(), rec, n, None, 0, out.data_ptr(), sh) == 0


t_end = time.perf_counter() + 0.5
while time.perf_counter() < t_end:
    run(LIBS["new"], 4096, 1 << 20, outs["fixed 1M x 4 KiB"]["new"])
    torch.cuda.synchronize()
res = {(n, v): [] for n in cases for v in LIBS}
for rnd in range(int(os.environ.get("ROUNDS", "8"))):
    for n, (rec, cnt) in cases.items():
        for v, lib in LIBS.items():
            for _ in range(3):
                run(lib, rec, cnt, outs[n][v])
            torch.cuda.synchronize()
            ts = []
            for _ in range(20):
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record()
                run(lib, rec, cnt, outs[n][v])
                b.record()
                b.synchronize()
                ts.append(a.elapsed_time(b))
            res[(n, v)].append(float(np.median(ts)))
        assert torch.equal(outs[n]["head"], outs[n]["new"]), n
    print(f"round {rnd}: " + "  ".join(f"{n}/{v} {res[(n, v)][-1] * 1e3:.1f}us" for n in cases for v in LIBS),
          flush=True)
for n in cases:
    print(n, "  ".join(f"{v}: {np.median(res[(n, v)]) * 1e3:.1f} us" for v in LIBS), flush=True)
