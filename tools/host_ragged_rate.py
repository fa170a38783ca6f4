#!/usr/bin/env python3
"""End-to-end rate of karma_crc32c_batch_ragged_host on BASELINE configs[2]'s mix (454K log-uniform
64 B - 64 KiB records, 8-byte headers between them, ~4 GiB) from pageable and from page-locked host
memory, one or more builds side by side (rounds interleaved), every CRC compared with the first
build's and a sample with the host crc32c.  Run on the GPU box from the repo root:

    LIBS="prev=tools/lib/libkarma_crc32c_prev.so,new=karma_amd/lib/libkarma_crc32c.so" \\
        python tools/host_ragged_rate.py [--gib 2] [--rounds 3] [--json out.json]
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import karma_amd as K  # noqa: E402
from karma_amd import _lib  # noqa: E402
import synth  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--gib", type=float, default=2.0)
    p.add_argument("--rounds", type=int, default=3)
    p.add_argument("--json", default="")
    a = p.parse_args()
    libs = {}
    for item in os.environ.get("LIBS", f"shipped={_lib.LIB_PATH}").split(","):
        name, _, path = item.partition("=")
        libs[name] = _lib.load(path if os.path.isabs(path) else os.path.join(ROOT, path))
    target = int(a.gib * (1 << 30))
    count = int(target / (((65536 - 64) / np.log(1024)) + 8))
    lens = synth.loguniform_lengths(7, count, 64, 65536).astype(np.uint32)
    offs, arena_bytes = synth.ragged_layout(lens, header=8)
    offs = offs.astype(np.uint64)
    pageable = synth.splitmix_np(42, 0, arena_bytes + 16).copy()
    pinned_t = torch.empty(arena_bytes + 16, dtype=torch.uint8).pin_memory()
    pinned = pinned_t.numpy()
    pinned[:] = pageable
    payload = int(lens.sum())
    outs = {(n, m): np.zeros(lens.size, np.uint32) for n in libs for m in ("pageable", "pinned")}
    times = {k: [] for k in outs}
    for n, L in libs.items():  # first calls: contexts, staging, workspaces
        for m, src in (("pageable", pageable), ("pinned", pinned)):
            _lib.check("ragged_host", L.karma_crc32c_batch_ragged_host(src.ctypes.data, src.nbytes, offs.ctypes.data,
                                                                       lens.ctypes.data, lens.size, 0,
                                                                       outs[(n, m)].ctypes.data, 0))
    for r in range(a.rounds):
        order = list(outs) if r % 2 == 0 else list(reversed(list(outs)))
        for key in order:
            n, m = key
            src = pageable if m == "pageable" else pinned
            t0 = time.perf_counter()
            _lib.check("ragged_host", libs[n].karma_crc32c_batch_ragged_host(src.ctypes.data, src.nbytes,
                                                                              offs.ctypes.data, lens.ctypes.data,
                                                                              lens.size, 0, outs[key].ctypes.data, 0))
            times[key].append(time.perf_counter() - t0)
    first = next(iter(outs))
    sample = np.random.default_rng(1).integers(0, lens.size, 64)
    bad_host = sum(int(K.Value(pageable[int(offs[i]): int(offs[i]) + int(lens[i])]) != int(outs[first][i])) for i in sample)
    rep = {"records": int(lens.size), "payload_bytes": payload, "arena_bytes": int(arena_bytes), "rounds": a.rounds,
           "sampled_vs_host_crc32c": {"records": 64, "mismatches": bad_host}, "builds": {}}
    for (n, m), t in times.items():
        med = float(np.median(t))
        rep["builds"].setdefault(n, {})[m] = {"s_median": round(med, 5), "payload_GiBps": round(payload / med / 2**30, 2),
                                             "mismatches_vs_first": int((outs[(n, m)] != outs[first]).sum())}
    print(json.dumps(rep), flush=True)
    if a.json:
        with open(a.json, "w") as f:
            json.dump(rep, f, indent=1)


if __name__ == "__main__":
    main()
