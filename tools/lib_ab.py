#!/usr/bin/env python3
"""Same-process A/B of two builds of the library on the ragged batch: the committed HEAD's
(build it first: git archive HEAD karma_amd/csrc include | tar -x -C build/head &&
make -C build/head/karma_amd/csrc) against the working tree's.  Interleaved rounds, medians of
10 calls, the units kernel timed alone (karma_crc32c_time_next_units), every call's CRCs
compared between the builds.  Run on the GPU box from the repo root:  python tools/lib_ab.py
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

LIBS = {"head": _lib.load(os.path.join(ROOT, "build", "head", "karma_amd", "lib", "libkarma_crc32c.so")),
        "new": _lib.load(_lib.LIB_PATH)}
ENV = {v: {} for v in LIBS}
# tools-build edge placements (KARMA_RAGGED_EDGES): 1 = head in the plan + tail in finalize,
# 2 = head in the plan only, 3 = tail in finalize only
_AB = _lib.load(_lib.AB_LIB_PATH)
for e in os.environ.get("EDGE_VARIANTS", "1").split():
    LIBS[f"edges{e}"] = _AB
    ENV[f"edges{e}"] = {"KARMA_RAGGED_EDGES": e}
dev = torch.device("cuda:0")
GB = 4 << 30
RAW = GB + (64 << 20)
raw = torch.empty(RAW, dtype=torch.uint8, device=dev)
K.fill_splitmix64(raw, 42)
torch.cuda.synchronize()
sh = torch.cuda.current_stream().cuda_stream


def ragged_case(lens, offs):
    d_off = torch.from_numpy(offs.astype(np.int64)).to(dev)
    d_len = torch.from_numpy(lens.astype(np.int32)).to(dev)
    n = lens.size
    total = int(lens.sum())
    end = int((offs.astype(np.uint64) + lens.astype(np.uint64)).max())
    assert end <= RAW, f"layout ends at {end} > buffer {RAW}"
    outs = {v: torch.empty(n, dtype=torch.uint32, device=dev) for v in LIBS}

    def run(v):
        os.environ.update(ENV[v])
        for k in ("KARMA_RAGGED_EDGES",):
            if k not in ENV[v]:
                os.environ.pop(k, None)
        _lib.check("ragged", LIBS[v].karma_crc32c_batch_ragged(raw.data_ptr(), d_off.data_ptr(), d_len.data_ptr(), n,
                                                                total, None, 0, outs[v].data_ptr(), sh))
    return run, total, outs


cases = {}
count = int(GB / (((65536 - 64) / np.log(1024)) + 8))
lens = synth.loguniform_lengths(7, count, 64, 65536)
offs, _ = synth.ragged_layout(lens, header=8)
cases["config3 log-uniform 64B-64KiB"] = ragged_case(lens, offs)
n4 = GB // 4096
cases["aligned 4 KiB"] = ragged_case(np.full(n4, 4096, np.uint32), np.arange(n4, dtype=np.uint64) * 4096)
l2 = synth.uniform_lengths(11, 800_000, 1025, 8192)
o2, _ = synth.ragged_layout(l2, header=8)
cases["800K uniform 1-8 KiB"] = ragged_case(l2, o2)
l3 = synth.uniform_lengths(12, 3 << 20, 1025, 1500)
o3, _ = synth.ragged_layout(l3, header=8)
cases["3M x 1-1.5 KiB"] = ragged_case(l3, o3)
if os.environ.get("WITH_1MIB", "1") == "1":
    l4 = synth.loguniform_lengths(13, 200_000, 64, 1 << 20)
    o4, _ = synth.ragged_layout(l4, header=8)
    keep = int(np.searchsorted(o4 + l4.astype(np.uint64), np.uint64(GB)))
    cases["log-uniform 64B-1MiB"] = ragged_case(l4[:keep].copy(), o4[:keep].copy())

names = list(LIBS)
for name, (run, nbytes, outs) in cases.items():
    for v in names:
        run(v)
    torch.cuda.synchronize()
    assert all(torch.equal(outs[names[0]], outs[v]) for v in names), f"{name}: builds differ"
    print("first calls agree:", name, flush=True)
res = {(k, v): ([], []) for k in cases for v in names}
for rnd in range(int(os.environ.get("ROUNDS", "5"))):
    for name, (run, nbytes, outs) in cases.items():
        for v in names if rnd % 2 == 0 else names[::-1]:
            for _ in range(2):
                run(v)
            torch.cuda.synchronize()
            ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(10)]
            uev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(10)]
            for a, b in uev:
                a.record()
                b.record()
            for i in range(10):
                ev[i][0].record()
                LIBS[v].karma_crc32c_time_next_units(uev[i][0].cuda_event, uev[i][1].cuda_event)
                run(v)
                ev[i][1].record()
            torch.cuda.synchronize()
            res[(name, v)][0].append(np.median([a.elapsed_time(b) for a, b in ev]))
            res[(name, v)][1].append(np.median([a.elapsed_time(b) for a, b in uev]))
        assert all(torch.equal(outs[names[0]], outs[v]) for v in names), f"{name}: builds differ"
    print("round", rnd, "ok", flush=True)
for name, (run, nbytes, outs) in cases.items():
    line = f"{name:30s} {nbytes / 2**30:5.2f} GiB"
    for v in names:
        c, u = np.median(res[(name, v)][0]), np.median(res[(name, v)][1])
        line += f" | {v}: call {c:.4f} ms ({nbytes / c / 8e9:.3f} of 8 TB/s) units {u:.4f}"
    c0, c1 = (np.median(res[(name, v)][0]) for v in names[:2])
    print(line + f" | new vs head: call {100 * (c0 - c1) / c0:+.1f} %", flush=True)
