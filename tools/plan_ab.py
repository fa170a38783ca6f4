#!/usr/bin/env python3
"""Ragged plan A/B: the single-pass plan (k_ragged_plan, look-back) against round 1's two-pass
plan (k_ragged_scan + k_ragged_desc), same process, interleaved rounds, tools build
(KARMA_RAGGED_PLAN=1 / 2).  Every timed call's CRCs are compared between the two plans.
Run on the GPU box from the repo root:  python tools/plan_ab.py
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

_lib._LIB = _lib.load(_lib.AB_LIB_PATH)
import synth  # noqa: E402

L = _lib.lib()
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
    outs = {v: torch.empty(n, dtype=torch.uint32, device=dev) for v in ("1", "2")}

    def run(v):
        os.environ["KARMA_RAGGED_PLAN"] = v
        _lib.check("ragged", L.karma_crc32c_batch_ragged(raw.data_ptr(), d_off.data_ptr(), d_len.data_ptr(), n, total,
                                                         None, 0, outs[v].data_ptr(), sh))
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

for name, (run, nbytes, outs) in cases.items():
    for v in ("1", "2"):
        run(v)
    torch.cuda.synchronize()
    assert torch.equal(outs["1"], outs["2"]), f"{name}: plans differ"
    print("first calls agree:", name, flush=True)
res = {(k, v): [] for k in cases for v in ("1", "2")}
ures = {(k, v): [] for k in cases for v in ("1", "2")}
for rnd in range(int(os.environ.get("ROUNDS", "5"))):
    for name, (run, nbytes, outs) in cases.items():
        for v in ("1", "2") if rnd % 2 == 0 else ("2", "1"):
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
                L.karma_crc32c_time_next_units(uev[i][0].cuda_event, uev[i][1].cuda_event)
                run(v)
                ev[i][1].record()
            torch.cuda.synchronize()
            res[(name, v)].append(np.median([a.elapsed_time(b) for a, b in ev]))
            ures[(name, v)].append(np.median([a.elapsed_time(b) for a, b in uev]))
        assert torch.equal(outs["1"], outs["2"]), f"{name}: plans differ"
    print("round", rnd, "ok", flush=True)
for name, (run, nbytes, outs) in cases.items():
    t1, t2 = np.median(res[(name, "1")]), np.median(res[(name, "2")])
    print(f"{name:32s} {nbytes / 2**30:5.2f} GiB  single-pass {t1:.4f} ms ({nbytes / t1 / 1e6:7.1f} GB/s)  "
          f"two-pass {t2:.4f} ms ({nbytes / t2 / 1e6:7.1f} GB/s)  gain {100 * (t2 - t1) / t2:+.1f} %  units kernel "
          f"{np.median(ures[(name, '1')]):.4f} / {np.median(ures[(name, '2')]):.4f} ms", flush=True)
