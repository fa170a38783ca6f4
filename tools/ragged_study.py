#!/usr/bin/env python3
"""Where does the ragged path lose against the fixed one?  Times the units kernel alone
(karma_crc32c_time_next_units) and the whole call for several 4 GiB layouts, the byte grid and the
unit plan (the tools build's KARMA_RAGGED_GRID=1 / 0) side by side, one process, interleaved
rounds.  Run on the GPU box from the repo root:  python tools/ragged_study.py
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

# the tools build (the KARMA_* A/B variants, karma_amd/csrc/ab.h), or another build of it named by KARMA_STUDY_LIB
_lib._LIB = _lib.load(os.environ.get("KARMA_STUDY_LIB", _lib.AB_LIB_PATH))
import synth  # noqa: E402

L = _lib.lib()
dev = torch.device("cuda:0")
GB = 4 << 30
RAW = GB + (64 << 20)  # config 3 arena = 4.01 GiB of payload + 8-B headers
raw = torch.empty(RAW, dtype=torch.uint8, device=dev)
K.fill_splitmix64(raw, 42)
torch.cuda.synchronize()
print("fill ok", hex(raw.data_ptr()), flush=True)
stream = torch.cuda.current_stream()
sh = stream.cuda_stream


def fixed_case(rec, variant="0"):
    n = GB // rec
    out = torch.empty(n, dtype=torch.uint32, device=dev)

    def run():
        os.environ["KARMA_CRC_VARIANT"] = variant
        _lib.check("fixed", L.karma_crc32c_batch_fixed(raw.data_ptr(), rec, n, None, 0, out.data_ptr(), sh))
    return run, n * rec


def ragged_case(lens, offs, grid="1", mode="0"):
    d_off = torch.from_numpy(offs.astype(np.int64)).to(dev)
    d_len = torch.from_numpy(lens.astype(np.int32)).to(dev)
    n = lens.size
    total = int(lens.sum())
    end = int((offs.astype(np.uint64) + lens.astype(np.uint64)).max())
    assert end <= RAW, f"layout ends at {end} > buffer {RAW}"  # checked on the host before any launch
    out = torch.empty(n, dtype=torch.uint32, device=dev)

    def run():
        os.environ["KARMA_RAGGED_GRID"] = grid
        os.environ["KARMA_GRID_MODE"] = mode  # timing-only grid modes (1: loads xored, 2: unmasked steps)
        _lib.check("ragged", L.karma_crc32c_batch_ragged(raw.data_ptr(), d_off.data_ptr(), d_len.data_ptr(), n, total,
                                                         None, 0, out.data_ptr(), sh))
    return run, total


cases = {}
FV = os.environ.get("FIXED_VARIANTS", "").split()
for rec in (4096,):
    cases[f"fixed {rec}"] = fixed_case(rec)
    for v in FV:
        cases[f"fixed {rec} v{v}"] = fixed_case(rec, v)
count = int(GB / (((65536 - 64) / np.log(1024)) + 8))
lens = synth.loguniform_lengths(7, count, 64, 65536)
offs, _ = synth.ragged_layout(lens, header=8)
srt = np.sort(lens)[::-1].copy()
o2, _ = synth.ragged_layout(srt, header=8)
layouts = {"aligned 4096": (np.full(GB // 4096, 4096, np.uint32), np.arange(GB // 4096, dtype=np.uint64) * 4096),
           "aligned 2048": (np.full(GB // 2048, 2048, np.uint32), np.arange(GB // 2048, dtype=np.uint64) * 2048),
           "config3": (lens, offs), "config3 sorted desc": (srt, o2)}
for name, (ln, of) in layouts.items():
    for g in ("1", "0"):
        cases[f"ragged {name} {'grid' if g == '1' else 'units'}"] = ragged_case(ln, of, g)
    for m in os.environ.get("GRID_MODES", "").split():
        cases[f"ragged {name} grid mode {m}"] = ragged_case(ln, of, "1", m)

for name, (run, nbytes) in cases.items():
    print("first call:", name, flush=True)
    run()
    torch.cuda.synchronize()
res = {k: ([], []) for k in cases}
for rnd in range(int(os.environ.get("ROUNDS", "5"))):
    for name, (run, nbytes) in cases.items():
        for _ in range(2):
            run()
        torch.cuda.synchronize()
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(10)]
        uev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(10)]
        for a, b in uev:
            a.record()
            b.record()
        torch.cuda.synchronize()
        for i in range(10):
            ev[i][0].record()
            L.karma_crc32c_time_next_units(uev[i][0].cuda_event, uev[i][1].cuda_event)
            run()
            ev[i][1].record()
        torch.cuda.synchronize()
        res[name][0].append(np.median([a.elapsed_time(b) for a, b in ev]))
        res[name][1].append(np.median([a.elapsed_time(b) for a, b in uev]))
for name, (run, nbytes) in cases.items():
    call, units = np.median(res[name][0]), np.median(res[name][1])
    print(f"{name:34s} payload {nbytes / 2**30:5.2f} GiB  call {call:.4f} ms ({nbytes / call / 1e6:7.1f} GB/s)  "
          f"units {units:.4f} ms ({nbytes / units / 1e6:7.1f} GB/s)", flush=True)
