#!/usr/bin/env python3
"""Where does one 64 MiB segment scan spend its time?  (DESIGN.md §4, round-3 VERDICT item 7.)
Run on the GPU box from the repo root (the tools build: its wave log and KARMA_CRC_VARIANT):

    python tools/segment_gap.py [--variants 0,8,9,10] [--calls 64] [--json out.json]

The call is karma_crc32c_stream over one of 64 distinct 64 MiB segments in rotation (bench.py
--workload segment): one k_units_fixed launch whose last workgroup folds the 4,096 wave states
(FUSE).  Per variant (crc_fixed.hip launch_fixed_ab: 0 shipped, 8 = 8 chunks in flight per lane,
9 = 2, 10 = static wave-steps): the isolated call (events around it, each call waited for) and
the units kernel alone (events inside the library), medians; CRCs equal to variant 0's.
Then one logged call per variant (wavelog.h): per wave its kernel entry, stream start (after the
LDS table fill), stream end; the last workgroup's fold as one extra record.  Times in us from
the first wave's entry.
"""
import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import karma_amd as K  # noqa: E402
from karma_amd import _lib  # noqa: E402

_lib._LIB = _lib.load(_lib.AB_LIB_PATH)

REC = np.dtype([("t0", "<u8"), ("t1", "<u8"), ("hw", "<u4"), ("xcc", "<u4"), ("units", "<u4"), ("kib", "<u4"),
                ("steps", "<u4"), ("fill", "<u4")])


def pct(x, qs=(0, 10, 50, 90, 100)):
    return [round(float(np.percentile(x, q)), 2) for q in qs]


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--variants", default="0,8,9,10")
    p.add_argument("--calls", type=int, default=64)
    p.add_argument("--json", default="")
    a = p.parse_args()
    L = _lib.lib()
    dev = torch.device("cuda:0")
    seg, nseg = 64 << 20, 64
    arena = torch.empty(seg * nseg, dtype=torch.uint8, device=dev)
    K.fill_splitmix64(arena, 42)
    out = torch.zeros(nseg, dtype=torch.uint32, device=dev)
    st = torch.cuda.current_stream()
    sh = st.cuda_stream
    state = {"i": 0}

    def call():
        i = state["i"] % nseg
        state["i"] += 1
        _lib.check("stream", L.karma_crc32c_stream(0, arena.data_ptr() + i * seg, seg, out.data_ptr() + 4 * i, sh))

    nlog = 256 * 16 + 64
    log = torch.zeros(nlog * REC.itemsize, dtype=torch.uint8, device=dev)
    report = {}
    want = None
    t_end = time.perf_counter() + 0.5  # clocks settle
    while time.perf_counter() < t_end:
        call()
        torch.cuda.synchronize()
    for v in a.variants.split(","):
        os.environ["KARMA_CRC_VARIANT"] = v
        state["i"] = 0
        for _ in range(nseg):  # every segment once: the CRCs to compare
            call()
        torch.cuda.synchronize()
        got = out.cpu().numpy().copy()
        if want is None:
            want = got
        lat, kern = [], []
        for _ in range(a.calls):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            u0, u1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            u0.record()
            u1.record()
            torch.cuda.synchronize()
            L.karma_crc32c_time_next_units(u0.cuda_event, u1.cuda_event)
            e0.record()
            call()
            e1.record()
            torch.cuda.synchronize()
            lat.append(e0.elapsed_time(e1) * 1e3)
            kern.append(u0.elapsed_time(u1) * 1e3)
        ent = {"call_us_p50": round(float(np.median(lat)), 2), "units_kernel_us_p50": round(float(np.median(kern)), 2),
               "call_us_p10_p90": [round(float(np.percentile(lat, 10)), 2), round(float(np.percentile(lat, 90)), 2)],
               "mismatches_vs_variant0": int((got != want).sum())}
        log.zero_()
        torch.cuda.synchronize()
        _lib.check("wave_log", L.karma_ab_wave_log(ctypes.c_void_p(log.data_ptr()), ctypes.c_uint64(nlog)))
        call()
        torch.cuda.synchronize()
        _lib.check("wave_log", L.karma_ab_wave_log(None, ctypes.c_uint64(0)))
        rec = np.frombuffer(log.cpu().numpy().tobytes(), REC)
        fold = rec[(rec["t1"] > 0) & (rec["steps"] == 1) & (rec["kib"] == 0) & (rec["units"] == 0)
                   & (np.arange(rec.size) >= 4096)]
        w = rec[:4096]
        w = w[w["t1"] > 0]
        entry = w["t0"] - w["fill"]
        base = entry.min()
        us = lambda t: (t.astype(np.int64) - int(base)) / 100.0  # noqa: E731
        ent.update({
            "waves": int(w.size),
            "entry_us": pct(us(entry)),
            "fill_us": pct(w["fill"] / 100.0),
            "stream_start_us": pct(us(w["t0"])),
            "stream_us": pct((w["t1"] - w["t0"]) / 100.0),
            "stream_end_us": pct(us(w["t1"])),
            "kib_per_wave_mean": round(float(w["kib"].mean()), 1),
            "xcc_end_p50_us": {int(x): round(float(np.median(us(w["t1"][w["xcc"] == x]))), 2)
                               for x in np.unique(w["xcc"])},
        })
        if fold.size:
            ent["fold_start_end_us"] = [round(float(us(fold["t0"])[0]), 2), round(float(us(fold["t1"])[0]), 2)]
        report[v] = ent
        print(v, json.dumps(ent), flush=True)
    os.environ["KARMA_CRC_VARIANT"] = "0"
    if a.json:
        with open(a.json, "w") as f:
            json.dump(report, f, indent=1)


if __name__ == "__main__":
    main()
