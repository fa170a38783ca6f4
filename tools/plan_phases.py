#!/usr/bin/env python3
"""Where the ragged call's plan and finalize time goes (round-4 VERDICT item 1: plan 32 us +
finalize 18 us on configs[2]).  The tools build's k_ragged_plan / k_ragged_finalize write
wall-clock stamps per workgroup (karma_ab_plan_log, 100 MHz); this prints, over several calls of
BASELINE configs[2]'s 454K-record mix (and an aligned 4 KiB layout), each phase's end relative to
the first plan workgroup's entry -- median and max over workgroups -- and the units kernel's event
time, so the call splits into plan, units, finalize and the gaps between them.  On the GPU box:

    python tools/plan_phases.py [--lib tools/lib/libkarma_crc32c_ab.so] [--calls 5] [--json out.json]
"""
import argparse
import ctypes
import json
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

PLAN = ["entry", "tables", "scan", "injections", "lookback", "descs"]
FIN = ["entry", "tables", "loads", "records"]
FIN_BASE = 8 * 4096


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--lib", default="tools/lib/libkarma_crc32c_ab.so")
    p.add_argument("--calls", type=int, default=5)
    p.add_argument("--json", default="")
    p.add_argument("--b2b", type=int, default=4, help="calls back to back per sample (the stamps are the last one's)")
    a = p.parse_args()
    L = _lib.load(a.lib if os.path.isabs(a.lib) else os.path.join(ROOT, a.lib))
    dev = torch.device("cuda:0")
    GB = 4 << 30
    raw = torch.empty(GB + (64 << 20), dtype=torch.uint8, device=dev)
    K.fill_splitmix64(raw, 42)
    count = int(GB / (((65536 - 64) / np.log(1024)) + 8))
    lens = synth.loguniform_lengths(7, count, 64, 65536)
    offs, _ = synth.ragged_layout(lens, header=8)
    layouts = {"config3": (lens, offs),
               "aligned 4096": (np.full(GB // 4096, 4096, np.uint32), np.arange(GB // 4096, dtype=np.uint64) * 4096)}
    log = torch.zeros(2 * FIN_BASE, dtype=torch.int64, device=dev)
    sh = torch.cuda.current_stream().cuda_stream
    rep = {"clock_MHz": 100, "layouts": {}}
    for name, (ln, of) in layouts.items():
        assert int((of.astype(np.uint64) + ln.astype(np.uint64)).max()) <= raw.numel()
        d_off = torch.from_numpy(of.astype(np.int64)).to(dev)
        d_len = torch.from_numpy(ln.astype(np.int32)).to(dev)
        n, total = ln.size, int(ln.sum())
        out = torch.empty(n, dtype=torch.uint32, device=dev)

        def run():
            _lib.check("ragged", L.karma_crc32c_batch_ragged(raw.data_ptr(), d_off.data_ptr(), d_len.data_ptr(), n, total,
                                                             None, 0, out.data_ptr(), sh))
        for _ in range(3):
            run()
        torch.cuda.synchronize()
        calls = []
        for c in range(a.calls):
            log.zero_()
            torch.cuda.synchronize()
            L.karma_ab_plan_log(ctypes.c_void_p(log.data_ptr()))
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
            ev[1].record()  # (recorded once, so the library may record them again)
            ev[2].record()
            torch.cuda.synchronize()
            for _ in range(a.b2b - 1):  # the GPU busy (clocks, TLBs) when the sampled call starts
                run()
            ev[0].record()
            L.karma_crc32c_time_next_units(ev[1].cuda_event, ev[2].cuda_event)
            run()
            ev[3].record()
            torch.cuda.synchronize()
            L.karma_ab_plan_log(None)
            g = log.cpu().numpy()
            nplan = int((g[:FIN_BASE].reshape(-1, 8)[:, 0] != 0).sum())  # (blocks of 1-4 x 1024 records)
            full = g[: 8 * nplan].reshape(nplan, 8).astype(np.float64)
            pl = full[:, : len(PLAN)]
            nfin = int((g[FIN_BASE:].reshape(-1, 8)[:, 0] != 0).sum())
            fl = g[FIN_BASE: FIN_BASE + 8 * nfin].reshape(nfin, 8)[:, : len(FIN)].astype(np.float64)
            t0 = pl[:, 0].min()
            rec = {"back_to_back": a.b2b, "call_ms": ev[0].elapsed_time(ev[3]), "units_ms": ev[1].elapsed_time(ev[2]),
                   "plan_blocks": int(nplan), "finalize_blocks": nfin}
            for i, ph in enumerate(PLAN):
                t = (pl[:, i] - t0) / 100.0
                rec[f"plan_{ph}_us"] = {"median": round(float(np.median(t)), 2), "max": round(float(t.max()), 2)}
                if i:  # the phase's own length per block
                    d = (pl[:, i] - pl[:, i - 1]) / 100.0
                    rec[f"plan_{ph}_us"]["len_median"] = round(float(np.median(d)), 2)
            for i, ph in ((6, "offsets_landed"), (7, "wave_scans")):  # finer stamps inside the scan phase
                d = (full[:, i] - full[:, 1]) / 100.0
                rec[f"plan_{ph}_after_tables_us"] = {"median": round(float(np.median(d)), 2), "max": round(float(d.max()), 2)}
            for i, ph in enumerate(FIN):
                t = (fl[:, i] - t0) / 100.0
                rec[f"fin_{ph}_us"] = {"min": round(float(t.min()), 2), "median": round(float(np.median(t)), 2),
                                       "max": round(float(t.max()), 2)}
                if i:
                    d = (fl[:, i] - fl[:, i - 1]) / 100.0
                    rec[f"fin_{ph}_us"]["len_median"] = round(float(np.median(d)), 2)
            calls.append(rec)
        rep["layouts"][name] = {"records": int(n), "calls": calls}
        print(name, json.dumps(calls[len(calls) // 2]), flush=True)
    if a.json:
        with open(a.json, "w") as f:
            json.dump(rep, f, indent=1)


if __name__ == "__main__":
    main()
