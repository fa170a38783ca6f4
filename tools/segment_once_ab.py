#!/usr/bin/env python3
"""One segment, isolated calls: k_segment_once (the tools build's KARMA_SEGMENT_ONCE=1, shipped)
against the looping fused kernel it replaced (=0), at 64 MiB (configs[3]) and smaller sizes.
Per size and variant: the isolated call (events around it, each call waited for) and the kernel
alone (events inside the library), medians over interleaved rounds after a 500 ms pre-warm, 64
distinct segments in rotation; CRCs equal across variants.  Run on the GPU box from the repo root:

    python tools/segment_once_ab.py [--sizes 64,16,4,1] [--json out.json]
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

L = _lib.load(_lib.AB_LIB_PATH)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--sizes", default="64,16,4,1")
    p.add_argument("--rounds", type=int, default=6)
    p.add_argument("--json", default="")
    p.add_argument("--libs", default="", help="name=path,... : builds compared at their defaults "
                   "(instead of the tools build's KARMA_SEGMENT_ONCE=1 / 0)")
    p.add_argument("--variants", default="1,0", help="KARMA_SEGMENT_ONCE values of the tools build (1 = the grid's "
                   "last workgroup folds, 2 = the last-arriving one, 0 = the looping fused kernel; r8 = 1 on the "
                   "8-copy stride image; late = 1 with the workgroup fold's maps loaded behind the chunks; wide = 1 with the "
                   "phased window step)")
    a = p.parse_args()
    dev = torch.device("cuda:0")
    nseg, top = 64, 64 << 20
    arena = torch.empty(nseg * top, dtype=torch.uint8, device=dev)
    K.fill_splitmix64(arena, 42)
    sh = torch.cuda.current_stream().cuda_stream
    V = a.variants.split(",")
    libs = {}
    for item in filter(None, a.libs.split(",")):
        name, _, path = item.partition("=")
        libs[name] = _lib.load(path if os.path.isabs(path) else os.path.join(ROOT, path))
    if libs:
        V = list(libs)
    report = {}
    for mib in [int(x) for x in a.sizes.split(",")]:
        seg = mib << 20
        outs = {v: torch.zeros(nseg, dtype=torch.uint32, device=dev) for v in V}
        state = {"i": 0}

        def call(v):
            lib = libs.get(v, L)
            if not libs:  # (r8 / late: KARMA_SEGMENT_ONCE=1 with KARMA_SEGMENT_R8=1 / KARMA_SEGMENT_LATE=1)
                os.environ["KARMA_SEGMENT_ONCE"] = "1" if v in ("r8", "late", "wide") else v
                for name, knob in (("r8", "KARMA_SEGMENT_R8"), ("late", "KARMA_SEGMENT_LATE"), ("wide", "KARMA_SEGMENT_WIDE")):
                    if v == name:
                        os.environ[knob] = "1"
                    else:
                        os.environ.pop(knob, None)
            i = state["i"] % nseg
            state["i"] += 1
            _lib.check("stream", lib.karma_crc32c_stream(0, arena.data_ptr() + i * top, seg,
                                                         outs[v].data_ptr() + 4 * i, sh))

        t_end = time.perf_counter() + 0.5
        while time.perf_counter() < t_end:
            call(V[0])
            torch.cuda.synchronize()
        lat = {v: [] for v in V}
        kern = {v: [] for v in V}
        for rnd in range(a.rounds):
            for v in V if rnd % 2 == 0 else V[::-1]:
                for _ in range(16):
                    u0, u1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    u0.record()
                    u1.record()
                    torch.cuda.synchronize()
                    libs.get(v, L).karma_crc32c_time_next_units(u0.cuda_event, u1.cuda_event)
                    e0.record()
                    call(v)
                    e1.record()
                    torch.cuda.synchronize()
                    lat[v].append(e0.elapsed_time(e1) * 1e3)
                    kern[v].append(u0.elapsed_time(u1) * 1e3)
        for v in V:  # every segment once per variant: the CRCs to compare
            state["i"] = 0
            for _ in range(nseg):
                call(v)
        torch.cuda.synchronize()
        same = all(bool(torch.equal(outs[V[0]], outs[v])) for v in V)
        ent = {v: {"call_us_p50": round(float(np.median(lat[v])), 2),
                   "kernel_us_p50": round(float(np.median(kern[v])), 2),
                   "call_us_p10_p90": [round(float(np.percentile(lat[v], q)), 2) for q in (10, 90)]} for v in V}
        ent["crcs_equal"] = same
        report[f"{mib}MiB"] = ent
        # one logged call of k_segment_once: per-workgroup stamps (us from the earliest entry)
        if hasattr(L, "karma_ab_seg_log") and not libs:
            os.environ["KARMA_SEGMENT_ONCE"] = "1"
            os.environ.pop("KARMA_SEGMENT_R8", None)
            log = torch.zeros(256 * 8, dtype=torch.int64, device=dev)
            torch.cuda.synchronize()
            L.karma_ab_seg_log(ctypes.c_void_p(log.data_ptr()))
            call("1")
            torch.cuda.synchronize()
            L.karma_ab_seg_log(None)
            st = log.cpu().numpy().reshape(256, 8)
            st = st[st[:, 0] > 0]
            t0 = st[:, 0].min()
            us = (st - t0) / 100.0
            ent["stamps_us"] = {nm: [round(float(np.percentile(us[:, i], q)), 2) for q in (0, 50, 100)]
                                for i, nm in [(0, "entry"), (6, "tables_issued"), (1, "tables_in_lds"), (7, "chunks_issued"),
                                              (2, "waves_folded"), (3, "published")]}
            last = us[-1]
            ent["last_wg_us"] = {"entry": round(float(last[0]), 2), "loaded": round(float(last[1]), 2),
                                 "published": round(float(last[3]), 2), "waited": round(float(last[4]), 2),
                                 "end": round(float(last[5]), 2)}
            ent["workgroups"] = int(st.shape[0])
            # the same segment twice back to back, the second logged: data in the MALL and L2,
            # TLB warm, GPU busy (what is left is the kernel's own latency chain)
            log.zero_()
            torch.cuda.synchronize()
            L.karma_ab_seg_log(ctypes.c_void_p(log.data_ptr()))
            state["i"] = 0
            call("1")
            state["i"] = 0
            call("1")
            torch.cuda.synchronize()
            L.karma_ab_seg_log(None)
            st = log.cpu().numpy().reshape(256, 8)
            st = st[st[:, 0] > 0]
            us = (st - st[:, 0].min()) / 100.0
            ent["warm_stamps_us"] = {nm: [round(float(np.percentile(us[:, i], q)), 2) for q in (0, 50, 100)]
                                     for i, nm in [(0, "entry"), (6, "tables_issued"), (1, "tables_in_lds"),
                                                   (7, "chunks_issued"), (2, "waves_folded"), (3, "published")]}
            ent["warm_last_wg_end_us"] = round(float(us[-1, 5]), 2)
        print(f"{mib} MiB", json.dumps(ent), flush=True)
        assert same, "variants differ"
    os.environ.pop("KARMA_SEGMENT_ONCE", None)
    if a.json:
        with open(a.json, "w") as f:
            json.dump(report, f, indent=1)


if __name__ == "__main__":
    main()
