#!/usr/bin/env python3
"""Where does an isolated 64 MiB segment call (bench.py --workload segment's
single_segment_latency_us) spend its time: the host enqueue, the launch, or the kernel?
Run on the GPU box from the repo root:  python tools/call_overhead.py [--mib 64]

Printed (medians, microseconds):
  enqueue_us        host time of one karma_crc32c_stream call, 200 calls back to back, no sync
  torch_enqueue_us  the same for a one-element torch add (the HIP launch floor)
  isolated_event_us events before / after the call on its stream, then a sync (the bench's figure)
  isolated_wall_us  perf_counter around call + stream sync
  graph_event_us    the call captured once in a hipGraph, replayed: events around each replay
  empty_event_us    events around a one-element torch add (an empty kernel's isolated figure)
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
import karma_amd as K  # noqa: E402
from karma_amd import _lib  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--mib", type=int, default=64)
    p.add_argument("--json", default="")
    a = p.parse_args()
    L = _lib.lib()
    dev = torch.device("cuda:0")
    seg, nseg = a.mib << 20, 16
    arena = torch.empty(seg * nseg, dtype=torch.uint8, device=dev)
    K.fill_splitmix64(arena, 5)
    out = torch.zeros(nseg, dtype=torch.uint32, device=dev)
    st = torch.cuda.Stream()
    sh = st.cuda_stream
    x = torch.zeros(1, device=dev)
    state = {"i": 0}

    def call():
        i = state["i"] % nseg
        state["i"] += 1
        _lib.check("stream", L.karma_crc32c_stream(0, arena.data_ptr() + i * seg, seg, out.data_ptr() + 4 * i, sh))

    def tadd():
        with torch.cuda.stream(st):
            x.add_(1)

    t_end = time.perf_counter() + 0.5
    while time.perf_counter() < t_end:
        call()
        st.synchronize()
    rep = {}
    for name, f in (("enqueue_us", call), ("torch_enqueue_us", tadd)):
        v = []
        for _ in range(5):
            st.synchronize()
            t0 = time.perf_counter()
            for _ in range(200):
                f()
            v.append((time.perf_counter() - t0) / 200 * 1e6)
            st.synchronize()
        rep[name] = round(float(np.median(v)), 2)
    for name, f in (("isolated_event_us", call), ("empty_event_us", tadd)):
        ev, wall = [], []
        for _ in range(50):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            st.synchronize()
            t0 = time.perf_counter()
            e0.record(st)
            f()
            e1.record(st)
            st.synchronize()
            wall.append((time.perf_counter() - t0) * 1e6)
            ev.append(e0.elapsed_time(e1) * 1e3)
        rep[name] = round(float(np.median(ev)), 2)
        if name == "isolated_event_us":
            rep["isolated_wall_us"] = round(float(np.median(wall)), 2)
    # the call captured in a graph (its host path runs once, at capture)
    g = torch.cuda.CUDAGraph()
    state["i"] = 0
    with torch.cuda.graph(g, stream=st):
        _lib.check("stream", L.karma_crc32c_stream(0, arena.data_ptr(), seg, out.data_ptr(), st.cuda_stream))
    gv = []
    for _ in range(50):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        e0.record()
        g.replay()
        e1.record()
        torch.cuda.synchronize()
        gv.append(e0.elapsed_time(e1) * 1e3)
    rep["graph_event_us"] = round(float(np.median(gv)), 2)
    want = int(K.Value(arena[:seg].cpu().numpy()))
    rep["graph_crc_ok"] = int(out[0].item()) == want
    print(json.dumps(rep), flush=True)
    assert rep["graph_crc_ok"]
    if a.json:
        with open(a.json, "w") as f:
            json.dump(rep, f, indent=1)


if __name__ == "__main__":
    main()
