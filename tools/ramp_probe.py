#!/usr/bin/env python3
"""tools/ramp_probe.py -- why the first ~40 config-2 dispatches of a process run slow.

Per-dispatch durations (HIP events around each karma_crc32c_batch_fixed call, 1M x 4 KiB) in
series separated by idle gaps, with and without a preceding burn on a DIFFERENT buffer:

  S1  fresh process, arena just filled
  S2  after 1 s idle (page tables warm, clocks may have dropped)
  S3  after 1 s idle + a 300 ms read-only burn (karma_stream_probe) over another 4 GiB buffer
  S4  after 1 s idle + a 300 ms burn of CRC batches over the other buffer

If S3/S4 start at steady state while S2 ramps again, the ramp is the clock/power state (DPM),
not first touch or TLB warm-up of the arena.  The GPU's sclk/mclk DPM levels are sampled from
sysfs every ~2 ms meanwhile when readable.
"""
import glob
import json
import os
import sys
import threading
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import karma_amd as K  # noqa: E402

dev = torch.device("cuda:0")
n, rec = 1 << 20, 4096
A = torch.empty(n * rec, dtype=torch.uint8, device=dev)
B = torch.empty(n * rec, dtype=torch.uint8, device=dev)
out = torch.empty(n, dtype=torch.uint32, device=dev)
pout = torch.empty(1, dtype=torch.uint32, device=dev)
K.fill_splitmix64(A, 42)
K.fill_splitmix64(B, 43)
torch.cuda.synchronize()

# ---- DPM level sampler (sysfs; silently absent when not readable) -------------------------
samples = []
paths = {}
for kind in ("sclk", "mclk", "fclk"):
    c = sorted(glob.glob(f"/sys/class/drm/card*/device/pp_dpm_{kind}"))
    if c:
        paths[kind] = c[0]


def level(p):
    try:
        with open(p) as f:
            for line in f:
                if line.rstrip().endswith("*"):
                    return line.split(":", 1)[1].strip().rstrip("*").strip()
    except OSError:
        return None
    return None


stop = threading.Event()
t_start = time.perf_counter()


def sampler():
    while not stop.is_set():
        samples.append((round((time.perf_counter() - t_start) * 1e3, 2),) + tuple(level(p) for p in paths.values()))
        time.sleep(0.002)


th = threading.Thread(target=sampler, daemon=True)
if paths:
    th.start()


def series(tag, m=60):
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(m)]
    t0 = (time.perf_counter() - t_start) * 1e3
    for a, b in evs:
        a.record()
        K.value_batch_fixed(A, rec, out=out)
        b.record()
    torch.cuda.synchronize()
    ms = np.array([a.elapsed_time(b) for a, b in evs])
    print(json.dumps({"series": tag, "t_ms": round(t0, 1), "first20": round(float(ms[:20].mean()), 4),
                      "next20": round(float(ms[20:40].mean()), 4), "last20": round(float(ms[40:].mean()), 4),
                      "per_dispatch": [round(float(x), 4) for x in ms]}), flush=True)


def burn(fn, ms):
    t0 = time.perf_counter()
    while (time.perf_counter() - t0) * 1e3 < ms:
        for _ in range(8):
            fn()
        torch.cuda.synchronize()


series("S1_fresh")
time.sleep(1.0)
series("S2_after_idle")
time.sleep(1.0)
burn(lambda: K.stream_probe(B, out=pout), 300)
series("S3_after_probe_burn_other_buffer")
time.sleep(1.0)
burn(lambda: K.value_batch_fixed(B, rec, out=out), 300)
series("S4_after_crc_burn_other_buffer")
stop.set()
if paths:
    th.join()
    print(json.dumps({"dpm_paths": paths, "samples": samples[::5]}))
else:
    print(json.dumps({"dpm_paths": None}))
