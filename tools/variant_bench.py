#!/usr/bin/env python3
"""A/B the streaming-kernel variants (KARMA_CRC_VARIANT) in ONE process, interleaved rounds.

    python tools/variant_bench.py [variants...]

A variant is a KARMA_CRC_VARIANT number, or ENV=VAL[,ENV=VAL...] (e.g. KARMA_FOLD_MAX_K=1);
every spec sets all the variables any spec names (unnamed ones back to their defaults).
"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import karma_amd as K  # noqa: E402
from karma_amd import _lib  # noqa: E402

_lib._LIB = _lib.load(_lib.AB_LIB_PATH)  # the tools build: the KARMA_* A/B variants (karma_amd/csrc/ab.h)

variants = sys.argv[1:] or ["0", "1", "2", "6"]


def spec_env(v):
    return dict(kv.split("=", 1) for kv in v.split(",")) if "=" in v else {"KARMA_CRC_VARIANT": v}


ENV_KEYS = sorted({k for v in variants for k in spec_env(v)})
dev = torch.device("cuda:0")
n, rec = int(os.environ.get("NREC", 1 << 20)), int(os.environ.get("REC", 4096))  # config 4: NREC=64 REC=67108864
MIS = int(os.environ.get("MISALIGN", "0"))  # byte offset of the arena (alignment experiments)
raw = torch.empty(n * rec + 256, dtype=torch.uint8, device=dev)
K.fill_splitmix64(raw, 42)
buf = raw[MIS: MIS + n * rec]
out = torch.empty(n, dtype=torch.uint32, device=dev)
ref = None
res = {v: [] for v in variants}
for rnd in range(int(os.environ.get('ROUNDS', '8'))):
    for v in variants:
        for k in ENV_KEYS:
            os.environ.pop(k, None)
        os.environ.update(spec_env(v))
        for _ in range(2):
            K.value_batch_fixed(buf, rec, out=out)
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(10):
            K.value_batch_fixed(buf, rec, out=out)
        b.record()
        torch.cuda.synchronize()
        res[v].append(a.elapsed_time(b) / 10)
        out.zero_()  # a variant that skips records must not pass on the previous call's CRCs
        K.value_batch_fixed(buf, rec, out=out)
        got = out.cpu().numpy()
        if ref is None:
            ref = got.copy()
        if v != "6":  # variant 6 is a timing experiment with wrong results by design
            assert np.array_equal(got, ref), f"variant {v} differs"
for v in variants:
    ms = np.array(res[v])
    print(f"variant {v}: median {np.median(ms):.4f} ms  min {ms.min():.4f}  -> {n * rec / np.median(ms) / 1e6:.1f} GB/s"
          f"  (best {n * rec / ms.min() / 1e6:.1f})  rounds {' '.join(f'{x:.3f}' for x in ms)}")
pr = torch.zeros(1, dtype=torch.uint32, device=dev)
probe_buf = raw[: n * rec]
for _ in range(3):
    K.stream_probe(probe_buf, pr)
torch.cuda.synchronize()
ts = []
for _ in range(5):
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(10):
        K.stream_probe(probe_buf, pr)
    b.record()
    torch.cuda.synchronize()
    ts.append(a.elapsed_time(b) / 10)
print(f"read probe (nt slab): median {np.median(ts):.4f} ms -> {n * rec / np.median(ts) / 1e6:.1f} GB/s")
