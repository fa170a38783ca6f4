#!/usr/bin/env python3
"""Forms of the uniform-stride replay kernel (tools build knobs per form, e.g. KARMA_SPEC_TIMING=1..3:
no CRC steps, no record loads or stage stores, neither -- wrong results by design, so the calls'
results are not checked here; KARMA_SPEC_P2=1: two batches in flight).  1M x 180 B records in 1 MiB
segments, 4 rotated device images; per form the median of the library's own HIP events around the
CRC kernel (karma_crc32c_time_next_units), forms interleaved round by round.

    python3 tools/spec_timing.py [--rounds 5] [--calls 20]
"""
import argparse
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--rounds", type=int, default=5)
    p.add_argument("--calls", type=int, default=20)
    p.add_argument("--size", type=int, default=180)
    p.add_argument("--count", type=int, default=1 << 20)
    p.add_argument("--forms", default="full=,nosteps=KARMA_SPEC_TIMING:1,noloads=KARMA_SPEC_TIMING:2,"
                                      "neither=KARMA_SPEC_TIMING:3",
                   help="name=KNOB:V+KNOB:V,... (tools-build knobs per form)")
    args = p.parse_args()
    import torch
    import synth
    from karma_amd import _lib
    L = _lib.load(_lib.AB_LIB_PATH)
    seg, n, size = 1 << 20, args.count, args.size
    per = seg // (size + 8)
    wal_bytes = ((n + per - 1) // per + 1) * seg
    lens = np.full(n, size, np.uint32)
    offs = (np.arange(n, dtype=np.uint64) * size).astype(np.uint64)
    imgs = []
    for k in range(4):
        src = synth.splitmix_np(7 + k, 0, n * size + 16).copy()
        wal = np.zeros(wal_bytes, np.uint8)
        cur, nf = ctypes.c_uint64(0), ctypes.c_size_t()
        _lib.check("append", L.karma_wal_append_batch(src.ctypes.data, offs.ctypes.data, lens.ctypes.data, n,
                                                      wal.ctypes.data, wal_bytes, seg, ctypes.byref(cur), None,
                                                      ctypes.byref(nf), 0))
        imgs.append(torch.from_numpy(wal).cuda())
    torch.cuda.synchronize()
    os.environ["KARMA_WAL_SPEC"] = "2"
    nr, stop, status = ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_int()
    forms = [f.split("=") for f in args.forms.split(",")]  # name=KNOB:V+KNOB:V
    res = {name: [] for name, _ in forms}
    i = 0
    for r in range(args.rounds):
        for name, knobs in forms:
            for k in ("KARMA_SPEC_TIMING", "KARMA_SPEC_P2", "KARMA_SPEC_WIDE", "KARMA_SPEC_R8", "KARMA_SPEC_AL"):
                os.environ.pop(k, None)
            for kv in filter(None, knobs.split("+")):
                k, v = kv.split(":")
                os.environ[k] = v
            for c in range(args.calls):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                e1.record()
                torch.cuda.synchronize()
                L.karma_crc32c_time_next_units(e0.cuda_event, e1.cuda_event)
                d = imgs[i % 4]
                i += 1
                _lib.check("replay", L.karma_wal_replay(None, d.data_ptr(), wal_bytes, seg, 0, ctypes.byref(nr),
                                                       ctypes.byref(stop), ctypes.byref(status), None, 0, 0))
                e1.synchronize()
                if "KARMA_SPEC_TIMING" not in knobs:  # (a form with true results: every record, CORRUPT at the tail)
                    assert nr.value == n and status.value == 1, (name, nr.value, status.value)
                if c >= 2:
                    res[name].append(e0.elapsed_time(e1) * 1e3)
        print(f"round {r}: " + "  ".join(f"{name} {np.median(res[name][-(args.calls - 2):]):.1f} us"
                                         for name, _ in forms), flush=True)
    for name, knobs in forms:
        print(f"{name:>12} ({knobs or 'shipped form'}): {np.median(res[name]):.1f} us (median of {len(res[name])})")


if __name__ == "__main__":
    main()
