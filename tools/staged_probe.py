#!/usr/bin/env python3
"""Where the LDS-staged small-record kernel's time goes (round-4 VERDICT item 2b: 57 us for the
WAL replay's 1M x 180-B batch).  Builds K rotated device arenas of 1M WAL-framed records (an 8-byte
header, then the payload: the replay image's layout, 188-byte stride), and times
karma_crc32c_batch_ragged_bounded over them through the tools build's forms of the kernel:

    staged      KARMA_DIRECT_VARIANT=21: k_ragged_staged_pipe, plain stage (the replay's form)
    tm=1        ... without the CRC steps (the record loads, stage stores and per-batch work only)
    tm=2        ... without the record loads and stage stores (the steps over a stale stage)
    tm=3        ... without either (the per-batch metadata, extents and loop)
(Round 5 also timed a two-lanes-per-record form here, since removed: profiles/r05_staged_probe_pair.json.)
    direct4     KARMA_DIRECT_VARIANT=0: k_ragged_direct4 (the bounded ABI's shipped kernel)

Events around each call (back to back, arenas rotated past the Infinity Cache), median of rounds.
Run on the GPU box from the repo root:

    python tools/staged_probe.py [--size 180] [--count 1048576] [--images 4] [--json out.json]
"""
import argparse
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

FORMS = {"staged": {"KARMA_DIRECT_VARIANT": "21"},
         "tm=1": {"KARMA_DIRECT_VARIANT": "21", "KARMA_STAGE_TIMING": "1"},
         "tm=2": {"KARMA_DIRECT_VARIANT": "21", "KARMA_STAGE_TIMING": "2"},
         "tm=3": {"KARMA_DIRECT_VARIANT": "21", "KARMA_STAGE_TIMING": "3"},
         "direct4": {"KARMA_DIRECT_VARIANT": "0"}}


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--size", type=int, default=180)
    p.add_argument("--count", type=int, default=1 << 20)
    p.add_argument("--images", type=int, default=4)
    p.add_argument("--rounds", type=int, default=5)
    p.add_argument("--calls", type=int, default=20)
    p.add_argument("--forms", default=",".join(FORMS))
    p.add_argument("--json", default="")
    a = p.parse_args()
    L = _lib.load(os.path.join(ROOT, "tools/lib/libkarma_crc32c_ab.so"))
    dev = torch.device("cuda:0")
    stride = a.size + 8
    n = a.count
    nbytes = n * stride + 64
    arenas = []
    for k in range(a.images):
        t = torch.empty(nbytes, dtype=torch.uint8, device=dev)
        K.fill_splitmix64(t, 42 + k)
        arenas.append(t)
    off = torch.arange(n, dtype=torch.int64, device=dev) * stride + 8
    ln = torch.full((n,), a.size, dtype=torch.int32, device=dev)
    assert int(off[-1]) + a.size <= nbytes
    out = torch.empty(n, dtype=torch.uint32, device=dev)
    sh = torch.cuda.current_stream().cuda_stream
    forms = a.forms.split(",")

    def run(k):
        _lib.check("bounded", L.karma_crc32c_batch_ragged_bounded(arenas[k % a.images].data_ptr(), off.data_ptr(),
                                                                   ln.data_ptr(), n, n * a.size, a.size, None, 0,
                                                                   out.data_ptr(), sh))
    # the exact forms agree with each other
    ref = None
    for f in ("staged", "direct4"):
        if f in forms:
            os.environ.update(FORMS[f])
            run(0)
            torch.cuda.synchronize()
            got = out.cpu().numpy().copy()
            ref = got if ref is None else ref
            assert (got == ref).all(), f"{f} differs"
            for key in FORMS[f]:
                os.environ.pop(key, None)
    res = {f: [] for f in forms}
    for r in range(a.rounds):
        for f in (forms if r % 2 == 0 else forms[::-1]):
            for key in ("KARMA_DIRECT_VARIANT", "KARMA_STAGE_TIMING"):  # (each form sets its own)
                os.environ.pop(key, None)
            os.environ.update(FORMS[f])
            for i in range(3):
                run(i)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for i in range(a.calls):
                run(i)
            e1.record()
            torch.cuda.synchronize()
            res[f].append(e0.elapsed_time(e1) * 1e3 / a.calls)
    rep = {"records": n, "payload": a.size, "stride": stride, "images": a.images,
           "us_per_call": {f: round(float(np.median(v)), 2) for f, v in res.items()}}
    print(json.dumps(rep), flush=True)
    if a.json:
        with open(a.json, "w") as fh:
            json.dump(rep, fh, indent=1)


if __name__ == "__main__":
    main()
