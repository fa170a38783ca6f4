#!/usr/bin/env python3
"""Same-process A/B of library builds on the ragged batch (configs[2] and 1-1.5 KiB records):

    python tools/ragged_unit_libs.py name=path.so [name=path.so ...]

Typical use: builds with other ragged unit sizes (make -C karma_amd/csrc OBJDIR=$PWD/build/obj2k
LIBDIR=$PWD/build/lib2k EXTRA=-DKARMA_RAGGED_UNIT=2048) against the shipped one.  Interleaved
rounds; per build the median call time (HIP events around the call) and units-kernel time
(karma_crc32c_time_next_units); every build's CRCs must equal the first build's."""
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

LIBS = {}
for a in sys.argv[1:]:
    n, _, p = a.partition("=")
    LIBS[n] = _lib.load(os.path.abspath(p))
dev = torch.device("cuda:0")
GB = 4 << 30
raw = torch.empty(GB + (64 << 20), dtype=torch.uint8, device=dev)
K.fill_splitmix64(raw, 42)
sh = torch.cuda.current_stream().cuda_stream
layouts = {}
count = int(GB / (((65536 - 64) / np.log(1024)) + 8))
lens = synth.loguniform_lengths(7, count, 64, 65536)
offs, _ = synth.ragged_layout(lens, header=8)
layouts["config3"] = (lens.astype(np.uint32), offs)
n = int(GB / 1280)
l1 = np.random.default_rng(3).integers(1024, 1536, n).astype(np.uint32)
layouts["1-1.5KiB"] = (l1, np.concatenate([[0], np.cumsum(l1.astype(np.uint64) + 8)[:-1]]).astype(np.uint64))
dl = {k: (torch.from_numpy(o.astype(np.int64)).to(dev), torch.from_numpy(l.astype(np.int32)).to(dev), l.size,
          int(l.sum())) for k, (l, o) in layouts.items()}
outs = {(k, v): torch.empty(dl[k][2], dtype=torch.int32, device=dev) for k in dl for v in LIBS}
res = {(k, v): ([], []) for k in dl for v in LIBS}
for rnd in range(int(os.environ.get("ROUNDS", "6"))):
    for k, (d_off, d_len, cnt, total) in dl.items():
        for v, lib in LIBS.items():
            def call():
                assert lib.karma_crc32c_batch_ragged(raw.data_ptr(), d_off.data_ptr(), d_len.data_ptr(), cnt, total,
                                                     None, 0, outs[(k, v)].data_ptr(), sh) == 0
            for _ in range(3):
                call()
            torch.cuda.synchronize()
            cs, us = [], []
            for _ in range(10):
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                c, d = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                c.record()
                d.record()
                a.record()
                lib.karma_crc32c_time_next_units(c.cuda_event, d.cuda_event)
                call()
                b.record()
                b.synchronize()
                cs.append(a.elapsed_time(b))
                us.append(c.elapsed_time(d))
            res[(k, v)][0].append(float(np.median(cs)))
            res[(k, v)][1].append(float(np.median(us)))
        first = next(iter(LIBS))
        for v in LIBS:
            assert torch.equal(outs[(k, first)], outs[(k, v)]), (k, v)
    print(f"round {rnd}: " + "  ".join(f"{k}/{v} {res[(k, v)][0][-1]:.4f}/{res[(k, v)][1][-1]:.4f}"
                                       for k in dl for v in LIBS), flush=True)
for k in dl:
    for v in LIBS:
        c, u = np.median(res[(k, v)][0]), np.median(res[(k, v)][1])
        tot = dl[k][3]
        print(f"{k:9s} {v:8s} call {c:.4f} ms ({tot / c / 8e9:.3f} of 8 TB/s)  units {u:.4f} ms "
              f"({tot / u / 8e9:.3f})", flush=True)
