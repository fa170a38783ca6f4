#!/usr/bin/env python3
"""Small-record CRC kernel A/B on the WAL replay shape (run on the GPU box from the repo root):

    python tools/direct_study.py [--variants 0,6,7,8,9,10] [--n 1048576] [--size 180]

n payloads of --size bytes at a 188-byte stride (+8: the WAL image's header offsets) in HBM,
karma_crc32c_batch_ragged_bounded(max_len 1024) through the tools build with
KARMA_DIRECT_VARIANT = each variant, interleaved rounds; kernel time from HIP events around
--calls calls.  Variants 6-10 are timing-only (wrong CRCs): 6 no body lookups, 7 no lane fold
and group tree, 8 neither, 9 no head / tail steps, 10 none of these.  11 / 12: every round's
first 2 / 4 chunk loads issued at once (direct_batch ALL); 13: the shipped pipeline with 2 chunks
(11-13 are exact: checked against the shipped kernel's CRCs; list "0" first).
14 / 15: the LDS-staged one-record-per-lane kernel, un-pipelined / next batch in flight (exact).
"""
import argparse
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--variants", default="0,6,7,8,9,10")
    p.add_argument("--n", type=int, default=1 << 20)
    p.add_argument("--size", type=int, default=180)
    p.add_argument("--calls", type=int, default=20)
    p.add_argument("--rounds", type=int, default=5)
    a = p.parse_args()
    import torch
    import karma_amd as K
    from karma_amd import _lib
    L = _lib.load(_lib.AB_LIB_PATH)
    dev = torch.device("cuda:0")
    stride = a.size + 8
    arena = torch.empty(a.n * stride + 64, dtype=torch.uint8, device=dev)
    K.fill_splitmix64(arena, 7)
    off = (torch.arange(a.n, dtype=torch.int64, device=dev) * stride + 8)
    ln = torch.full((a.n,), a.size, dtype=torch.int32, device=dev)
    out = torch.empty(a.n, dtype=torch.int32, device=dev)
    s = torch.cuda.current_stream()
    variants = a.variants.split(",")
    res = {v: [] for v in variants}

    def call():
        st = L.karma_crc32c_batch_ragged_bounded(arena.data_ptr(), off.data_ptr(), ln.data_ptr(), a.n, a.n * a.size,
                                                 1024, None, 0, out.data_ptr(), s.cuda_stream)
        assert st == 0

    ref = None
    for r in range(a.rounds):
        for v in variants:
            os.environ["KARMA_DIRECT_VARIANT"] = v
            for _ in range(3):
                call()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.calls):
                call()
            e1.record()
            torch.cuda.synchronize()
            res[v].append(e0.elapsed_time(e1) / a.calls * 1e3)
            if v == "0" and ref is None:
                ref = out.clone()
            elif r == 0 and v in ("11", "12", "13", "14", "15", "19", "20", "21", "22", "23", "24", "25", "26", "27") and ref is not None:  # exact variants: the same CRCs
                bad = int((out != ref).sum().item())
                print(f"variant {v}: {bad} CRCs differ from the shipped kernel's", flush=True)
                assert bad == 0
        print(f"round {r}: " + "  ".join(f"v{v} {res[v][-1]:.2f}" for v in variants), flush=True)
    if ref is not None:  # the shipped kernel against the oracle's first records
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        import oracle_lib
        host = arena[: 64 * stride + 16].cpu().numpy()
        offs = np.arange(64, dtype=np.uint64) * stride + 8
        want = oracle_lib.ragged_crcs(host, offs, np.full(64, a.size, np.uint32))
        assert np.array_equal(ref[:64].cpu().numpy().view(np.uint32), want)
    for v in variants:
        us = float(np.median(res[v]))
        print(f"v{v:>3}: {us:8.2f} us/call  {a.n * a.size / us / 1e3:.1f} GB/s payload", flush=True)


if __name__ == "__main__":
    main()
