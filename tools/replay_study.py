#!/usr/bin/env python3
"""Device-resident WAL replay A/B (run on the GPU box from the repo root):

    python tools/replay_study.py [--mix fixed|config3] [--rounds 5] [--calls 20]

Builds the bench's WAL image (1M x 180 B records, or configs[2]'s mix, in 1 MiB segments) with
karma_wal_append_batch, copies it into HBM, and times karma_wal_replay_tuned over the device
copy for each variant in interleaved rounds (same process, same image):

    shipped              the shipped library, default plan
    sub=<bytes>          the shipped library, sub-range walkers of <bytes> (walk_sub_bytes)
    units                the shipped library, ragged plan instead of the direct kernel (crc_batch)
    ab                   tools build, default plan
    nodirect             tools build, KARMA_WALK_DIRECT=0: the walkers read tiles only (no direct header rounds)
    direct=<k>           tools build, direct header rounds after a fast round of k headers
    inline               the shipped library, KARMA_WAL_CRC_INLINE: the CRCs inside the walk (k_wal_walk_crc)
    listcrc              tools build, KARMA_WAL_CRC_INLINE + KARMA_WAL_LIST_CRC=1: the walk, then the walkers' lists checksummed by
                         the LDS-staged one-record-per-lane kernel (k_wal_list_crc)
    sepdirect4           tools build, KARMA_WAL_CRC_SEPARATE with KARMA_SMALL_STAGED=0 (the 4-lane batch)
    ab:NAME=VALUE        tools build, default plan, with one KARMA_* knob set (e.g. KARMA_GATHER_PARTS=1,
                         KARMA_SMALL_WHICH=0: both small-record launches)
    lib=<path>           another build of the library (e.g. the previous commit's), default plan
    sep                  the shipped library, KARMA_WAL_CRC_SEPARATE: walk, gather, one batch (round 2's path;
                         the default now checksums inside the walk kernel, k_wal_walk_crc)

Every call's result is checked (record count).  Prints ms per call and GB/s of image bytes per
variant (median over rounds).

--images K (default 4): K distinct images (different payload seeds, same framing) are copied
into HBM and the calls rotate over them, so that (K x ~201 MB > 512 MiB) no call finds its image
in the 256 MB Infinity Cache (MALL) left behind by the previous one (SURVEY.md §7 measurement
trap); --images 1 is the single reused image of round 2.  --single also times each variant on
image 0 alone, printed beside the rotated rate.
"""
import argparse
import ctypes
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--mix", default="fixed", choices=["fixed", "config3"])
    p.add_argument("--rounds", type=int, default=5)
    p.add_argument("--calls", type=int, default=20)
    p.add_argument("--variants", default="shipped,direct4,direct_v1,sub=24576,sub=32768,sub=40960")
    p.add_argument("--images", type=int, default=4)
    p.add_argument("--single", action="store_true")
    p.add_argument("--size", type=int, default=180, help="--mix fixed: payload bytes")
    p.add_argument("--count", type=int, default=1 << 20, help="--mix fixed: records")
    a = p.parse_args()
    import torch
    import synth
    from karma_amd import _lib
    seg = 1 << 20
    if a.mix == "config3":
        count = int((4 << 30) / (((65536 - 64) / np.log(1024)) + 8))
        lens = synth.loguniform_lengths(7, count, 64, 65536).astype(np.uint32)
        wal_bytes = ((int(lens.sum()) + 8 * count) // (seg - 65544) + 2) * seg
    else:
        count, size = a.count, a.size
        lens = np.full(count, size, dtype=np.uint32)
        wal_bytes = ((count + seg // (size + 8) - 1) // (seg // (size + 8)) + 1) * seg
    offs = np.concatenate([[0], np.cumsum(lens, dtype=np.uint64)[:-1]]).astype(np.uint64)
    L = _lib.lib()
    cur, nf = ctypes.c_uint64(0), ctypes.c_size_t()
    d_wals = []
    for k in range(a.images):
        src = synth.splitmix_np(42 + k, 0, int(lens.sum()) + 16).copy()
        wal = np.zeros(wal_bytes, dtype=np.uint8)
        cur.value = 0
        _lib.check("append", L.karma_wal_append_batch(src.ctypes.data, offs.ctypes.data, lens.ctypes.data, count,
                                                      wal.ctypes.data, wal_bytes, seg, ctypes.byref(cur), None,
                                                      ctypes.byref(nf), 0))
        assert nf.value == count
        d_wals.append(torch.from_numpy(wal).cuda())
        del src, wal
    torch.cuda.synchronize()
    rot = {"i": 0, "single": False}
    AB = _lib.load(_lib.AB_LIB_PATH)
    n, stop, status = ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_int()

    def call(lib, sub, batch):
        t = _lib.WalTuning(sub, batch, 0)
        d_wal = d_wals[0] if rot["single"] else d_wals[rot["i"] % len(d_wals)]
        rot["i"] += 1
        st = lib.karma_wal_replay_tuned(None, d_wal.data_ptr(), wal_bytes, seg, 0, ctypes.byref(n), ctypes.byref(stop),
                                        ctypes.byref(status), None, 0, 0, ctypes.byref(t))
        assert st == 0 and n.value == count, (st, n.value)

    variants = {}
    for v in a.variants.split(","):
        if v == "shipped":
            variants[v] = (L, 0, 0, None)
        elif v == "listcrc":  # the walk, then the walkers' lists by the LDS-staged kernel (k_wal_list_crc)
            variants[v] = (AB, 0, 4, ("KARMA_WAL_LIST_CRC", "1"))
        elif v == "inline":  # the shipped library, KARMA_WAL_CRC_INLINE (k_wal_walk_crc)
            variants[v] = (L, 0, 4, None)
        elif v == "sepdirect4":  # the separate path with the 4-lane small-record kernel only (round 2's)
            variants[v] = (AB, 0, 3, ("KARMA_SMALL_STAGED", "0"))
        elif v == "nodirect":  # the walkers on tiles only (no direct header rounds)
            variants[v] = (AB, 0, 0, ("KARMA_WALK_DIRECT", "0"))
        elif v.startswith("direct="):  # direct header rounds after a fast round of this many headers
            variants[v] = (AB, 0, 0, ("KARMA_WALK_DIRECT", v[7:]))
        elif v == "ab":  # the tools build's default plan (same-library reference for listcrc)
            variants[v] = (AB, 0, 0, None)
        elif v == "units":
            variants[v] = (L, 0, 2, None)
        elif v == "sep":  # the walk, then one small-record batch over the gathered lists (round 2's path)
            variants[v] = (L, 0, 3, None)
        elif v.startswith("sub="):
            variants[v] = (L, int(v[4:]), 0, None)
        elif v.startswith("ab:"):  # tools build, default plan, knobs: ab:NAME=VALUE[+NAME2=VALUE2...]
            variants[v] = (AB, 0, 0, [tuple(kv.split("=", 1)) for kv in v[3:].split("+")])
        elif v.startswith("lib="):  # another build's default plan, loaded beside the shipped one
            path = v[4:]
            variants[v] = (_lib.load(path if os.path.isabs(path) else os.path.join(ROOT, path)), 0, 0, None)
    res = {v: [] for v in variants}
    res1 = {v: [] for v in variants}

    def timed(lib, sub, batch, single):
        rot["single"] = single
        for _ in range(3):
            call(lib, sub, batch)
        t0 = time.perf_counter()
        for _ in range(a.calls):
            call(lib, sub, batch)
        rot["single"] = False
        return (time.perf_counter() - t0) / a.calls * 1e3

    for r in range(a.rounds):
        for v, (lib, sub, batch, env) in variants.items():
            for k in ("KARMA_DIRECT_VARIANT", "KARMA_WAL_LIST_CRC", "KARMA_SMALL_STAGED", "KARMA_WALK_DIRECT",
                      "KARMA_GATHER_PARTS", "KARMA_SMALL_WHICH", "KARMA_STAGE_SKEW", "KARMA_STAGE_R8",
                      "KARMA_WAL_SLICES", "KARMA_STAGE_BLOCKS", "KARMA_WAL_SLICE_PLAN"):
                os.environ.pop(k, None)
            pairs = env if isinstance(env, list) else [env] if env else []
            for name, val in pairs:
                os.environ[name] = val
            res[v].append(timed(lib, sub, batch, False))
            if a.single:
                res1[v].append(timed(lib, sub, batch, True))
            for name, _ in pairs:
                del os.environ[name]
        print(f"round {r}: " + "  ".join(f"{v} {res[v][-1]:.4f}" + (f" (single {res1[v][-1]:.4f})" if a.single else "")
                                         for v in variants), flush=True)
    print(f"images: {len(d_wals)} x {wal_bytes / 1e6:.1f} MB rotated ({len(d_wals) * wal_bytes / 2**20:.0f} MiB)")
    for v in variants:
        ms = float(np.median(res[v]))
        line = (f"{v:>14}: {ms:.4f} ms/call  {wal_bytes / ms / 1e6:.1f} GB/s image  "
                f"{int(lens.sum()) / ms / 1e6:.1f} GB/s payload (rotated)")
        if a.single:
            m1 = float(np.median(res1[v]))
            line += f"   single image: {m1:.4f} ms/call  {wal_bytes / m1 / 1e6:.1f} GB/s image"
        print(line, flush=True)


if __name__ == "__main__":
    main()
