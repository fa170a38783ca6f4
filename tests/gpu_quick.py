"""Quick GPU bring-up check (test infrastructure): parity on a few shapes + a timing probe.

    python tests/gpu_quick.py
"""
from __future__ import annotations

import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import karma_amd as K  # noqa: E402
import oracle_lib  # noqa: E402
import synth  # noqa: E402


def check(name, got, want):
    got = np.asarray(got, dtype=np.uint32)
    want = np.asarray(want, dtype=np.uint32)
    bad = int((got != want).sum())
    print(f"[{'OK ' if bad == 0 else 'BAD'}] {name}: {got.size} values, {bad} mismatches", flush=True)
    if bad:
        idx = np.nonzero(got != want)[0][:5]
        print("   first bad", [(int(i), hex(int(got[i])), hex(int(want[i]))) for i in idx])
    return bad == 0


def main():
    dev = torch.device("cuda:0")
    print("device", torch.cuda.get_device_name(0), "CUs", K.device_cu_count(), flush=True)
    ok = True
    # 1. fixed 4 KiB splitmix
    n, rec = 65536, 4096
    buf = torch.empty(n * rec, dtype=torch.uint8, device=dev)
    K.fill_splitmix64(buf, 42)
    torch.cuda.synchronize()
    host = buf.cpu().numpy()
    ok &= check("fill vs synth", host[:1 << 20], synth.splitmix_np(42, 0, 1 << 20))
    crc = K.value_batch_fixed(buf, rec).cpu().numpy()
    ok &= check("fixed 4KiB x 64K", crc, oracle_lib.splitmix_fixed_crcs(42, rec, 0, n))
    # 2. various fixed sizes / misalignments from one host buffer
    rng = np.random.default_rng(5)
    raw = rng.integers(0, 256, size=(1 << 22) + 64, dtype=np.uint8)
    draw = torch.from_numpy(raw).to(dev)
    for rb in [1, 3, 4, 15, 16, 17, 31, 32, 33, 100, 127, 128, 129, 255, 256, 1000, 4095, 4096, 4097, 65536, 100000]:
        for mis in [0, 1, 5, 8, 13]:
            nrec = min(2000, ((1 << 22) - mis) // rb)
            sub = draw[mis: mis + nrec * rb]
            got = K.value_batch_fixed(sub, rb).cpu().numpy()
            want = oracle_lib.fixed_crcs(raw[mis: mis + nrec * rb], rb)
            ok &= check(f"fixed rb={rb} mis={mis} n={nrec}", got, want)
    # 3. few huge records (split units + combine levels)
    for rb, nrec in [(1 << 22, 1), (3 << 20, 1), ((1 << 22) - 7, 1), (1 << 20, 4), (123457, 30)]:
        for mis in [0, 3]:
            sub = draw[mis: mis + nrec * rb]
            got = K.value_batch_fixed(sub, rb).cpu().numpy()
            want = oracle_lib.fixed_crcs(raw[mis: mis + nrec * rb], rb)
            ok &= check(f"split rb={rb} n={nrec} mis={mis}", got, want)
    # 4. init values
    init = torch.from_numpy(rng.integers(0, 1 << 32, size=1000, dtype=np.uint64).astype(np.uint32)).to(dev)
    got = K.value_batch_fixed(draw[:1000 * 333], 333, init=init).cpu().numpy()
    want = np.array([oracle_lib.extend(int(i), raw[r * 333:(r + 1) * 333].tobytes()) for r, i in
                     enumerate(init.cpu().numpy())], dtype=np.uint32)
    ok &= check("fixed init array", got, want)
    # 5. ragged golden fixtures
    recs = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "crc32c_records.json")))
    for key in ("ragged_replay_mix", "ragged_small_init", "ragged_tiny_unaligned"):
        g = recs[key]
        lens = synth.loguniform_lengths(g["seed_len"], g["count"], g["lo"], g["hi"])
        offs, arena = synth.ragged_layout(lens, header=g["header"])
        data = torch.from_numpy(synth.splitmix_np(g["seed_data"], 0, arena + 16).copy()).to(dev)
        ini = None
        if g["with_init"]:
            ini = torch.from_numpy(synth.splitmix_words(g["seed_len"] ^ 0x5A5A, 0, g["count"]).astype(np.uint32)).to(dev)
        got = K.extend_batch_ragged(data, torch.from_numpy(offs.astype(np.int64)).to(dev),
                                    torch.from_numpy(lens.astype(np.int32)).to(dev), init=ini,
                                    total_len=int(lens.sum())).cpu().numpy()
        ok &= check(f"ragged golden {key}", got, np.array([int(c, 16) for c in g["crc"]], dtype=np.uint32))
        got2 = K.extend_batch_ragged(data, torch.from_numpy(offs.astype(np.int64)).to(dev),
                                     torch.from_numpy(lens.astype(np.int32)).to(dev), init=ini).cpu().numpy()
        ok &= check(f"ragged golden {key} (no total)", got2, np.array([int(c, 16) for c in g["crc"]], dtype=np.uint32))
    # 6. 64 MiB pattern stream KAT
    pat = torch.from_numpy(np.frombuffer(synth.pattern(64 << 20), dtype=np.uint8).copy()).to(dev)
    v = int(K.extend_stream(0, pat).item())
    ok &= check("stream 64MiB pattern KAT", [v], [0x0C49B210])
    # 7. timing probe 1M x 4 KiB
    n, rec = 1 << 20, 4096
    big = torch.empty(n * rec, dtype=torch.uint8, device=dev)
    K.fill_splitmix64(big, 42)
    out = torch.empty(n, dtype=torch.uint32, device=dev)
    for _ in range(3):
        K.value_batch_fixed(big, rec, out=out)
    torch.cuda.synchronize()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    iters = 20
    ev0.record()
    for _ in range(iters):
        K.value_batch_fixed(big, rec, out=out)
    ev1.record()
    torch.cuda.synchronize()
    ms = ev0.elapsed_time(ev1) / iters
    gbs = n * rec / (ms * 1e-3) / 1e9
    print(f"fixed 1M x 4KiB: {ms:.3f} ms/step  {gbs:.1f} GB/s  ({gbs / 8000 * 100:.1f}% of 8 TB/s)", flush=True)
    t = time.time()
    want = oracle_lib.splitmix_fixed_crcs(42, rec, 0, n, threads=16)
    print(f"oracle 1M x 4KiB on 16 threads: {time.time() - t:.2f}s", flush=True)
    ok &= check("fixed 1M x 4KiB full", out.cpu().numpy(), want)
    pr = torch.zeros(1, dtype=torch.uint32, device=dev)
    for _ in range(3):
        K.stream_probe(big, pr)
    torch.cuda.synchronize()
    ev0.record()
    for _ in range(iters):
        K.stream_probe(big, pr)
    ev1.record()
    torch.cuda.synchronize()
    ms = ev0.elapsed_time(ev1) / iters
    print(f"read probe 4 GiB: {ms:.3f} ms  {n * rec / (ms * 1e-3) / 1e9:.1f} GB/s", flush=True)
    print("ALL OK" if ok else "FAILURES", flush=True)
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())
