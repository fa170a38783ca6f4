#!/usr/bin/env python3
"""Where does the ragged units kernel lose against the fixed one?  (DESIGN.md §4, round-3
VERDICT item 4.)  Run on the GPU box from the repo root:

    python tools/ragged_gap.py                    # wave logs + unit-kernel times, every case
    python tools/ragged_gap.py --case config3 --calls 20 --no-log   # one case (rocprofv3 passes)

Cases (4 GiB of payload each, the tools build so the fixed v1 kernel and the wave log exist):
    fixed      1M x 4 KiB through karma_crc32c_batch_fixed (k_units_fixed, 2 KiB units folded in the wave)
    fixed_v1   the same with KARMA_CRC_VARIANT=1 (k_units_fixed_v1: each unit's loads issued when it starts)
    ragged4k   the same records through karma_crc32c_batch_ragged (k_units_ragged)
    config3    BASELINE configs[2]: 454,320 log-uniform 64 B-64 KiB records (k_units_ragged)

The wave log (wavelog.h, karma_ab_wave_log) gives per wave: stream start / end (100 MHz
wall clock), its CU / XCC, units and bytes.  Printed per case: kernel span, the spread of the
wave end times (first / median / p90 / last, relative to the first start), the mean active
fraction (sum of wave busy time / (waves x span)), units and KiB per wave, per-XCC median end.
"""
import argparse
import ctypes
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

_lib._LIB = _lib.load(os.environ.get("KARMA_STUDY_LIB", _lib.AB_LIB_PATH))  # (or another tools build)
import synth  # noqa: E402

REC = np.dtype([("t0", "<u8"), ("t1", "<u8"), ("hw", "<u4"), ("xcc", "<u4"), ("units", "<u4"), ("kib", "<u4"),
                ("steps", "<u4"), ("pad", "<u4")])


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--case", default="all")
    p.add_argument("--calls", type=int, default=10)
    p.add_argument("--no-log", action="store_true")
    p.add_argument("--json", default="")
    p.add_argument("--lib", default="", help="another build of the library (e.g. a unit-size build)")
    a = p.parse_args()
    if a.lib:
        _lib.select(a.lib)
    L = _lib.lib()
    dev = torch.device("cuda:0")
    GB = 4 << 30
    raw = torch.empty(GB + (64 << 20), dtype=torch.uint8, device=dev)
    K.fill_splitmix64(raw, 42)
    sh = torch.cuda.current_stream().cuda_stream
    cases = {}

    def fixed(variant, rec=4096, fold="2"):
        n = GB // rec
        out = torch.empty(n, dtype=torch.uint32, device=dev)

        def run():
            os.environ["KARMA_CRC_VARIANT"] = variant
            os.environ["KARMA_FOLD_MAX_K"] = fold
            _lib.check("fixed", L.karma_crc32c_batch_fixed(raw.data_ptr(), rec, n, None, 0, out.data_ptr(), sh))
        return run, n * rec

    layouts = {}

    def ragged(key, lens, offs, variant="0"):
        if key not in layouts:
            d_off = torch.from_numpy(offs.astype(np.int64)).to(dev)
            d_len = torch.from_numpy(lens.astype(np.int32)).to(dev)
            assert int((offs.astype(np.uint64) + lens.astype(np.uint64)).max()) <= raw.numel()
            layouts[key] = (d_off, d_len, lens.size, int(lens.sum()), {})
        d_off, d_len, n, total, ref = layouts[key]
        out = torch.empty(n, dtype=torch.uint32, device=dev)

        def run():
            os.environ["KARMA_CRC_VARIANT"] = "0"
            _lib.check("ragged", L.karma_crc32c_batch_ragged(raw.data_ptr(), d_off.data_ptr(), d_len.data_ptr(), n,
                                                             total, None, 0, out.data_ptr(), sh))

        def check():  # every variant's CRCs equal the shipped kernel's (variant 0) on the layout
            torch.cuda.synchronize()
            got = out.cpu().numpy().copy()
            if "want" not in ref:
                ref["want"] = got
            return int((got != ref["want"]).sum())
        run.check = check
        return run, total

    want = a.case.split(",") if a.case != "all" else ["fixed", "fixed_v1", "ragged4k", "config3"]
    for w in want:
        base, _, var = w.partition(":")
        var = var or "0"
        if base == "fixed":
            cases[w] = fixed("0")
        elif base == "fixed_v1":
            cases[w] = fixed("1")
        elif base == "fixed_k1":  # 4 KiB records, one 4 KiB unit each (no in-wave fold)
            cases[w] = fixed("0", 4096, "1")
        elif base == "fixed2k":  # 2 KiB records, one unit each
            cases[w] = fixed("0", 2048, "1")
        elif base.startswith("fixedrec"):  # fixedrec<bytes>: one unit per record (no fold)
            cases[w] = fixed("0", int(base[8:]), "1")
        elif base == "ragged2k":
            n = GB // 2048
            cases[w] = ragged(base, np.full(n, 2048, np.uint32), np.arange(n, dtype=np.uint64) * 2048, var)
        elif base == "ragged4k":
            n = GB // 4096
            cases[w] = ragged(base, np.full(n, 4096, np.uint32), np.arange(n, dtype=np.uint64) * 4096, var)
        elif base == "ragged1k":  # 1-1.5 KiB records: every unit partial and short
            n = int(GB / 1280)
            lens = np.random.default_rng(3).integers(1024, 1536, n).astype(np.uint32)
            offs = np.concatenate([[0], np.cumsum(lens.astype(np.uint64) + 8)[:-1]]).astype(np.uint64)
            cases[w] = ragged(base, lens, offs, var)
        elif base == "config3":
            count = int(GB / (((65536 - 64) / np.log(1024)) + 8))
            lens = synth.loguniform_lengths(7, count, 64, 65536)
            offs, _ = synth.ragged_layout(lens, header=8)
            cases[w] = ragged(base, lens.astype(np.uint32), offs, var)
    nwav = 256 * 16 * 4
    log = torch.zeros(nwav * REC.itemsize, dtype=torch.uint8, device=dev)
    report = {}
    import time
    t_end = time.perf_counter() + 0.5  # the clocks settle before anything is timed
    while time.perf_counter() < t_end:
        next(iter(cases.values()))[0]()
        torch.cuda.synchronize()
    for name, (run, nbytes) in cases.items():
        for _ in range(3):
            run()
        torch.cuda.synchronize()
        # unit-kernel time (events inside the library around the k_units_* launch)
        ts = []
        for _ in range(a.calls):
            s0, s1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s0.record()
            s1.record()
            torch.cuda.synchronize()
            L.karma_crc32c_time_next_units(s0.cuda_event, s1.cuda_event)
            run()
            torch.cuda.synchronize()
            ts.append(s0.elapsed_time(s1))
        ms = float(np.median(ts))
        ent = {"units_ms": round(ms, 4), "payload_bytes": nbytes, "units_frac_8tbs": round(nbytes / ms / 8e9, 4)}
        if hasattr(run, "check"):
            ent["mismatches_vs_variant0"] = run.check()
        if not a.no_log:
            log.zero_()
            torch.cuda.synchronize()
            _lib.check("wave_log", L.karma_ab_wave_log(ctypes.c_void_p(log.data_ptr()), ctypes.c_uint64(nwav)))
            run()
            torch.cuda.synchronize()
            _lib.check("wave_log", L.karma_ab_wave_log(None, ctypes.c_uint64(0)))
            rec = np.frombuffer(log.cpu().numpy().tobytes(), REC)
            rec = rec[rec["t1"] > 0]
            t0 = rec["t0"].min()
            start = (rec["t0"] - t0) / 100.0  # us
            end = (rec["t1"] - t0) / 100.0
            busy = end - start
            span = end.max()
            ent.update({
                "waves": int(rec.size), "span_us": round(float(span), 1),
                "start_us_p50_max": [round(float(np.median(start)), 1), round(float(start.max()), 1)],
                "end_us_first_p10_p50_p90_last": [round(float(np.percentile(end, q)), 1) for q in (0, 10, 50, 90, 100)],
                "active_frac": round(float(busy.sum() / (rec.size * span)), 4),
                "units_per_wave_mean_min_max": [round(float(rec["units"].mean()), 1), int(rec["units"].min()),
                                                int(rec["units"].max())],
                "kib_per_wave_mean_min_max": [round(float(rec["kib"].mean()), 1), int(rec["kib"].min()),
                                              int(rec["kib"].max())],
                "steps_per_wave_mean": round(float(rec["steps"].mean()), 2),
                "xcc_end_p50_us": {int(x): round(float(np.median(end[rec["xcc"] == x])), 1)
                                   for x in np.unique(rec["xcc"])},
            })
            # the work rate across the kernel: bytes finished per 10 % time bin (waves' bytes
            # spread evenly over their busy time)
            bins = np.linspace(0, span, 11)
            rate = np.zeros(10)
            for s, e, kb in zip(start, end, rec["kib"]):
                for i in range(10):
                    ov = max(0.0, min(e, bins[i + 1]) - max(s, bins[i]))
                    if e > s:
                        rate[i] += kb * 1024 * ov / (e - s)
            ent["gbs_per_decile"] = [round(float(r / (bins[1] - bins[0]) / 1e3), 0) for r in rate]
        report[name] = ent
        print(name, json.dumps(ent), flush=True)
    if a.json:
        with open(a.json, "w") as f:
            json.dump(report, f, indent=1)


if __name__ == "__main__":
    main()
