#!/usr/bin/env python3
"""Turn a tools/profile_round.sh output directory into the committed profiles/ summaries.

    python tools/pmc_summary.py r01 fixed   # reads gpurun_out/prof/, writes profiles/

HBM bytes per launch of the dominant kernel, corrected as MI355X_MICROARCH.md §HBM says:
FETCH_SIZE (KB) x 1024 x 2   -- on gfx950 FETCH_SIZE reports half the bytes of a wide
                                (16 B/lane) coalesced streaming read;
WRITE_SIZE (KB) x 1024       -- exact for 16-B/lane stores; our CRC stores are 4 B per
                                record (uncalibrated width, reported as measured).
"""
import csv
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def per_kernel(path, counter):
    acc = {}
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        acc.setdefault(r["Kernel_Name"], []).append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in acc.items()}, {k: len(v) for k, v in acc.items()}


def main():
    rnd, wl = sys.argv[1], sys.argv[2]
    src = os.path.join(ROOT, "gpurun_out", "prof")
    dst = os.path.join(ROOT, "profiles")
    os.makedirs(dst, exist_ok=True)
    fetch, nf = per_kernel(os.path.join(src, f"pmc_fetch_{rnd}_{wl}", "run_counter_collection.csv"), "FETCH_SIZE")
    write, nw = per_kernel(os.path.join(src, f"pmc_write_{rnd}_{wl}", "run_counter_collection.csv"), "WRITE_SIZE")
    bench = json.load(open(os.path.join(src, f"bench_{rnd}_{wl}.json")))
    kernel = bench["config"]["kernel"]  # the dominant kernel bench.py timed
    payload = bench["config"]["records_per_gpu"] * bench["config"]["rec_bytes"] if wl != "ragged" else None
    stats = {}
    for r in csv.DictReader(open(os.path.join(src, f"trace_{rnd}_{wl}", "run_kernel_stats.csv"))):
        stats[r["Name"]] = {"calls": int(r["Calls"]), "avg_ns": float(r["AverageNs"]), "min_ns": float(r["MinNs"]),
                            "max_ns": float(r["MaxNs"])}
    ks = [v for k, v in stats.items() if kernel in k][0]
    kf = [k for k in fetch if kernel in k][0]
    fetch_b = fetch[kf] * 1024 * 2
    write_b = write.get(kf, 0.0) * 1024
    out = {
        "round": rnd,
        "workload": wl,
        "kernel": kernel,
        "payload_bytes_per_launch": payload,
        "fetch_size_kb_raw": fetch[kf],
        "write_size_kb_raw": write.get(kf),
        "launches_sampled": {"fetch": nf[kf], "write": nw.get(kf, 0)},
        "hbm_read_bytes_per_launch": fetch_b,
        "hbm_write_bytes_per_launch": write_b,
        "hbm_bytes_per_launch": fetch_b + write_b,
        "correction": "FETCH_SIZE*1024*2 (gfx950 half-count on 16B/lane streaming reads) + WRITE_SIZE*1024",
        "rocprof_kernel_avg_ns": ks["avg_ns"],
        "rocprof_kernel_calls": ks["calls"],
        "bench_kernel_ms_avg": bench["roofline"]["kernel_ms_avg"],
        "bench_value_gibs": bench["value"],
    }
    with open(os.path.join(dst, f"pmc_{wl}_4k.json" if wl == "fixed" else f"pmc_{wl}.json"), "w") as f:
        json.dump(out, f, indent=1)
    with open(os.path.join(dst, f"{rnd}_{wl}_pmc.json"), "w") as f:
        json.dump(out, f, indent=1)
    shutil.copy(os.path.join(src, f"trace_{rnd}_{wl}", "run_kernel_stats.csv"),
                os.path.join(dst, f"{rnd}_{wl}_kernel_stats.csv"))
    shutil.copy(os.path.join(src, f"bench_{rnd}_{wl}.json"), os.path.join(dst, f"{rnd}_{wl}_bench.json"))
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
