#!/usr/bin/env python3
"""Per-kernel summary of a rocprofv3 kernel trace + counter passes (tools/pmc_replay.sh layout):

    python tools/pmc_kernels.py gpurun_out/pmc_replay_r02 profiles/r02_wal_replay_pmc.json k_wal_walk_sub ...

For each named kernel (substring match): dispatches, average duration (kernel trace), and the
average per dispatch of every counter collected, plus derived figures -- instructions per wave,
wait / busy fractions, and HBM bytes with the MI355X_MICROARCH.md gfx950 correction
(FETCH_SIZE KB x 1024 x 2 for 16-B/lane streaming reads; WRITE_SIZE KB x 1024).
"""
import csv
import glob
import json
import os
import sys


def main():
    src, dst, names = sys.argv[1], sys.argv[2], sys.argv[3:]
    out = {"source": os.path.relpath(src), "kernels": {}}
    stats = {}
    for r in csv.DictReader(open(os.path.join(src, "trace", "run_kernel_stats.csv"))):
        stats[r["Name"]] = r
    ctr = {}
    for path in sorted(glob.glob(os.path.join(src, "pass*", "run_counter_collection.csv"))):
        for r in csv.DictReader(open(path)):
            ctr.setdefault(r["Kernel_Name"], {}).setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
    for want in names:
        ks = [k for k in stats if want in k and "v1" not in k]
        if not ks:
            continue
        k = ks[0]
        st = stats[k]
        ent = {"kernel": k, "calls": int(st["Calls"]), "avg_us": float(st["AverageNs"]) / 1e3,
               "min_us": float(st["MinNs"]) / 1e3, "max_us": float(st["MaxNs"]) / 1e3, "counters": {}}
        cs = [c for c in ctr if want in c and "v1" not in c]
        if cs:
            for name, vals in ctr[cs[0]].items():
                ent["counters"][name] = sum(vals) / len(vals)
        c = ent["counters"]
        waves = c.get("SQ_WAVES")
        if waves:
            for name in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_INSTS_VMEM_RD", "SQ_INSTS_SMEM"):
                if name in c:
                    ent[name + "_per_wave"] = c[name] / waves
        if c.get("SQ_WAVE_CYCLES"):
            for name in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
                if name in c:
                    ent[name + "_frac_of_wave_cycles"] = c[name] / c["SQ_WAVE_CYCLES"]
        if "FETCH_SIZE" in c:
            ent["hbm_read_bytes"] = c["FETCH_SIZE"] * 1024 * 2
        if "WRITE_SIZE" in c:
            ent["hbm_write_bytes"] = c["WRITE_SIZE"] * 1024
        out["kernels"][want] = ent
    with open(dst, "w") as f:
        json.dump(out, f, indent=1)
    for want, e in out["kernels"].items():
        keep = {k: (round(v, 3) if isinstance(v, float) else v) for k, v in e.items() if k not in ("counters", "kernel")}
        print(want, json.dumps(keep))


if __name__ == "__main__":
    main()
