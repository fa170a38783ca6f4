#!/usr/bin/env python3
"""bench.py -- CRC32C GiB/s, device-resident, batched WAL records, on 1..8 MI355X.

Contract (driver): ``python bench.py --gpus N --steps K --warmup W``; for N > 1 either launched
by ``torch.distributed.run`` with one rank per GPU, or run as a plain command, in which case this
process starts the N ranks itself (``launch_ranks``: the same arguments, torch.distributed.run's
environment contract, before anything touches a GPU) and exits with the worst rank's status.
One "step" = one pass of the hot path over
one batch: every rank checksums its shard of records (``karma_crc32c_batch_fixed``) and, for
N > 1, the per-record CRCs are gathered to rank 0 over RCCL (``karma_crc32c_gather_u32``).
Rank 0 prints ONE JSON line.

Default workload = BASELINE.json configs[1]: 1M x 4 KiB records per GPU (weak scaling), bytes
of the splitmix64 stream generated on the device before timing (inputs resident in HBM).
Other workloads (``--workload ragged|stream|host``) measure configs[2], configs[3] and the
PCIe-inclusive host-memory path; they are reported in DESIGN.md, not by the driver.
``--dry-backend gloo`` runs the N-rank plumbing on CPU processes (tests/test_bench_launch.py): no
GPU, the host crc32c::Value for the batch, a gloo gather for RCCL; its line is not a measurement.
"""
from __future__ import annotations

import argparse
import json
import math
import os
import platform
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak, GB/s (MI355X_MICROARCH.md chip table)
GIB = float(1 << 30)
METRIC = "CRC32C GiB/s device-resident, batched WAL records, 1/2/4/8 MI355X"
CONFIG5_RECORDS = 256 << 20  # BASELINE configs[4]: 256M x 4 KiB records over 8 GPUs


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=200)
    p.add_argument("--warmup", type=int, default=50)  # the first 20-40 dispatches run slow
    p.add_argument("--workload", default="fixed",
                   choices=["fixed", "ragged", "stream", "segment", "host", "wal_append", "wal_replay", "kfp_encode",
                            "kfp_parse"])
    p.add_argument("--wal-record", type=int, default=180, help="wal_* payload bytes (configs[0]: ~180 B)")
    p.add_argument("--wal-mix", default="fixed", choices=["fixed", "config3"],
                   help="wal_*: every payload --wal-record bytes, or configs[2]'s log-uniform 64 B-64 KiB mix (~4 GiB)")
    p.add_argument("--wal-image", default="pinned", choices=["pinned", "pageable"],
                   help="wal_*: the WAL image in page-locked host memory (a writer's own write buffer, like "
                        "sivir's aligned O_DIRECT buffer: replay DMAs it with no staging copy) or in pageable memory "
                        "(replay stages it); the other mode is measured too (a shorter run) and reported beside it")
    p.add_argument("--records-per-gpu", type=int, default=0,
                   help="0 = the BASELINE config of the run: configs[1]'s 1M x 4 KiB per GPU, or with --gpus 8 "
                        "configs[4]'s shard, 256M / 8 = 33,554,432 records of 4 KiB per GPU")
    p.add_argument("--prewarm-ms", type=float, default=400.0,
                   help="time-based burn of the same step before --warmup (the GPU's clocks settle: "
                        "tools/ramp_probe.py, DESIGN.md §4); outside the timed region, reported as prewarm_ms")
    p.add_argument("--rec-bytes", type=int, default=4096)
    p.add_argument("--seed", type=int, default=42)
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--call-events", choices=["auto", "on", "off"], default="auto",
                   help="bracket every call with its own events too (auto: when a call is more than one kernel)")
    p.add_argument("--no-numa-bind", action="store_true",
                   help="do not restrict the process to the CPUs of its GPU's NUMA node")
    p.add_argument("--cpu-threads", type=int, default=0, help="0 = every CPU this process may run on (affinity)")
    p.add_argument("--pmc", default=os.path.join(ROOT, "profiles", "pmc_fixed_4k.json"),
                   help="per-launch HBM bytes from a rocprofv3 --pmc pass (tools/profile.sh)")
    p.add_argument("--streams", type=int, choices=[1, 2], default=1,
                   help="fixed workload, one GPU: consecutive batches on 1 or 2 streams (2: each into its own "
                        "output buffer, so batch i + 1 may start while batch i drains)")
    p.add_argument("--dry-backend", choices=["gloo"], default=None,
                   help="test the N-rank plumbing on CPU (tests/test_bench_launch.py): ranks over gloo, the "
                        "device batch replaced by the library's host crc32c::Value, the RCCL gather by "
                        "torch.distributed.gather; no GPU is touched and the line is not a measurement")
    p.add_argument("--dry-fail-rank", type=int, default=-1,
                   help="--dry-backend only: this rank exits with status 3 before joining the group "
                        "(the launcher must end the others and report 3)")
    return p.parse_args()


# ---------------------------------------------------------------------------------------------
def _free_port() -> int:
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _exit_status(code: int) -> int:
    """A child's return code as a shell exit status (a signal -S becomes 128 + S)."""
    return 128 - code if code < 0 else code


def launch_ranks(argv, n: int, grace_s: float = 20.0) -> int:
    """Start N ranks of this script as child processes with torch.distributed.run's environment
    (RANK, LOCAL_RANK, WORLD_SIZE, LOCAL_WORLD_SIZE, MASTER_ADDR=127.0.0.1, MASTER_PORT), the same
    arguments, and wait for them.  Called before torch is imported: the parent never initialises
    a GPU or loads the HIP library, so starting children is safe.  When a rank fails, the others
    would block in their next collective: they get `grace_s` to finish, then are terminated (the
    exact PIDs started here); a SIGTERM / SIGINT / SIGHUP to this process is passed on to the ranks
    before it exits.  Returns the worst exit status of the ranks that ended on their own
    (0 only if every rank returned 0); ranks terminated here do not mask the failure's status."""
    import signal
    import subprocess
    port = int(os.environ.get("MASTER_PORT") or _free_port())
    script = os.path.abspath(__file__)
    procs = []

    def forward(signum, frame):  # a launcher told to stop stops its ranks first (no orphan holds a GPU)
        for p in procs:
            if p.poll() is None:
                p.send_signal(signum)
        for p in procs:
            try:
                p.wait(10)
            except subprocess.TimeoutExpired:
                p.kill()
        sys.exit(128 + signum)

    for sig in (signal.SIGTERM, signal.SIGINT, signal.SIGHUP):
        signal.signal(sig, forward)
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, script] + list(argv), env=env))
    codes = [None] * n
    failed_at = own = None
    while any(c is None for c in codes):
        for i, p in enumerate(procs):
            if codes[i] is None:
                codes[i] = p.poll()
        if failed_at is None and any(c not in (None, 0) for c in codes):
            failed_at = time.monotonic()
        if failed_at is not None and time.monotonic() - failed_at > grace_s:
            own = [_exit_status(c) for c in codes if c is not None]
            for i, p in enumerate(procs):
                if codes[i] is None:
                    p.terminate()
            for i, p in enumerate(procs):
                if codes[i] is None:
                    try:
                        codes[i] = p.wait(10)
                    except subprocess.TimeoutExpired:
                        p.kill()
                        codes[i] = p.wait()
        time.sleep(0.05)
    statuses = [_exit_status(c) for c in codes]
    if any(statuses):
        print(f"bench.py: rank exit statuses {statuses}", file=sys.stderr, flush=True)
    return max(own) if own is not None else max(statuses)


# ---------------------------------------------------------------------------------------------
def host_cpus() -> int:
    """CPUs this process may run on (its affinity mask)."""
    try:
        return len(os.sched_getaffinity(0))
    except AttributeError:  # pragma: no cover - non-Linux
        return os.cpu_count() or 1


def bind_to_gpu_node(torch, local: int):
    """Restrict this process to the CPUs of its GPU's PCIe root (sysfs local_cpulist), as a
    deployment runs one process per GPU bound to that GPU's NUMA node (numactl --cpunodebind).
    Done before any host buffer is allocated, so the bench's host memory is first-touched on
    that node too.  Host-memory paths (WAL append / replay from host memory) depend on it: the
    library's copy threads otherwise float over both sockets (1M x 180 B append: 27 GiB/s
    unbound, 33 bound).  Returns a description, or None if unknown."""
    try:
        p = torch.cuda.get_device_properties(local)
        bus = f"{p.pci_domain_id:04x}:{p.pci_bus_id:02x}:{p.pci_device_id:02x}.0"
        with open(f"/sys/bus/pci/devices/{bus}/local_cpulist") as f:
            spec = f.read().strip()
        with open(f"/sys/bus/pci/devices/{bus}/numa_node") as f:
            node = f.read().strip()
        cpus = set()
        for part in spec.split(","):
            a, _, b = part.partition("-")
            cpus.update(range(int(a), int(b or a) + 1))
        want = cpus & os.sched_getaffinity(0)
        if not want:
            return None
        os.sched_setaffinity(0, want)
        return f"NUMA node {node} of GPU {bus}: {len(want)} CPUs ({spec})"
    except (AttributeError, OSError, ValueError):
        return None


def cgroup_cpu_quota():
    """The cgroup v2 CPU quota in CPUs (cpu.max), or None when unlimited / unreadable."""
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, period = f.read().split()
        return None if q == "max" else round(int(q) / int(period), 2)
    except (OSError, ValueError):
        return None


def baseline_threads(affinity) -> int:
    """Threads of the headline CPU baseline: the CPUs the process may use AND the CPU time the
    cgroup grants it, min(affinity CPUs, ceil(cgroup quota)).  More threads than the quota only
    time-slice (the box grants 16 CPUs of 256 visible: 128 threads there measured 23 % below 16)."""
    q = cgroup_cpu_quota()
    n = len(affinity)
    return max(1, min(n, math.ceil(q))) if q else n


class Affinity:
    """Run a block on a given CPU set (the CPU baselines run on the process's original mask, not
    only the GPU's NUMA node the bench binds to), restoring the current mask afterwards."""

    def __init__(self, cpus):
        self.cpus = set(cpus) if cpus else None

    def __enter__(self):
        self.saved = os.sched_getaffinity(0)
        if self.cpus:
            os.sched_setaffinity(0, self.cpus)
        return self

    def __exit__(self, *exc):
        os.sched_setaffinity(0, self.saved)
        return False


def cpu_baseline(workload: str, rec_bytes: int, threads: int, sample=None, orig_cpus=None, node_cpus=None) -> dict:
    """Reference crc32c (oracle/_ref, built from /root/reference/karma-util/crc32c.cc) on host cores.

    A bounded sample of the same workload, at least 1 GiB (larger than the host's last-level
    cache, so it streams from DRAM like the device batch streams from HBM), checksummed for ~2 s
    per figure, records round-robin over std::threads:
      value (headline) -- `threads` threads (baseline_threads: min(affinity CPUs, ceil(cgroup
                          quota))) on the process's ORIGINAL affinity mask `orig_cpus` (before the
                          bench bound itself to its GPU's NUMA node);
      single_thread_value, all_affinity_value (one thread per CPU of the original mask: more than
      the quota, so time-sliced), numa_node_value (the node's CPUs, on the node the bench binds to).
    Samples:
      fixed/host -- the first 1 GiB of records of the timed batch (`sample`, copied off the device);
      ragged     -- the first ~1 GiB of records of the configs[2] layout (same lengths, seed 7);
      stream     -- 16 distinct 64 MiB segments (one thread per segment at most).
    """
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_lib  # the CPU checker; only the cpu_baseline leg touches it
    import synth
    ref = oracle_lib.ref()
    kind = "reference" if ref is not None else "port"
    if workload == "ragged":
        lens_all = synth.loguniform_lengths(7, 1 << 20, 64, 65536)
        k = int(np.searchsorted(np.cumsum(lens_all, dtype=np.uint64), np.uint64(1 << 30)))
        lens = lens_all[:max(k, 1)].astype(np.uint32)
        offs, arena_bytes = synth.ragged_layout(lens, header=8)
        buf = sample[: arena_bytes + 16] if sample is not None and sample.size >= arena_bytes + 16 else \
            synth.splitmix_np(42, 0, arena_bytes + 16).copy()
        offs = np.ascontiguousarray(offs.astype(np.uint64))
        n, nbytes = lens.size, int(lens.sum())
        out = np.empty(n, dtype=np.uint32)
        desc = f"{n} ragged records (log-uniform 64 B-64 KiB, configs[2] layout, {nbytes >> 20} MiB payload)"

        def run(nthr):
            if ref is not None:
                ref.ref_crc32c_ragged_mt(buf.ctypes.data, offs.ctypes.data, lens.ctypes.data, None, n,
                                         out.ctypes.data, nthr)
            else:
                oracle_lib.port().oracle_ragged_crcs(buf.ctypes.data, offs.ctypes.data, lens.ctypes.data, None, n,
                                                     out.ctypes.data, nthr)
    else:
        if workload in ("stream", "segment"):
            rec_bytes, n = 64 << 20, 16
        else:
            n = max(1, (1 << 30) // rec_bytes)
        nbytes = n * rec_bytes
        if sample is not None and sample.size >= nbytes:
            buf = np.ascontiguousarray(sample[:nbytes])
        else:
            buf = synth.splitmix_np(42, 0, nbytes).copy()
        out = np.empty(n, dtype=np.uint32)
        desc = f"{n} x {rec_bytes} B splitmix64 records of the timed batch ({nbytes >> 20} MiB)"

        def run(nthr):
            nthr = min(nthr, n)
            if ref is not None:
                ref.ref_crc32c_fixed_mt(buf.ctypes.data, rec_bytes, n, out.ctypes.data, nthr)
            else:
                oracle_lib.port().oracle_fixed_crcs(buf.ctypes.data, rec_bytes, n, out.ctypes.data, nthr)

    def rate(nthr, budget):
        run(nthr)
        reps, t0 = 0, time.perf_counter()
        while True:
            run(nthr)
            reps += 1
            dt = time.perf_counter() - t0
            if dt > budget:
                return reps * nbytes / dt / GIB, reps

    orig_cpus = set(orig_cpus) if orig_cpus else os.sched_getaffinity(0)
    with Affinity(orig_cpus):
        multi, reps_m = rate(threads, 2.0)
        single, _ = rate(1, 2.0)
        all_aff = rate(len(orig_cpus), 2.0)[0] if len(orig_cpus) != threads else multi
    node = None
    if node_cpus and set(node_cpus) != orig_cpus:
        with Affinity(node_cpus):
            node = rate(len(node_cpus), 2.0)[0]
    cpu = platform.processor() or platform.machine()
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    cpu = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return {"value": round(multi, 3), "unit": "GiB/s", "cores": threads, "kind": kind,
            "sample": f"{desc}, crc32c::Value per record, round-robin over {threads} std::threads "
                      f"(min(affinity CPUs, ceil(cgroup quota)), on the process's original CPU mask), "
                      f"repeated {reps_m}x (~2 s)",
            "threads_rule": "min(affinity CPUs, ceil(cgroup cpu.max quota))",
            "single_thread_value": round(single, 3),
            "all_affinity_value": round(all_aff, 3), "all_affinity_threads": len(orig_cpus),
            "numa_node_value": round(node, 3) if node is not None else None,
            "numa_node_threads": len(node_cpus) if node is not None else None,
            "cpu_model": cpu, "host_cpus_affinity": len(orig_cpus), "host_cpus_visible": os.cpu_count(),
            "cgroup_cpu_quota": cgroup_cpu_quota()}


def units_kernel_name(wl: str) -> str:
    """The dominant kernel a batch runs (capi.cc planning, crc_fixed.hip / crc_ragged.hip launchers)."""
    return {"ragged": "k_units_ragged", "segment": "k_segment_once"}.get(wl, "k_units_fixed")


def pmc_traffic(path: str, workload: str, n_bytes_per_launch: int):
    try:
        with open(path) as f:
            d = json.load(f)
    except (OSError, ValueError):
        return None
    if d.get("workload") != workload or int(d.get("payload_bytes_per_launch", -1)) != n_bytes_per_launch:
        return None
    return d.get("hbm_bytes_per_launch")


REPLAY_PMC = "r06wide_wal_replay_pmc.json"  # tools/pmc_replay.sh + tools/pmc_kernels.py: the uniform-stride pass


def replay_pmc_traffic(n_rec: int, rec_bytes: int):
    """(HBM bytes of the replay's CRC kernel per launch, of the whole call) from the per-kernel PMC
    file of tools/pmc_replay.sh (FETCH_SIZE x 2 + WRITE_SIZE per dispatch; the call: the kernels
    the file lists, summed -- for the uniform-stride pass its one kernel), whose calls replay
    tools/replay_study.py's default image: 1M x 180 B records in 1 MiB segments.  (None, None) for
    another shape (not measured)."""
    if (n_rec, rec_bytes) != (1 << 20, 180):
        return None, None
    try:
        with open(os.path.join(ROOT, "profiles", REPLAY_PMC)) as f:
            ks = json.load(f)["kernels"]
        crc = ks["k_ragged_staged_pipe"]
        return (float(crc["hbm_read_bytes"] + crc["hbm_write_bytes"]),
                float(sum(k["hbm_read_bytes"] + k["hbm_write_bytes"] for k in ks.values())))
    except (OSError, ValueError, KeyError, TypeError):
        return None, None


# ---------------------------------------------------------------------------------------------
def wal_bench(args, L, rank):
    """configs[0] shape end to end from host memory: karma_wal_append_batch (sivir::build_sqe +
    append_record framing, CRCs in one GPU batch) or karma_wal_replay (sivir::open's scan_record
    loop) over n records of --wal-record bytes in 1 MiB segments (options.h:8).  The CPU
    baseline is the reference's crc32c::Value in the same framing / replay loop
    (oracle/ref_shim.cc ref_wal_append_mt / ref_wal_replay_mt), 1 thread and 16 independent WALs."""
    import ctypes
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import synth
    from karma_amd import _lib
    seg = 1 << 20
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.wal_mix == "config3":  # configs[2]'s replay mix framed into 1 MiB segments
        import torch
        import karma_amd as K
        count = int((4 << 30) / (((65536 - 64) / np.log(1024)) + 8))
        lens = synth.loguniform_lengths(7, count, 64, 65536).astype(np.uint32)
        n, size = count, None
        offs = np.concatenate([[0], np.cumsum(lens, dtype=np.uint64)[:-1]]).astype(np.uint64)
        total = int(lens.sum())
        d_src = torch.empty(total + 16, dtype=torch.uint8, device=torch.device("cuda", local))
        K.fill_splitmix64(d_src, args.seed + rank)
        src = d_src.cpu().numpy()
        del d_src
        # every segment loses at most one record's header + payload to its footer
        wal_bytes = ((total + 8 * n) // (seg - 65544) + 2) * seg
    else:
        n, size = args.records_per_gpu or (1 << 20), args.wal_record
        lens = np.full(n, size, dtype=np.uint32)
        offs = (np.arange(n, dtype=np.uint64) * np.uint64(size)).astype(np.uint64)
        src = synth.splitmix_np(args.seed + rank, 0, n * size + 16).copy()
        per_seg = seg // (size + 8)
        wal_bytes = ((n + per_seg - 1) // per_seg + 1) * seg
    payload = int(lens.sum())
    import torch
    images = {"pageable": np.zeros(wal_bytes, dtype=np.uint8),
              "pinned": torch.zeros(wal_bytes, dtype=torch.uint8).pin_memory().numpy()}
    wal = images[args.wal_image]
    cur, nf = ctypes.c_uint64(0), ctypes.c_size_t()

    def append():
        cur.value = 0
        _lib.check("wal_append", L.karma_wal_append_batch(src.ctypes.data, offs.ctypes.data, lens.ctypes.data, n,
                                                          wal.ctypes.data, wal_bytes, seg, ctypes.byref(cur), None,
                                                          ctypes.byref(nf), local))
        assert nf.value == n

    nrec, stop, status = ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_int()

    def replay():
        _lib.check("wal_replay", L.karma_wal_replay(wal.ctypes.data, None, wal_bytes, seg, 0, ctypes.byref(nrec),
                                                    ctypes.byref(stop), ctypes.byref(status), None, 0, local))
        assert nrec.value == n

    append()
    other = "pageable" if args.wal_image == "pinned" else "pinned"
    images[other][:] = wal  # the same image in the other kind of host memory
    step = append if args.workload == "wal_append" else replay
    dev_rate = dir_rate = None
    dev_single = None
    if args.workload == "wal_replay":
        # The same replay over copies already in HBM (no upload).  Four distinct images (payloads
        # of other seeds, same framing: 4 x ~201 MB > 512 MiB) are replayed in rotation, so no call
        # finds its image in the 256 MB Infinity Cache the previous call left: the
        # rotated rate is the HBM figure.  The single reused image is reported beside it.
        import torch
        d_wals = [torch.from_numpy(wal).to(torch.device("cuda", local))]
        img_k = np.zeros_like(wal)
        for k in range(1, 4):
            src_k = synth.splitmix_np(args.seed + rank + 1000 * k, 0, src.size).copy()
            cur.value = 0
            _lib.check("wal_append", L.karma_wal_append_batch(src_k.ctypes.data, offs.ctypes.data, lens.ctypes.data,
                                                              n, img_k.ctypes.data, wal_bytes, seg, ctypes.byref(cur),
                                                              None, ctypes.byref(nf), local))
            d_wals.append(torch.from_numpy(img_k).to(torch.device("cuda", local)))
            del src_k
        del img_k
        rot = {"i": 0, "k": len(d_wals)}

        def replay_dev():
            d_wal = d_wals[rot["i"] % rot["k"]]
            rot["i"] += 1
            _lib.check("wal_replay", L.karma_wal_replay(None, d_wal.data_ptr(), wal_bytes, seg, 0, ctypes.byref(nrec),
                                                        ctypes.byref(stop), ctypes.byref(status), None, 0, local))
            assert nrec.value == n

        for k in (len(d_wals), 1):  # rotated, then the single image
            rot["k"] = k
            for _ in range(args.warmup):
                replay_dev()
            t0 = time.perf_counter()
            for _ in range(args.steps):
                replay_dev()
            r = payload / ((time.perf_counter() - t0) / args.steps) / GIB
            if k > 1:
                dev_rate = r
            else:
                dev_single = r
        # the same rotated images through the walk (the path of WALs whose records vary in size):
        # a forced sub-range size -- the planner's own for these images -- skips the uniform-stride pass
        walk_rate = None
        if size:
            rot["k"] = len(d_wals)
            tune = _lib.WalTuning(40960, _lib.KARMA_WAL_CRC_PLAN, 0)

            def replay_walk():
                d_wal = d_wals[rot["i"] % rot["k"]]
                rot["i"] += 1
                _lib.check("wal_replay_tuned", L.karma_wal_replay_tuned(
                    None, d_wal.data_ptr(), wal_bytes, seg, 0, ctypes.byref(nrec), ctypes.byref(stop),
                    ctypes.byref(status), None, 0, local, ctypes.byref(tune)))
                assert nrec.value == n

            for _ in range(args.warmup):
                replay_walk()
            t0 = time.perf_counter()
            for _ in range(args.steps):
                replay_walk()
            walk_rate = payload / ((time.perf_counter() - t0) / args.steps) / GIB
        # the replay's CRC kernel alone (HIP events the library records on its replay stream
        # around that launch: karma_crc32c_time_next_units), rotated images, after the timed loop
        rot["k"] = len(d_wals)
        crc_ms = []
        for _ in range(max(8, min(args.steps, 32))):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()  # (torch only times events it has recorded once; the library re-records them)
            e1.record()
            torch.cuda.synchronize()
            L.karma_crc32c_time_next_units(e0.cuda_event, e1.cuda_event)
            replay_dev()
            e1.synchronize()
            crc_ms.append(e0.elapsed_time(e1))
        crc_kernel_ms = float(np.median(crc_ms))
        del d_wals
        # the same replay from segment files named by their WAL offsets (karma_wal_replay_dir),
        # page-cached: the files are read straight into the pinned staging buffers
        import shutil
        import tempfile
        tmp = tempfile.mkdtemp(prefix="karma_wal_", dir="/dev/shm" if os.path.isdir("/dev/shm") else None)
        try:
            for i in range(wal_bytes // seg):
                wal[i * seg:(i + 1) * seg].tofile(os.path.join(tmp, str(i * seg)))
            base = ctypes.c_uint64()

            def replay_dir():
                _lib.check("wal_replay_dir", L.karma_wal_replay_dir(tmp.encode(), seg, 0, ctypes.byref(base),
                                                                    ctypes.byref(nrec), ctypes.byref(stop),
                                                                    ctypes.byref(status), None, 0, local))
                assert nrec.value == n

            for _ in range(args.warmup):
                replay_dir()
            t0 = time.perf_counter()
            for _ in range(args.steps):
                replay_dir()
            dir_rate = payload / ((time.perf_counter() - t0) / args.steps) / GIB
        finally:
            shutil.rmtree(tmp, ignore_errors=True)
    for _ in range(args.warmup):
        step()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    dt = (time.perf_counter() - t0) / args.steps
    mix = f"{n} x {size} B" if size else f"{n} log-uniform 64 B-64 KiB ({payload / GIB:.2f} GiB)"
    # the other kind of host memory, a shorter run of the same step
    keep, wal = wal, images[other]
    for _ in range(2):
        step()
    k_other = max(3, args.steps // 4)
    t1 = time.perf_counter()
    for _ in range(k_other):
        step()
    other_rate = payload / ((time.perf_counter() - t1) / k_other) / GIB
    wal = keep
    res = {"metric": METRIC + f" [{args.workload}: host memory end to end]",
           "value": round(payload / dt / GIB, 3), "unit": "GiB/s", "n_gpus": 1, "steps": args.steps,
           "warmup": args.warmup, "ms_per_step": round(dt * 1e3, 3), "higher_is_better": True, "scaling": "weak",
           "vs_baseline": None, "dtype": "u8",
           "data": f"synthetic splitmix64 payloads; the WAL image in {args.wal_image} host memory",
           "records_per_s": round(n / dt, 1), "wal_image": args.wal_image,
           f"{other}_image_value": round(other_rate, 3),
           "device_resident_value": round(dev_rate, 3) if dev_rate is not None else None,
           "device_resident_image_tbs": round(wal_bytes / (payload / dev_rate / GIB) / 1e12, 3)
           if dev_rate is not None else None,
           "device_resident_single_image_value": round(dev_single, 3) if dev_single is not None else None,
           "device_resident_walk_value": round(walk_rate, 3) if walk_rate is not None else None,
           "device_resident_walk_image_tbs": round(wal_bytes / (payload / walk_rate / GIB) / 1e12, 3)
           if walk_rate is not None else None,
           "device_resident_walk_note": "the same rotated images with the uniform-stride pass skipped (a forced "
                                        "40 KiB sub-range walk: the planner's own plan for them), i.e. the rate of "
                                        "the walk, gather and CRC batch that WALs of varying record sizes take"
           if walk_rate is not None else None,
           "device_resident_note": "karma_wal_replay over WAL images already in HBM, 4 distinct ~%d MB images "
                                   "in rotation (none left in the 256 MB MALL by the previous call); host wall "
                                   "clock over --steps synchronous calls; image TB/s = wal_bytes / call time; the "
                                   "single-image value reuses one image every call (MALL-resident)" % (wal_bytes // 10**6)
           if dev_rate is not None else None,
           "segment_files_value": round(dir_rate, 3) if dir_rate is not None else None,
           "config": {"workload": f"{mix} WAL records, 1 MiB segments, "
                                  f"{'karma_wal_append_batch' if step is append else 'karma_wal_replay'} "
                                  f"(BASELINE {'configs[0]' if size else 'configs[2]'} records)", "records": n,
                      "record_bytes": size},
           "roofline": None}
    if args.workload == "wal_replay" and dev_rate is not None:
        # the dominant kernel of a device-resident replay: for records of one size the
        # uniform-stride pass's CRC batch (each record's 8-byte header and payload, read once; no
        # lists), else the payload CRC batch over the gathered lists (payload bytes + offset 8 B,
        # length 4 B, stored CRC 4 B, result 4 B per record); the whole call's image rate beside it
        algo = n * (size + 8) if size else payload + 20 * n
        achieved = algo / (crc_kernel_ms * 1e-3) / 1e9
        call_s = payload / (dev_rate * GIB)
        pm, pm_call = replay_pmc_traffic(n, size) if size else (None, None)
        res["roofline"] = {"bound": "hbm", "achieved": round(achieved, 1), "peak": 8000.0, "unit": "GB/s",
                           "frac": round(achieved / 8000.0, 4), "traffic": round(pm) if pm is not None else None,
                           "traffic_source": f"profiles/{REPLAY_PMC} (FETCH_SIZE x 2 + WRITE_SIZE of the CRC "
                                             f"kernel per launch; a separate rocprofv3 --pmc pass, not this run)"
                           if pm is not None else None,
                           "call_traffic": round(pm_call) if pm_call is not None else None,
                           "call_traffic_vs_image": round(pm_call / wal_bytes, 3) if pm_call is not None else None,
                           "kernel": "the replay's CRC batch (k_ragged_staged_pipe" +
                                     (", uniform-stride form: headers and payloads of the slots)" if size else ")"),
                           "kernel_ms_avg": round(crc_kernel_ms, 4), "algorithmic_bytes_per_launch": algo,
                           "achieved_source": "algorithmic bytes / the CRC kernel's HIP-event time inside "
                                              "karma_wal_replay (rotated device-resident images)",
                           "call_image_bytes": wal_bytes, "call_ms": round(call_s * 1e3, 4),
                           "call_image_frac": round(wal_bytes / call_s / 8e12, 4)}
    if not args.no_cpu_baseline and size:
        import oracle_lib
        ref = oracle_lib.ref()
        if ref is not None:
            # one independent WAL per thread (one per sivir io thread), as many as the CPU grant
            # runs at once (baseline_threads), on the process's original CPU mask
            thr = args.cpu_threads or baseline_threads(args.orig_cpus)
            k = min(n, 1 << 20)
            img = ((k // thr + per_seg - 1) // per_seg + 2) * seg
            imgs = np.zeros(img * thr, dtype=np.uint8)

            def rate(nthr, fn):
                fn(nthr)
                reps, t1 = 0, time.perf_counter()
                while True:
                    got = fn(nthr)
                    reps += 1
                    el = time.perf_counter() - t1
                    if el > 2.0:
                        return got, reps * got * size / el / GIB, reps

            def app(nthr):
                return ref.ref_wal_append_mt(src.ctypes.data, offs.ctypes.data, lens.ctypes.data, k, imgs.ctypes.data,
                                             img, seg, nthr)

            def rep(nthr):
                return ref.ref_wal_replay_mt(imgs.ctypes.data, img, seg, nthr, nthr)

            fn = app if step is append else rep
            with Affinity(args.orig_cpus):
                app(thr)  # the images the replay baseline reads
                _, multi, reps = rate(thr, fn)
                _, single, _ = rate(1, fn)
            res["cpu_baseline"] = {"value": round(multi, 3), "unit": "GiB/s", "cores": thr, "kind": "reference",
                                   "sample": f"{k} x {size} B records framed ({'append' if fn is app else 'replay'}) "
                                             f"into {thr} independent WAL images, one per std::thread, reference "
                                             f"crc32c::Value, repeated {reps}x (~2 s)",
                                   "threads_rule": "min(affinity CPUs, ceil(cgroup cpu.max quota))",
                                   "cgroup_cpu_quota": cgroup_cpu_quota(),
                                   "single_thread_value": round(single, 3)}
    return res


def kfp_bench(args, L, rank):
    """KFP frame batches from host memory (frame::encode / connection::read_frame's parse loop,
    frame.cc:29-130): --records-per-gpu frames (default 256 Ki here) of a 64-byte header and a
    --rec-bytes payload; all frame CRCs of a call in one GPU batch."""
    import ctypes
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import synth
    from karma_amd import _lib
    n = args.records_per_gpu or (1 << 18)
    hl = np.full(n, 64, np.uint32)
    pl = np.full(n, args.rec_bytes, np.uint32)
    hsrc = synth.splitmix_np(args.seed + 2 * rank, 0, 64 * n + 8).copy()
    psrc = synth.splitmix_np(args.seed + 2 * rank + 1, 0, args.rec_bytes * n + 8).copy()
    hoff = (np.arange(n, dtype=np.uint64) * np.uint64(64)).astype(np.uint64)
    poff = (np.arange(n, dtype=np.uint64) * np.uint64(args.rec_bytes)).astype(np.uint64)
    op = np.ones(n, np.int16)
    flag = np.zeros(n, np.uint8)
    seq = np.arange(n, dtype=np.uint32)
    frame = 16 + 64 + args.rec_bytes + 4
    out = np.zeros(n * frame, np.uint8)
    local = int(os.environ.get("LOCAL_RANK", "0"))
    ne, nb = ctypes.c_size_t(), ctypes.c_uint64()

    def encode():
        _lib.check("kfp_encode", L.karma_kfp_encode_batch(hsrc.ctypes.data, hoff.ctypes.data, hl.ctypes.data,
                                                          psrc.ctypes.data, poff.ctypes.data, pl.ctypes.data,
                                                          op.ctypes.data, flag.ctypes.data, seq.ctypes.data, n,
                                                          out.ctypes.data, out.nbytes, None, ctypes.byref(ne),
                                                          ctypes.byref(nb), local))
        assert ne.value == n and nb.value == out.nbytes

    nf, used, why = ctypes.c_size_t(), ctypes.c_uint64(), ctypes.c_int()

    def parse():
        _lib.check("kfp_parse", L.karma_kfp_parse_batch(out.ctypes.data, None, out.nbytes, n, None, ctypes.byref(nf),
                                                        ctypes.byref(used), ctypes.byref(why), local))
        assert nf.value == n and why.value == 0

    encode()
    step = encode if args.workload == "kfp_encode" else parse
    for _ in range(args.warmup):
        step()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    dt = (time.perf_counter() - t0) / args.steps
    return {"metric": METRIC + f" [{args.workload}: host memory end to end]",
            "value": round(out.nbytes / dt / GIB, 3), "unit": "GiB/s", "n_gpus": 1, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(dt * 1e3, 3), "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "u8", "data": "synthetic splitmix64 headers and payloads in pageable host memory",
            "frames_per_s": round(n / dt, 1),
            "config": {"workload": f"{n} KFP frames of a 64 B header + {args.rec_bytes} B payload "
                                   f"({'karma_kfp_encode_batch' if step is encode else 'karma_kfp_parse_batch'})",
                       "frames": n, "frame_bytes": frame},
            "roofline": None}


def records_per_gpu(requested: int, world: int, workload: str):
    """(records per GPU, is it BASELINE configs[4]'s shard): --records-per-gpu when given, else
    configs[4] on 8 GPUs (256M x 4 KiB sharded: 33,554,432 per GPU, 128 GiB of HBM each) and
    configs[1] otherwise (1M x 4 KiB per GPU)."""
    if requested:
        return requested, False
    if world == 8 and workload == "fixed":
        return CONFIG5_RECORDS // 8, True
    return 1 << 20, False


def config5_anchor():
    """The one-GPU rate of configs[4]'s per-GPU shard (33,554,432 x 4 KiB, 128 GiB), measured by
    `bench.py --records-per-gpu 33554432` and committed under profiles/: the N = 8 line's per-GPU
    work at N = 1, so a scaling curve can separate shard size from scaling.  Not measured in
    this run; the source file is named."""
    for name in ("r06final_bench_config5_slice.json", "r03_bench_config5_slice.json", "r02_bench_config5_slice.json"):
        path = os.path.join(ROOT, "profiles", name)
        try:
            with open(path) as f:
                d = json.loads(f.read().strip().splitlines()[-1])
            return {"value": d["value"], "unit": d.get("unit", "GiB/s"),
                    "frac": d.get("roofline", {}).get("frac"), "source": f"profiles/{name}"}
        except (OSError, ValueError, KeyError, IndexError):
            continue
    return None


class TorchSync:
    """Streams and events of the GPU run: the compute stream (the caller's), a second stream for
    the gather, torch.cuda events between them."""

    def __init__(self, torch, compute_stream):
        self.torch = torch
        self.compute_stream = compute_stream
        self.gather_stream = torch.cuda.Stream()

    def event(self):
        return self.torch.cuda.Event()

    def record(self, ev, stream):
        ev.record(stream)

    def wait(self, stream, ev):
        stream.wait_event(ev)


class GatherPipeline:
    """The N > 1 step of the bench: step i checksums this rank's shard into outs[i % S] on the
    compute stream; the gather of that buffer to rank 0 (karma_crc32c_gather_u32 over RCCL) runs
    on the gather stream, ordered after the compute by an event, while step i + 1 computes into
    the other buffer; step i + S first waits for the gather that last read its buffer.  With one
    buffer and no gather (N = 1) a step is just the compute.

    `compute(out)` enqueues the batch into `out`; `gather(out, stream)` enqueues the gather of
    `out`; `sync` supplies streams and events (TorchSync here, a logging host stand-in in
    tests/test_bench_pipeline.py, which drives this class over gloo on CPU)."""

    def __init__(self, outs, compute, gather, sync):
        self.outs, self.compute, self.gather, self.sync = outs, compute, gather, sync
        self.computed = [sync.event() for _ in outs] if gather else []
        self.gathered = [sync.event() for _ in outs] if gather else []
        self.i = 0
        self.current = outs[0]

    def crc_step(self):
        slot = self.i % len(self.outs)
        if self.gather is not None and self.i >= len(self.outs):
            self.sync.wait(self.sync.compute_stream, self.gathered[slot])  # its last gather is done
        self.current = self.outs[slot]
        self.compute(self.current)
        self.i += 1

    def gather_step(self):
        if self.gather is None:
            return
        slot = (self.i - 1) % len(self.outs)  # the buffer the last crc_step wrote
        self.sync.record(self.computed[slot], self.sync.compute_stream)
        self.sync.wait(self.sync.gather_stream, self.computed[slot])
        self.gather(self.outs[slot], self.sync.gather_stream)
        self.sync.record(self.gathered[slot], self.sync.gather_stream)


def shard_self_check(arena, out, rec: int, n_rec: int, value, seed: int = 1, first: int = 64, rand: int = 64):
    """A sampled set of this rank's records checked after timing: the device CRCs of the first
    `first` records and `rand` random ones against value(bytes) (the host crc32c::Value of the
    product library: include/karma-util/crc32c.h).  arena / out are tensors (the rank's shard and
    its CRCs, on the device on the box; CPU tensors in tests/test_bench_pipeline.py).  Returns the
    record indices, their device CRCs (so rank 0 can check the gathered copy) and the mismatches."""
    import torch
    idx = np.unique(np.concatenate([np.arange(min(first, n_rec)),
                                    np.random.default_rng(seed).integers(0, n_rec, rand)])).astype(np.int64)
    o = out.view(torch.int32) if out.dtype == torch.uint32 else out  # (uint32 tensors index poorly)
    got = o[torch.from_numpy(idx).to(out.device)].cpu().numpy().astype(np.int64).astype(np.uint32)
    bad = 0
    for j, r in enumerate(idx):
        b = arena[int(r) * rec:(int(r) + 1) * rec].cpu().numpy()
        bad += int(int(value(b)) != int(got[j]))
    return {"idx": idx.tolist(), "crc": [int(x) for x in got], "mismatches": bad}


def aggregate_self_checks(checks, gathered=None, n_rec: int = 0):
    """Rank 0's view of every rank's shard_self_check (all-gathered): per rank the records
    sampled and mismatches, the totals, and -- with the CRCs rank 0 gathered over RCCL
    (`gathered`, n_rec per rank in rank order) -- how many sampled CRCs differ in the gathered
    copy (a gather that misplaces or corrupts a shard shows here)."""
    per_rank = [{"sampled_records": len(c["idx"]), "mismatches": int(c["mismatches"])} for c in checks]
    total = {"sampled_records": sum(p["sampled_records"] for p in per_rank),
             "mismatches": sum(p["mismatches"] for p in per_rank), "ranks": len(checks),
             "check": "per rank: the first 64 and 64 random records of its shard, device CRC vs host crc32c::Value"}
    if gathered is not None:
        g = np.asarray(gathered)
        total["gather_mismatches"] = int(sum(int(g[r * n_rec + i]) != int(v) for r, c in enumerate(checks)
                                             for i, v in zip(c["idx"], c["crc"])))
    return per_rank, total


class HostSync:
    """GatherPipeline's streams and events for the dry run: work runs at once on the host, so
    events only need to exist and be recorded before they are waited on."""

    compute_stream, gather_stream = "compute", "gather"

    def event(self):
        return {"recorded": False}

    def record(self, ev, stream):
        ev["recorded"] = True

    def wait(self, stream, ev):
        assert ev["recorded"], "waits on an event never recorded"


def dry_main(args, world: int, rank: int):
    """--dry-backend gloo: the N-rank path of main() -- rank launch, GatherPipeline, barrier +
    synchronise around K steps, max-over-ranks time, every rank's self-check aggregated on rank 0,
    one JSON line from rank 0 -- on CPU processes over gloo (tests/test_bench_launch.py).  The
    device batch is replaced by the product library's host crc32c::Value per record
    (host_crc32c.cc), the RCCL gather by torch.distributed.gather.  Nothing touches a GPU; the
    line is marked dry and is not a measurement.  It carries a digest of the CRCs rank 0 gathered,
    so the test can check every shard against the oracle."""
    import hashlib

    import torch
    import torch.distributed as dist
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import synth

    import karma_amd as K
    if rank == args.dry_fail_rank:
        raise SystemExit(3)
    if world > 1:
        dist.init_process_group("gloo")
    n_rec = args.records_per_gpu or 2048
    rec = args.rec_bytes
    payload = n_rec * rec
    host = synth.splitmix_np(args.seed, rank * payload, payload).copy()  # bench's fill: first_byte = rank * payload
    arena = torch.from_numpy(host)
    outs = [torch.zeros(n_rec, dtype=torch.int64) for _ in range(2 if world > 1 else 1)]
    gathered = {"last": None}

    def compute(o):
        o.copy_(torch.from_numpy(np.array([K.Value(host[i * rec:(i + 1) * rec]) for i in range(n_rec)],
                                          dtype=np.int64)))

    def gather(o, stream):
        full = [torch.zeros(n_rec, dtype=torch.int64) for _ in range(world)] if rank == 0 else None
        dist.gather(o, full, dst=0)
        if rank == 0:
            gathered["last"] = torch.cat(full)

    pipe = GatherPipeline(outs, compute, gather if world > 1 else None, HostSync())
    for _ in range(args.warmup):
        pipe.crc_step()
        pipe.gather_step()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        pipe.crc_step()
        pipe.gather_step()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    mine = shard_self_check(arena, pipe.current, rec, n_rec, K.Value, seed=1 + rank)
    res = None
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        checks = [None] * world
        dist.all_gather_object(checks, mine)
        if rank == 0:
            g = gathered["last"].numpy()
            per, check = aggregate_self_checks(checks, g, n_rec)
            res = {"per_rank": {"self_check": per}, "self_check": check,
                   "gathered_crcs": int(g.size),
                   "gathered_sha256_16": hashlib.sha256(g.astype("<u4").tobytes()).hexdigest()[:16]}
    elif rank == 0:
        g = pipe.current.numpy()
        res = {"self_check": {"sampled_records": len(mine["idx"]), "mismatches": mine["mismatches"]},
               "gathered_crcs": int(g.size),
               "gathered_sha256_16": hashlib.sha256(g.astype("<u4").tobytes()).hexdigest()[:16]}
    if rank == 0:
        line = {"metric": METRIC + " [dry run: gloo ranks on CPU, host crc32c::Value; not a measurement]",
                "value": round(payload * world * args.steps / elapsed / GIB, 4), "unit": "GiB/s",
                "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
                "ms_per_step": round(elapsed / args.steps * 1e3, 4), "higher_is_better": True, "scaling": "weak",
                "vs_baseline": None, "dtype": "u8", "data": "synthetic splitmix64 records on the host",
                "config": {"workload": f"{n_rec} x {rec} B records per rank", "records_per_gpu": n_rec,
                           "rec_bytes": rec, "parallelism": f"record-sharded x{world}"
                           + (" + gloo gather to rank 0" if world > 1 else "")},
                "roofline": None, "dry_backend": args.dry_backend, "rccl_nranks": None,
                "dry_nranks": dist.get_world_size() if world > 1 else 1,
                "launched_by": os.environ.get("KARMA_BENCH_LAUNCHER", "external")}
        line.update(res)
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        # a plain `python bench.py --gpus N`: start the N ranks here, before torch is imported
        os.environ["KARMA_BENCH_LAUNCHER"] = "bench.py"
        sys.exit(launch_ranks(sys.argv[1:], args.gpus, float(os.environ.get("KARMA_BENCH_GRACE_S", "20"))))
    if args.dry_backend:
        return dry_main(args, world, rank)
    import torch
    import torch.distributed as dist

    ndev = torch.cuda.device_count()
    local = local % max(ndev, 1)  # one rank per GPU; several ranks per GPU only for plumbing checks
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    args.orig_cpus = os.sched_getaffinity(0)  # before binding: the CPU baselines run on the whole mask
    numa = None if args.no_numa_bind else bind_to_gpu_node(torch, local)
    args.node_cpus = os.sched_getaffinity(0) if numa else None
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)

    import karma_amd as K
    from karma_amd import _lib

    L = _lib.lib()
    stream = torch.cuda.current_stream()
    sh = stream.cuda_stream

    comm = None
    rccl_nranks = None
    if world > 1:
        import ctypes
        uid = (ctypes.c_char * _lib.UNIQUE_ID_BYTES)()
        if rank == 0:
            _lib.check("get_unique_id", L.karma_crc32c_get_unique_id(uid, _lib.UNIQUE_ID_BYTES))
        obj = [bytes(uid) if rank == 0 else None]
        dist.broadcast_object_list(obj, src=0)
        uid = (ctypes.c_char * _lib.UNIQUE_ID_BYTES).from_buffer_copy(obj[0])
        comm = ctypes.c_void_p()
        _lib.check("comm_init", L.karma_crc32c_comm_init(ctypes.byref(comm), world, uid, rank))
        cnt = ctypes.c_int()
        _lib.check("comm_count", L.karma_crc32c_comm_count(comm, ctypes.byref(cnt)))
        rccl_nranks = cnt.value
        if rccl_nranks != world:
            raise SystemExit(f"RCCL reports {rccl_nranks} ranks, torch.distributed {world}")

    wl = args.workload
    if wl in ("wal_append", "wal_replay", "kfp_encode", "kfp_parse"):
        res = wal_bench(args, L, rank) if wl.startswith("wal") else kfp_bench(args, L, rank)
        if rank == 0:
            res["host_binding"] = numa
            print(json.dumps(res), flush=True)
        if comm is not None:
            L.karma_crc32c_comm_destroy(comm)
        if world > 1:
            dist.barrier()
            dist.destroy_process_group()
        return
    n_rec, config5 = records_per_gpu(args.records_per_gpu, world, args.workload)
    rec = args.rec_bytes
    cur = {}  # the output buffer the next crc_step writes (double-buffered for N > 1)
    if wl == "fixed":
        payload = n_rec * rec
        arena = torch.empty(payload, dtype=torch.uint8, device=dev)
        K.fill_splitmix64(arena, args.seed, first_byte=rank * payload)
        out = torch.empty(n_rec, dtype=torch.uint32, device=dev)

        def crc_step():
            st = L.karma_crc32c_batch_fixed(arena.data_ptr(), rec, n_rec, None, 0, cur['out'].data_ptr(),
                                            cur.get('sh', sh))
            if st:
                _lib.check("batch_fixed", st)

        algo_bytes = n_rec * (rec + 4)
        if config5:
            workload_desc = f"{n_rec * world} x {rec} B records over {world} GPUs ({n_rec} per GPU), batched " \
                            f"CRC32C + RCCL gather of the CRCs to rank 0 (BASELINE configs[4])"
        else:
            workload_desc = f"{n_rec} x {rec} B records per GPU, batched CRC32C (BASELINE configs[1] shape)"
    elif wl == "ragged":
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        import synth
        # configs[2]: log-uniform 64 B .. 64 KiB payloads packed like a segment image (8-B headers), ~4 GiB
        target = 4 << 30
        count = int(target / (((65536 - 64) / np.log(1024)) + 8))
        lens = synth.loguniform_lengths(7, count, 64, 65536)
        offs, arena_bytes = synth.ragged_layout(lens, header=8)
        arena = torch.empty(arena_bytes + 16, dtype=torch.uint8, device=dev)
        K.fill_splitmix64(arena, args.seed + rank)
        d_off = torch.from_numpy(offs.astype(np.int64)).to(dev)
        d_len = torch.from_numpy(lens.astype(np.int32)).to(dev)
        out = torch.empty(count, dtype=torch.uint32, device=dev)
        total = int(lens.sum())
        n_rec = count
        payload = total

        def crc_step():
            st = L.karma_crc32c_batch_ragged(arena.data_ptr(), d_off.data_ptr(), d_len.data_ptr(), count, total,
                                             None, 0, cur['out'].data_ptr(), sh)
            if st:
                _lib.check("batch_ragged", st)

        algo_bytes = total + count * (4 + 8 + 4)
        workload_desc = f"{count} ragged records, log-uniform 64 B-64 KiB ({total / GIB:.2f} GiB payload), " \
                        f"segment-image layout (BASELINE configs[2])"
    elif wl == "stream":
        seg = 64 << 20
        nseg = 64
        n_rec, rec = nseg, seg
        payload = nseg * seg
        arena = torch.empty(payload, dtype=torch.uint8, device=dev)
        K.fill_splitmix64(arena, args.seed, first_byte=rank * payload)
        out = torch.empty(nseg, dtype=torch.uint32, device=dev)

        def crc_step():
            st = L.karma_crc32c_batch_fixed(arena.data_ptr(), seg, nseg, None, 0, cur['out'].data_ptr(), sh)
            if st:
                _lib.check("batch_fixed(stream)", st)

        algo_bytes = payload + nseg * 4
        workload_desc = f"{nseg} distinct 64 MiB segment scans per step (chunked CRC + polynomial combine, " \
                        f"BASELINE configs[3])"
    elif wl == "segment":
        # configs[3] as latency: one 64 MiB segment -> one Value per step (karma_crc32c_stream),
        # rotating over 64 distinct segments so every step reads HBM, not the 256 MB MALL
        seg, nseg = 64 << 20, 64
        arena = torch.empty(nseg * seg, dtype=torch.uint8, device=dev)
        K.fill_splitmix64(arena, args.seed, first_byte=rank * nseg * seg)
        n_rec, rec = 1, seg
        payload = seg
        out = torch.empty(nseg, dtype=torch.uint32, device=dev)
        seg_i = {"i": 0}

        def crc_step():
            i = seg_i["i"] % nseg
            seg_i["i"] += 1
            st = L.karma_crc32c_stream(0, arena.data_ptr() + i * seg, seg, cur['out'].data_ptr() + 4 * i, sh)
            if st:
                _lib.check("stream", st)

        algo_bytes = seg + 4
        workload_desc = "one 64 MiB segment scan per step (karma_crc32c_stream: chunked CRC + polynomial combine), " \
                        "64 distinct segments in rotation (BASELINE configs[3], latency)"
    else:  # host: PCIe-inclusive end-to-end from pageable host memory
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        import synth
        n_rec = min(n_rec, 1 << 18)
        payload = n_rec * rec
        host = synth.splitmix_np(args.seed, rank * payload, payload).copy()
        hout = np.empty(n_rec, dtype=np.uint32)
        out = None
        arena = None

        def crc_step():
            st = L.karma_crc32c_batch_fixed_host(host.ctypes.data, rec, n_rec, 0, hout.ctypes.data, local)
            if st:
                _lib.check("batch_fixed_host", st)

        algo_bytes = payload + n_rec * 4
        workload_desc = f"{n_rec} x {rec} B records in pageable host memory -> H2D -> kernel -> D2H (synchronous)"

    gather_buf = torch.empty(n_rec * world, dtype=torch.uint32, device=dev) if (comm is not None and rank == 0) else None
    # N > 1: double-buffered outputs, the gather of step i overlapping step i + 1 (GatherPipeline)
    outs = [out, torch.empty_like(out)] if (comm is not None and out is not None) else [out]
    kernel_step = crc_step

    def compute(o):
        cur["out"] = o
        kernel_step()

    # the gather of each timed step bracketed by events on the gather stream (its own time per
    # rank, separate from the batch kernel's: the N > 1 line reports both per rank)
    gtime = {"i": None}
    gev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)] \
        if comm is not None else []

    def gather(o, gs):
        i = gtime["i"]
        if i is not None:
            gev[i][0].record(gs)
        st = L.karma_crc32c_gather_u32(comm, o.data_ptr(), n_rec,
                                       gather_buf.data_ptr() if gather_buf is not None else None, 0, gs.cuda_stream)
        if st:
            _lib.check("gather_u32", st)
        if i is not None:
            gev[i][1].record(gs)

    pipe = GatherPipeline(outs, compute, gather if (comm is not None and out is not None) else None,
                          TorchSync(torch, stream))
    crc_step, gather_step = pipe.crc_step, pipe.gather_step
    if args.streams == 2 and wl == "fixed" and comm is None:
        # consecutive batches on two streams, each into its own output: batch i + 1's workgroups
        # take the CUs batch i's last ones leave, instead of waiting for the whole of batch i
        s2 = torch.cuda.Stream()
        alt = {"i": 0, "outs": [out, torch.empty_like(out)], "sh": [sh, s2.cuda_stream]}

        def crc_step():
            k = alt["i"] % 2
            alt["i"] += 1
            cur["sh"] = alt["sh"][k]
            compute(alt["outs"][k])

    # ---- pre-warm: the batch alone (no collective: ranks stop at different counts) for a fixed
    # time, so the clocks settle before --warmup (tools/ramp_probe.py) -----------
    prewarm_ms = 0.0
    if args.prewarm_ms > 0:
        t0 = time.perf_counter()
        while (time.perf_counter() - t0) * 1e3 < args.prewarm_ms:
            for _ in range(4):
                compute(outs[0])
            torch.cuda.synchronize()
        prewarm_ms = (time.perf_counter() - t0) * 1e3

    # ---- warmup -------------------------------------------------------------------------
    for _ in range(args.warmup):
        crc_step()
        gather_step()
    torch.cuda.synchronize()

    # ---- timed region: K steps between barrier + synchronize --------------------------------
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    # the dominant kernel alone (k_units_*), bracketed inside the library on the launch stream
    uev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    timed_units = wl != "host"
    # segment: one ~17 us kernel per step, so the per-step instrumentation (two events and the
    # library's kernel-event arming, ~4 ctypes/HIP calls from Python) would make the loop host-bound;
    # the timed loop enqueues the calls alone and the kernel / call events come from an
    # instrumented pass of the same steps right after it
    instrument_after = wl == "segment" and args.call_events != "on"
    if timed_units:
        for a, b in uev:  # materialise the hipEvents so their raw handles exist
            a.record(stream)
            b.record(stream)
        torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    # a fixed batch of one-unit records is one kernel: its call events would only add two
    # records to the stream per step, so the call time is the kernel time there
    call_events = {"on": True, "off": False}.get(args.call_events, not (wl == "fixed" and n_rec >= 4 * 32768))

    def steps(instrument):
        for i in range(args.steps):
            if instrument and call_events:
                ev[i][0].record(stream)
            if instrument and timed_units:
                L.karma_crc32c_time_next_units(uev[i][0].cuda_event, uev[i][1].cuda_event)
            crc_step()
            if instrument and call_events:
                ev[i][1].record(stream)
            gtime["i"] = i
            gather_step()
        gtime["i"] = None
    steps(not instrument_after)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t1 = time.perf_counter()
    elapsed = t1 - t0
    if instrument_after:  # (outside the timed region)
        steps(True)
        torch.cuda.synchronize()
    kern_ms = [a.elapsed_time(b) for a, b in uev] if timed_units else None
    call_ms = [a.elapsed_time(b) for a, b in ev] if call_events else kern_ms
    kern_ms = kern_ms if kern_ms is not None else call_ms
    kern_avg = float(np.mean(kern_ms))
    call_avg = float(np.mean(call_ms))
    gather_avg = float(np.mean([a.elapsed_time(b) for a, b in gev])) if gev else None
    per_rank = None
    if world > 1:
        t = torch.tensor([elapsed, kern_avg, call_avg, gather_avg if gather_avg is not None else 0.0],
                         dtype=torch.float64, device=dev)
        rows = [torch.empty_like(t) for _ in range(world)]
        dist.all_gather(rows, t)
        rows = torch.stack(rows).cpu().numpy()
        elapsed, kern_max, call_max = float(rows[:, 0].max()), float(rows[:, 1].max()), float(rows[:, 2].max())
        per_rank = {"elapsed_s": [round(float(x), 6) for x in rows[:, 0]],
                    "kernel_ms_avg": [round(float(x), 4) for x in rows[:, 1]],
                    "call_ms_avg": [round(float(x), 4) for x in rows[:, 2]],
                    "gather_ms_avg": [round(float(x), 4) for x in rows[:, 3]],
                    "gather": "karma_crc32c_gather_u32 on the gather stream, events around each timed step's call; "
                              "it overlaps the next step's batch (GatherPipeline)"}
    else:
        kern_max, call_max = kern_avg, call_avg

    # ---- single-segment latency: isolated calls, each waited for ------------------------------
    extra = {}
    if wl == "segment" and rank == 0:
        # the library call alone between the events: its pointers computed beforehand (the
        # harness's own Python -- the step pipeline, torch's data_ptr() -- is not the call's latency)
        stream_fn, a_base, o_base = L.karma_crc32c_stream, arena.data_ptr(), cur["out"].data_ptr()
        lat = []
        for _ in range(20):
            i = seg_i["i"] % nseg
            seg_i["i"] += 1
            pa, po = a_base + i * seg, o_base + 4 * i
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(stream)
            st = stream_fn(0, pa, seg, po, sh)
            b.record(stream)
            torch.cuda.synchronize()
            if st:
                _lib.check("stream", st)
            lat.append(a.elapsed_time(b))
        extra["single_segment_latency_us"] = round(float(np.median(lat)) * 1e3, 2)
        extra["single_segment_latency_gibs"] = round(payload / (float(np.median(lat)) * 1e-3) / GIB, 1)

    # ---- self-check: a sample of records against the host crc32c::Extend (product path) ----
    check = {}
    if wl == "segment" and rank == 0:
        got = cur["out"].cpu().numpy()
        bad = sum(int(K.Value(arena[i * rec:(i + 1) * rec].cpu().numpy()) != int(got[i])) for i in range(4))
        check = {"sampled_records": 4, "mismatches": bad}
    rank_checks = None
    if out is not None and wl in ("fixed", "stream"):
        # every rank checks a sample of its own shard; rank 0 also checks those records in the
        # CRCs it gathered (N > 1), so the line proves every shard, not only rank 0's
        mine = shard_self_check(arena, cur["out"], rec, n_rec, K.Value, seed=1 + rank,
                                rand=64 if wl == "fixed" else 0, first=64 if wl == "fixed" else 16)
        if world > 1:
            rank_checks = [None] * world
            dist.all_gather_object(rank_checks, mine)
            if rank == 0:
                g = gather_buf.cpu().numpy() if gather_buf is not None else None
                per, check = aggregate_self_checks(rank_checks, g, n_rec)
                per_rank["self_check"] = per
        else:
            check = {"sampled_records": len(mine["idx"]), "mismatches": mine["mismatches"]}

    if rank == 0:
        total_bytes = payload * world * args.steps
        value = total_bytes / elapsed / GIB
        achieved = algo_bytes / (kern_avg * 1e-3) / 1e9
        traffic = pmc_traffic(args.pmc, wl, payload) if wl == "fixed" else None
        traffic_source = os.path.relpath(args.pmc, ROOT) if traffic is not None else None
        res = {
            "metric": METRIC,
            "value": round(value, 2),
            "unit": "GiB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic: little-endian splitmix64 byte stream generated on the device before timing",
            "config": {"workload": workload_desc, "records_per_gpu": int(n_rec), "rec_bytes": int(rec),
                       "parallelism": f"record-sharded x{world}" + (" + RCCL gather to rank 0" if world > 1 else ""),
                       "kernel": units_kernel_name(wl) if out is not None else
                                 "host->device pipeline"},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                         "traffic_source": traffic_source,
                         "traffic_note": "HBM bytes per launch from a separate rocprofv3 --pmc pass of the same "
                                         "workload (FETCH_SIZE x2 + WRITE_SIZE, MI355X_MICROARCH.md gfx950 "
                                         "correction), read from traffic_source: not measured in this run"
                                         if traffic is not None else None,
                         "achieved_source": "algorithmic bytes / kernel_ms_avg (HIP events around the "
                                            "k_units_* launch inside the library, on its stream, this run"
                                            + (", in an instrumented pass of the same steps right after the "
                                               "timed loop, which enqueues the calls alone)" if instrument_after
                                               else ")"),
                         "algorithmic_bytes_per_launch": int(algo_bytes),
                         "kernel_ms_avg": round(kern_avg, 4), "kernel_ms_max_over_ranks": round(kern_max, 4),
                         "call_ms_avg": round(call_avg, 4),
                         "call_frac": round(algo_bytes / (call_avg * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                         **({"timed_loop_frac": round(algo_bytes / (elapsed / args.steps) / 1e9 / HBM_PEAK_GBS, 4),
                             "timed_loop_note": "the timed loop's own rate (calls back to back, no events): the "
                                                "instrumented pass's events leave the GPU idle between calls, so "
                                                "its kernels start cold"} if instrument_after else {})},
            "compute_only_gibs": round(payload * world / (call_max * 1e-3) / GIB, 2),
            "prewarm_ms": round(prewarm_ms, 1),
            "host_binding": numa,
            "rccl_nranks": rccl_nranks,
        }
        if per_rank is not None:
            res["per_rank"] = per_rank
        if args.streams == 2 and wl == "fixed" and comm is None:
            res["config"]["streams"] = 2
            res["roofline"]["streams_note"] = ("two streams: consecutive launches overlap, so kernel_ms_avg spans "
                                               "both and frac understates the kernel; read it from a --streams 1 line")
        if config5:  # the N = 8 default is configs[4]'s shard, not configs[1]'s 1M records per GPU
            res["config"]["records_per_gpu_n1_equivalent"] = 1 << 20
            anchor = config5_anchor()
            if anchor:
                res["config"]["same_shard_one_gpu_anchor"] = anchor
        res.update(extra)
        if check:
            res["self_check"] = check
        if world == 1 and not args.no_cpu_baseline:
            thr = args.cpu_threads or baseline_threads(args.orig_cpus)
            sample = None
            if wl in ("fixed", "stream", "ragged") and arena is not None:  # the first 1 GiB of the timed input
                sample = arena[: min(arena.numel(), (1 << 30) + 16)].cpu().numpy()
            res["cpu_baseline"] = cpu_baseline(wl, rec, thr, sample, args.orig_cpus, args.node_cpus)
        print(json.dumps(res), flush=True)

    if comm is not None:
        L.karma_crc32c_comm_destroy(comm)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
