"""bench.py's N > 1 step (GatherPipeline: double-buffered outputs, the gather of step i on its own
stream overlapping step i + 1, event order) driven on CPU by world-2 gloo ranks.

On the GPU box the compute is karma_crc32c_batch_fixed on the rank's record shard and the gather
is karma_crc32c_gather_u32 over RCCL; here the compute is the oracle (test stand-in for the
device batch, with a per-step init so every step's CRCs differ) and the gather is
torch.distributed.gather over gloo.  A logging stand-in for the streams and events checks the
dependency order the pipeline enqueues: a buffer is reused only after the gather that last read
it, and every gather is ordered after the compute that wrote its buffer.  Rank 0 checks that
every step's gathered CRCs are the whole batch's, in record order (per-record independence,
karma-store/segment_file.cc:22).
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import oracle_lib
from karma_amd.shard import shard_range

N_REC, REC, STEPS = 3000, 256, 7


class LogSync:
    """Streams are names, events are objects; every record/wait is logged.  Work runs at once
    (host), so the log is the enqueue order the device streams would see."""

    compute_stream, gather_stream = "compute", "gather"

    def __init__(self):
        self.log = []
        self.n = 0

    def event(self):
        self.n += 1
        return {"id": self.n, "recorded_at": None}

    def record(self, ev, stream):
        ev["recorded_at"] = len(self.log)
        self.log.append(("record", stream, ev["id"]))

    def wait(self, stream, ev):
        assert ev["recorded_at"] is not None, "waits on an event never recorded"
        self.log.append(("wait", stream, ev["id"]))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import bench  # the repository's bench.py (its main() only runs as a script)
    try:
        lo, hi = shard_range(N_REC, world, rank)
        n_local = hi - lo
        outs = [torch.zeros(n_local, dtype=torch.int64), torch.zeros(n_local, dtype=torch.int64)]
        sync = LogSync()
        step = {"i": 0}
        results = []

        def compute(o):  # the device batch's stand-in: this rank's records, init = step number
            sync.log.append(("compute", "compute", id(o)))
            o.copy_(torch.from_numpy(oracle_lib.splitmix_fixed_crcs(42, REC, lo, n_local, init=step["i"])
                                     .astype(np.int64)))
            step["i"] += 1

        def gather(o, stream):
            sync.log.append(("gather", stream, id(o)))
            full = [torch.zeros(n_local, dtype=torch.int64) for _ in range(world)] if rank == 0 else None
            dist.gather(o, full, dst=0)
            if rank == 0:
                results.append(torch.cat(full).numpy().copy())

        pipe = bench.GatherPipeline(outs, compute, gather, sync)
        for _ in range(STEPS):
            pipe.crc_step()
            pipe.gather_step()
        # dependency order: before step i >= 2 computes into slot i % 2, the compute stream waits
        # on the event the gather of step i - 2 recorded; each gather waits on its compute's event
        computes = [k for k, e in enumerate(sync.log) if e[0] == "compute"]
        gathers = [k for k, e in enumerate(sync.log) if e[0] == "gather"]
        ok_order = len(computes) == STEPS and len(gathers) == STEPS
        for i in range(STEPS):
            c, g = computes[i], gathers[i]
            ok_order &= sync.log[c][2] == id(outs[i % 2])  # step i writes buffer i % 2
            ok_order &= sync.log[g][2] == id(outs[i % 2])  # and its gather reads that buffer
            ok_order &= sync.log[g - 1] == ("wait", "gather", pipe.computed[i % 2]["id"])
            ok_order &= sync.log[g - 2] == ("record", "compute", pipe.computed[i % 2]["id"])
            ok_order &= sync.log[g + 1] == ("record", "gather", pipe.gathered[i % 2]["id"])
            if i >= 2:
                ok_order &= sync.log[c - 1] == ("wait", "compute", pipe.gathered[i % 2]["id"])
                ok_order &= gathers[i - 2] < c - 1
        ok_data = None
        if rank == 0:
            ok_data = len(results) == STEPS and all(
                np.array_equal(results[i], oracle_lib.splitmix_fixed_crcs(42, REC, 0, N_REC, init=i).astype(np.int64))
                for i in range(STEPS))
        q.put((rank, bool(ok_order), ok_data))
    finally:
        dist.destroy_process_group()


def test_bench_gather_pipeline_world2():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(180)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    got = sorted(q.get(timeout=10) for _ in range(world))
    assert got == [(0, True, True), (1, True, None)], got


def test_bench_defaults_to_config5_shard_on_8_gpus():
    """--gpus 8 with no --records-per-gpu runs BASELINE configs[4]'s shard: 256M / 8 records."""
    import bench
    assert bench.records_per_gpu(0, 8, "fixed") == (33554432, True)
    assert bench.records_per_gpu(0, 1, "fixed") == (1 << 20, False)
    assert bench.records_per_gpu(0, 4, "fixed") == (1 << 20, False)
    assert bench.records_per_gpu(12345, 8, "fixed") == (12345, False)


def _check_worker(rank, world, port, q):
    """Each rank: its shard's bytes and CRCs (oracle CRCs standing in for the device batch; rank 1
    corrupts one sampled CRC), shard_self_check with the oracle standing in for the host Value,
    all_gather_object, and rank 0 aggregates against a gathered copy (as RCCL's gather leaves it)
    -- once intact, once with a shard misplaced."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import bench
    try:
        import synth
        n_local = 700
        lo = rank * n_local
        arena = torch.from_numpy(synth.splitmix_np(42, lo * REC, n_local * REC).copy())
        crcs = oracle_lib.splitmix_fixed_crcs(42, REC, lo, n_local).astype(np.int64)
        out = torch.from_numpy(crcs.copy())
        if rank == 1:
            out[3] ^= 1  # a wrong device CRC in a sampled record (the first 64 are always sampled)
        mine = bench.shard_self_check(arena, out, REC, n_local, lambda b: oracle_lib.extend(0, b.tobytes()),
                                      seed=1 + rank)
        checks = [None] * world
        dist.all_gather_object(checks, mine)
        full = [torch.zeros(n_local, dtype=torch.int64) for _ in range(world)] if rank == 0 else None
        dist.gather(out, full, dst=0)
        res = None
        if rank == 0:
            gathered = torch.cat(full).numpy()
            per, tot = bench.aggregate_self_checks(checks, gathered, n_local)
            swapped = np.concatenate([gathered[n_local:], gathered[:n_local]])  # shards in the wrong order
            _, tot_bad = bench.aggregate_self_checks(checks, swapped, n_local)
            res = (per, tot["mismatches"], tot["gather_mismatches"], tot_bad["gather_mismatches"] > 100,
                   tot["sampled_records"])
        q.put((rank, res))
    finally:
        dist.destroy_process_group()


def test_bench_self_check_every_shard_world2():
    """bench.py's N > 1 self-check: every rank samples its own shard after timing, rank 0 reports
    each rank's result (per_rank.self_check) and checks the sampled records in the CRCs it
    gathered, so one wrong shard or a misplaced gather shows in the line."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_check_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(180)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    got = dict(q.get(timeout=10) for _ in range(world))
    per, mism, gmism, swapped_seen, sampled = got[0]
    assert [p["mismatches"] for p in per] == [0, 1]
    assert all(p["sampled_records"] >= 64 for p in per) and sampled == sum(p["sampled_records"] for p in per)
    assert mism == 1 and gmism == 0 and swapped_seen
    assert got[1] is None
