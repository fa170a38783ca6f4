"""Multi-GPU path on CPU: record sharding + the CRC gather, world_size 2 over gloo.

On the GPU box each rank runs the HIP kernel on its shard and gathers over RCCL (bench.py,
karma_amd.shard.RcclComm); here the per-shard CRCs come from the oracle (test stand-in for
the device compute) so the sharding and ordering logic is checked without a GPU.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import oracle_lib
import synth
from karma_amd.shard import gather_to_root, ragged_partition, shard_range


def test_shard_range_partitions():
    for n in [0, 1, 7, 1000, 1 << 20]:
        for world in [1, 2, 3, 8]:
            parts = [shard_range(n, world, r) for r in range(world)]
            assert parts[0][0] == 0 and parts[-1][1] == n
            assert all(parts[i][1] == parts[i + 1][0] for i in range(world - 1))
            sizes = [b - a for a, b in parts]
            assert max(sizes) - min(sizes) <= 1


def test_ragged_partition_balances_bytes():
    lens = synth.loguniform_lengths(7, 20000, 64, 65536)
    for world in [1, 2, 4, 8]:
        parts = ragged_partition(lens, world)
        assert parts[0][0] == 0 and parts[-1][1] == lens.size
        assert all(parts[i][1] == parts[i + 1][0] for i in range(world - 1))
        total = int(lens.sum())
        for a, b in parts:
            assert abs(int(lens[a:b].sum()) - total / world) <= 65536
    assert ragged_partition([], 3) == [(0, 0)] * 3


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        # fixed-size: 1000 x 300 B records of the splitmix stream
        n, rec = 1000, 300
        lo, hi = shard_range(n, world, rank)
        local = oracle_lib.splitmix_fixed_crcs(42, rec, lo, hi - lo).astype(np.int64)
        counts = [shard_range(n, world, r)[1] - shard_range(n, world, r)[0] for r in range(world)]
        full = gather_to_root(torch.from_numpy(local), counts, root=0)
        ok_fixed = None
        if rank == 0:
            want = oracle_lib.splitmix_fixed_crcs(42, rec, 0, n).astype(np.int64)
            ok_fixed = bool(np.array_equal(full.numpy(), want))
        # ragged: byte-balanced contiguous ranges of a segment-image layout
        lens = synth.loguniform_lengths(5, 3000, 1, 9000)
        offs, arena = synth.ragged_layout(lens, header=8)
        data = synth.splitmix_np(3, 0, arena + 16).copy()
        parts = ragged_partition(lens, world)
        a, b = parts[rank]
        local = oracle_lib.ragged_crcs(data, offs[a:b], lens[a:b]).astype(np.int64)
        full = gather_to_root(torch.from_numpy(local), [y - x for x, y in parts], root=0)
        ok_ragged = None
        if rank == 0:
            want = oracle_lib.ragged_crcs(data, offs, lens).astype(np.int64)
            ok_ragged = bool(np.array_equal(full.numpy(), want))
        if rank == 0:
            q.put((ok_fixed, ok_ragged))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2])
def test_sharded_gather_matches_whole_batch(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    assert q.get(timeout=10) == (True, True)
