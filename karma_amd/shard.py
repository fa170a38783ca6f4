"""Record sharding over GPUs (one process per GPU) and the gather of per-record CRCs.

Records are independent (one ``crc32c::Value`` per record, segment_file.cc:22 / wal.cc:60), so
a batch shards with no data-path collective: rank r owns a contiguous record range and the
only exchange is the gather of 4-byte CRCs to the root, in record order.

* ``shard_range``         contiguous [lo, hi) of equal record counts (fixed-size batches)
* ``ragged_partition``    contiguous record ranges of near-equal payload bytes (ragged batches)
* ``gather_to_root``      torch.distributed gather of unequal shards (gloo on CPU, or nccl)
* ``RcclComm``            the library's own RCCL communicator (``karma_crc32c_comm_*``),
                          bootstrapped through torch.distributed, for the device path
"""
from __future__ import annotations

import ctypes
from typing import List, Optional, Sequence, Tuple

import numpy as np

from . import _lib


def shard_range(n: int, world: int, rank: int) -> Tuple[int, int]:
    """Records [lo, hi) of rank ``rank``: floor(r*n/world) .. floor((r+1)*n/world)."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError("bad world/rank")
    return (rank * n) // world, ((rank + 1) * n) // world


def ragged_partition(lengths: Sequence[int], world: int) -> List[Tuple[int, int]]:
    """Split records into ``world`` contiguous ranges with near-equal payload bytes.

    Boundary k is the first record whose byte prefix reaches k/world of the total, so each
    range's bytes differ from total/world by at most one record.
    """
    lens = np.asarray(lengths, dtype=np.uint64)
    n = lens.size
    if world < 1:
        raise ValueError("world must be >= 1")
    if n == 0:
        return [(0, 0)] * world
    csum = np.cumsum(lens, dtype=np.uint64)
    total = int(csum[-1])
    bounds = [0]
    for k in range(1, world):
        target = (total * k) // world
        b = int(np.searchsorted(csum, np.uint64(target), side="left")) + 1 if total else (n * k) // world
        bounds.append(min(max(b, bounds[-1]), n))
    bounds.append(n)
    return [(bounds[i], bounds[i + 1]) for i in range(world)]


def gather_to_root(local, counts: Sequence[int], root: int = 0, group=None):
    """Gather each rank's 1-D ``local`` tensor (``counts[r]`` elements) to ``root`` in rank order.

    Shards may be unequal: every rank pads to max(counts) (torch.distributed.gather needs
    equal sizes), the root trims.  Returns the concatenation on root, None elsewhere.
    """
    import torch
    import torch.distributed as dist

    rank = dist.get_rank(group)
    world = dist.get_world_size(group)
    m = max(int(c) for c in counts) if len(counts) else 0
    buf = torch.zeros(m, dtype=local.dtype, device=local.device)
    buf[: local.numel()] = local
    parts = [torch.empty_like(buf) for _ in range(world)] if rank == root else None
    dist.gather(buf, parts, dst=root, group=group)
    if rank != root:
        return None
    return torch.cat([parts[r][: int(counts[r])] for r in range(world)])


class RcclComm:
    """The engine's RCCL communicator (one per process/GPU), bootstrapped via torch.distributed.

    Rank 0 creates the unique id (``karma_crc32c_get_unique_id``), torch.distributed
    broadcasts it, every rank calls ``karma_crc32c_comm_init``.  ``gather_u32`` is
    ``ncclGather`` of equal-size uint32 shards onto the root over xGMI.
    """

    def __init__(self, group=None):
        import torch.distributed as dist

        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        L = _lib.lib()
        uid = (ctypes.c_char * _lib.UNIQUE_ID_BYTES)()
        if self.rank == 0:
            _lib.check("karma_crc32c_get_unique_id", L.karma_crc32c_get_unique_id(uid, _lib.UNIQUE_ID_BYTES))
        obj = [bytes(uid) if self.rank == 0 else None]
        dist.broadcast_object_list(obj, src=0, group=group)
        uid = (ctypes.c_char * _lib.UNIQUE_ID_BYTES).from_buffer_copy(obj[0])
        self.handle = ctypes.c_void_p()
        _lib.check("karma_crc32c_comm_init",
                   L.karma_crc32c_comm_init(ctypes.byref(self.handle), self.world, uid, self.rank))

    def gather_u32(self, local, out=None, root: int = 0, stream=None):
        """ncclGather of this rank's uint32 CUDA tensor; returns the [world * n] tensor on root."""
        import torch

        n = local.numel()
        if self.rank == root and out is None:
            out = torch.empty(n * self.world, dtype=local.dtype, device=local.device)
        s = (stream or torch.cuda.current_stream()).cuda_stream
        st = _lib.lib().karma_crc32c_gather_u32(self.handle, local.data_ptr(), n,
                                                out.data_ptr() if out is not None else None, root, s)
        _lib.check("karma_crc32c_gather_u32", st)
        return out

    def close(self) -> None:
        if self.handle:
            _lib.check("karma_crc32c_comm_destroy", _lib.lib().karma_crc32c_comm_destroy(self.handle))
            self.handle = ctypes.c_void_p()

    def __del__(self):  # pragma: no cover - best effort
        try:
            self.close()
        except Exception:
            pass


def shard_bytes(total_records: int, rec_bytes: int, world: int, rank: int) -> Tuple[int, int, int]:
    """(first_record, n_records, first_byte) of rank's contiguous shard of a fixed-size batch."""
    lo, hi = shard_range(total_records, world, rank)
    return lo, hi - lo, lo * rec_bytes


__all__ = ["shard_range", "ragged_partition", "gather_to_root", "RcclComm", "shard_bytes"]
