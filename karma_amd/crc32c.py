"""Python mirror of Karma's ``karma-util/crc32c.h`` surface plus the MI355X batch API.

Reference names and meaning are kept (``/root/reference/karma-util/crc32c.h:11-39``):

* ``Extend(init_crc, data)`` -- CRC-32C of A || data given ``init_crc`` = CRC-32C of A
* ``Value(data)``            -- ``Extend(0, data)``
* ``Mask`` / ``Unmask`` / ``kMaskDelta``

Those run on the host through ``crc32c::Extend`` in libkarma_crc32c.so (single buffer,
synchronous, like the reference).  Batches of records run on the GPU:

* ``value_batch_fixed``   -- fixed-size records      (``karma_crc32c_batch_fixed``)
* ``extend_batch_ragged`` -- offsets + lengths       (``karma_crc32c_batch_ragged``)
* ``extend_stream``       -- one long buffer         (``karma_crc32c_stream``)

The device functions take and return ``torch`` CUDA tensors (PyTorch is only the
allocator / stream provider here) and enqueue on the current stream.  Without a GPU or
without the built library they raise; they never compute on the CPU.
"""
from __future__ import annotations

import ctypes
import os
from typing import Optional, Union

from . import _lib

kMaskDelta = 0xA282EAD8
_M32 = 0xFFFFFFFF

BytesLike = Union[bytes, bytearray, memoryview]


def _host_buffer(data) -> tuple[int, int, object]:
    """(address, length, keepalive) of a host byte buffer (bytes / bytearray / numpy / memoryview)."""
    if isinstance(data, (bytes, bytearray)):
        buf = (ctypes.c_char * len(data)).from_buffer_copy(data) if isinstance(data, bytes) else \
            (ctypes.c_char * len(data)).from_buffer(data)
        return ctypes.addressof(buf), len(data), buf
    try:
        import numpy as np
        if isinstance(data, np.ndarray):
            a = np.ascontiguousarray(data)
            return a.ctypes.data, a.nbytes, a
    except ImportError:  # pragma: no cover
        pass
    mv = memoryview(data).cast("B")
    b = bytes(mv)
    buf = (ctypes.c_char * len(b)).from_buffer_copy(b)
    return ctypes.addressof(buf), len(b), buf


def Extend(init_crc: int, data) -> int:
    """crc32c::Extend (reference crc32c.h:16, crc32c.cc:275-376), host path."""
    addr, n, keep = _host_buffer(data)
    r = _lib.lib().karma_crc32c_extend_host(init_crc & _M32, addr if n else None, n)
    del keep
    return int(r)


def Value(data) -> int:
    """crc32c::Value (reference crc32c.h:19)."""
    return Extend(0, data)


def Combine(crc_a: int, crc_b: int, len_b: int) -> int:
    """CRC-32C of A || B from Value(A), Value(B) and len(B) (host GF(2) shift)."""
    return int(_lib.lib().karma_crc32c_combine(crc_a & _M32, crc_b & _M32, len_b))


def Mask(crc: int) -> int:
    """crc32c::Mask (reference crc32c.h:28-31): rotate right by 15 bits, add kMaskDelta."""
    crc &= _M32
    return ((((crc >> 15) | (crc << 17)) & _M32) + kMaskDelta) & _M32


def Unmask(masked_crc: int) -> int:
    """crc32c::Unmask (reference crc32c.h:34-37)."""
    rot = (masked_crc - kMaskDelta) & _M32
    return ((rot >> 17) | (rot << 15)) & _M32


# ---------------------------------------------------------------------------------------------
# device batches
# ---------------------------------------------------------------------------------------------

def _torch():
    import torch
    return torch


def _stream_handle(stream) -> Optional[int]:
    torch = _torch()
    s = stream if stream is not None else torch.cuda.current_stream()
    return s.cuda_stream


def _require_cuda(t, name: str):
    if not t.is_cuda:
        raise ValueError(f"{name} must be a CUDA (HIP) tensor")
    if not t.is_contiguous():
        raise ValueError(f"{name} must be contiguous")


def _init_args(init, n_rec: int):
    """(device pointer or None, scalar) for an int / tensor init."""
    torch = _torch()
    if init is None:
        return None, 0, None
    if isinstance(init, int):
        return None, init & _M32, None
    _require_cuda(init, "init")
    if init.numel() != n_rec or init.element_size() != 4:
        raise ValueError("init tensor must hold one 32-bit value per record")
    return init.data_ptr(), 0, init


_POISON = os.environ.get("KARMA_POISON_OUT") is not None  # tests: no stale CRCs in fresh outputs


def _out_tensor(out, n: int, device):
    torch = _torch()
    if out is None:
        t = torch.empty(n, dtype=torch.uint32, device=device)
        if _POISON:  # a kernel that skipped a record must not inherit a right answer
            t.fill_(0xA5A5A5A5)
        return t
    _require_cuda(out, "out")
    if out.numel() < n or out.element_size() != 4:
        raise ValueError("out must hold n 32-bit values")
    return out


def value_batch_fixed(data, rec_bytes: Optional[int] = None, init=None, out=None, stream=None):
    """CRC-32C of every fixed-size record of ``data`` (uint8 CUDA tensor).

    ``data`` is [n_rec, rec_bytes] or flat with ``rec_bytes`` given.  ``init`` is None
    (Value), an int (same Extend init for all records) or a uint32/int32 tensor.
    Returns a uint32 tensor of n_rec CRCs (batched segment_file.cc:22).
    """
    _require_cuda(data, "data")
    if rec_bytes is None:
        if data.dim() != 2:
            raise ValueError("pass rec_bytes for a flat buffer")
        rec_bytes = data.shape[1]
    total = data.numel() * data.element_size()
    n_rec = total // rec_bytes if rec_bytes else 0
    if rec_bytes and n_rec * rec_bytes != total:
        raise ValueError("buffer is not a whole number of records")
    d_init, s_init, _keep = _init_args(init, n_rec)
    out = _out_tensor(out, n_rec, data.device)
    st = _lib.lib().karma_crc32c_batch_fixed(data.data_ptr(), rec_bytes, n_rec, d_init, s_init, out.data_ptr(),
                                             _stream_handle(stream))
    _lib.check("karma_crc32c_batch_fixed", st)
    return out[:n_rec]


def extend_batch_ragged(arena, offsets, lengths, init=None, out=None, total_len: Optional[int] = None, stream=None):
    """CRC-32C of ``arena[offsets[r] : offsets[r] + lengths[r]]`` for every record r.

    ``offsets``: int64/uint64 CUDA tensor, ``lengths``: int32/uint32 CUDA tensor.
    ``total_len`` (sum of lengths, or an upper bound) keeps the call fully asynchronous;
    when None it is computed on the device side by the library (one host sync).
    Batched wal.cc:60.
    """
    torch = _torch()
    for t, nm in ((arena, "arena"), (offsets, "offsets"), (lengths, "lengths")):
        _require_cuda(t, nm)
    if offsets.element_size() != 8 or lengths.element_size() != 4:
        raise ValueError("offsets must be 64-bit and lengths 32-bit")
    n_rec = offsets.numel()
    if lengths.numel() != n_rec:
        raise ValueError("offsets and lengths differ in length")
    d_init, s_init, _keep = _init_args(init, n_rec)
    out = _out_tensor(out, n_rec, arena.device)
    st = _lib.lib().karma_crc32c_batch_ragged(arena.data_ptr(), offsets.data_ptr(), lengths.data_ptr(), n_rec,
                                              int(total_len or 0), d_init, s_init, out.data_ptr(),
                                              _stream_handle(stream))
    _lib.check("karma_crc32c_batch_ragged", st)
    return out[:n_rec]


def extend_stream(init_crc: int, data, out=None, stream=None):
    """Extend(init_crc, data) over one long CUDA buffer, split over the whole GPU.

    Returns a 1-element uint32 CUDA tensor (call ``int(t.item())`` to read it).
    """
    _require_cuda(data, "data")
    n = data.numel() * data.element_size()
    out = _out_tensor(out, 1, data.device)
    st = _lib.lib().karma_crc32c_stream(init_crc & _M32, data.data_ptr(), n, out.data_ptr(), _stream_handle(stream))
    _lib.check("karma_crc32c_stream", st)
    return out[:1]


def value_batch_fixed_host(data, rec_bytes: int, init: int = 0, device: int = -1):
    """Host-memory fixed-size batch (numpy uint8 buffer): H2D, GPU, D2H, synchronous."""
    import numpy as np
    a = np.ascontiguousarray(data).view(np.uint8).reshape(-1)
    n_rec = a.nbytes // rec_bytes if rec_bytes else 0
    out = np.empty(n_rec, dtype=np.uint32)
    st = _lib.lib().karma_crc32c_batch_fixed_host(a.ctypes.data, rec_bytes, n_rec, init & _M32, out.ctypes.data,
                                                  device)
    _lib.check("karma_crc32c_batch_fixed_host", st)
    return out


def extend_batch_ragged_host(arena, offsets, lengths, init: int = 0, device: int = -1):
    """Host-memory ragged batch (numpy arrays), synchronous."""
    import numpy as np
    a = np.ascontiguousarray(arena).view(np.uint8).reshape(-1)
    off = np.ascontiguousarray(offsets, dtype=np.uint64)
    ln = np.ascontiguousarray(lengths, dtype=np.uint32)
    out = np.empty(off.size, dtype=np.uint32)
    st = _lib.lib().karma_crc32c_batch_ragged_host(a.ctypes.data, a.nbytes, off.ctypes.data, ln.ctypes.data,
                                                   off.size, init & _M32, out.ctypes.data, device)
    _lib.check("karma_crc32c_batch_ragged_host", st)
    return out


def fill_splitmix64(dst, seed: int, first_byte: int = 0, stream=None) -> None:
    """Fill a CUDA byte tensor with the splitmix64 stream (tests/synth.py defines the same stream)."""
    _require_cuda(dst, "dst")
    n = dst.numel() * dst.element_size()
    st = _lib.lib().karma_fill_splitmix64(dst.data_ptr(), n, seed & 0xFFFFFFFFFFFFFFFF, first_byte,
                                          _stream_handle(stream))
    _lib.check("karma_fill_splitmix64", st)


def stream_probe(src, out=None, stream=None):
    """Read-only HBM streaming probe over a CUDA tensor (xor of its 16-byte words)."""
    torch = _torch()
    _require_cuda(src, "src")
    if out is None:
        out = torch.zeros(1, dtype=torch.uint32, device=src.device)
    st = _lib.lib().karma_stream_probe(src.data_ptr(), src.numel() * src.element_size(), out.data_ptr(),
                                       _stream_handle(stream))
    _lib.check("karma_stream_probe", st)
    return out


def device_cu_count() -> int:
    r = _lib.lib().karma_device_cu_count()
    if r < 0:
        _lib.check("karma_device_cu_count", r)
    return int(r)
