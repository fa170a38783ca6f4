"""karma_amd -- MI355X (gfx950) CRC-32C engine for Karma's WAL checksum path.

Host surface mirroring ``karma-util/crc32c.h`` (Extend / Value / Mask / Unmask) and the
GPU batch API (fixed-size, ragged and single-stream) over the C ABI in
``include/karma_crc32c.h``.  See DESIGN.md.
"""
from .crc32c import (  # noqa: F401
    Combine,
    Extend,
    Mask,
    Unmask,
    Value,
    device_cu_count,
    extend_batch_ragged,
    extend_batch_ragged_host,
    extend_stream,
    fill_splitmix64,
    kMaskDelta,
    stream_probe,
    value_batch_fixed,
    value_batch_fixed_host,
)
from ._lib import KarmaError, KarmaUnavailable, LIB_PATH  # noqa: F401
from . import wal  # noqa: F401  (WAL append / replay and KFP frames: karma_amd.wal)
