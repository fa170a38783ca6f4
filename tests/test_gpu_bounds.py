"""The bounds-checked debug build (karma_amd/csrc/bounds.h) reports what it must.

The GPU suite runs twice on the box: on the shipped library, and with `--karma-lib bounds` on the
build whose kernels check every record-byte load against the arena's allocation and every WAL
replay access (image bytes, candidate lists, sub-range reports, spans, gathered lists) against
its buffer; tests/conftest.py fails any test after which a violation was reported.  This module
is the positive control: a record that runs past its allocation must be reported (and, in that
build, redirected instead of faulting).  It is skipped on the shipped library, where the same
call would read unmapped memory.
"""
import ctypes

import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

from karma_amd import _lib  # noqa: E402


def test_out_of_bounds_record_is_reported(request):
    if request.config.getoption("--karma-lib") != "bounds":
        pytest.skip("the positive control runs on the bounds build only (--karma-lib bounds)")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    L = _lib.lib()
    rep = np.zeros(4, np.uint64)
    assert L.karma_debug_bounds_report(rep.ctypes.data_as(ctypes.c_void_p), 1) == 0  # start clean
    buf = torch.zeros(1 << 16, dtype=torch.uint8, device="cuda")
    off = torch.tensor([0, 100], dtype=torch.int64, device="cuda")
    n = torch.tensor([64, 1 << 30], dtype=torch.int32, device="cuda")  # record 1 runs 1 GiB past the buffer
    out = torch.empty(2, dtype=torch.int32, device="cuda")
    st = L.karma_crc32c_batch_ragged(buf.data_ptr(), off.data_ptr(), n.data_ptr(), 2, (1 << 30) + 64, None, 0,
                                     out.data_ptr(), torch.cuda.current_stream().cuda_stream)
    assert st == 0
    assert L.karma_debug_bounds_report(rep.ctypes.data_as(ctypes.c_void_p), 1) == 0
    count, site = int(rep[0]), int(rep[1])
    assert count > 0 and site == 10, (count, _lib.KB_SITES.get(site, site))
