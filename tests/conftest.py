"""pytest configuration: the `gpu` marker and shared fixtures.

    python -m pytest tests -m "not gpu"   # CPU: oracle vs golden, host path, ABI, sharding (gloo)
    python -m pytest tests -m gpu         # MI355X: parity of the HIP kernels with the oracle
"""
import json
import os
import sys

import pytest

# Fresh output tensors of the batch wrappers are filled with a poison value before each call, so a
# kernel that skips records cannot pass on stale CRCs left in reused memory.
os.environ.setdefault("KARMA_POISON_OUT", "1")

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
for p in (ROOT, HERE):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_addoption(parser):
    parser.addoption("--karma-lib", default="shipped", choices=["shipped", "bounds", "abbounds"],
                     help="bounds: run on the bounds-checked debug build (karma_amd/csrc/bounds.h); every GPU "
                          "test then also fails on any out-of-bounds access its kernels attempted; abbounds: "
                          "the same, and the variant tests on the tools build with the bounds checks")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (run with -m gpu on the GPU box)")
    if config.getoption("--karma-lib") in ("bounds", "abbounds"):
        import torch  # noqa: F401  (torch's HIP runtime first, as in every other run: the library binds to it)
        from karma_amd import _lib
        _lib.select(_lib.BOUNDS_LIB_PATH)
        if config.getoption("--karma-lib") == "abbounds":
            _lib.AB_LIB_PATH = _lib.ABBOUNDS_LIB_PATH


@pytest.fixture(autouse=True)
def _bounds_report(request):
    """Under --karma-lib bounds: after each GPU test, no kernel of the test may have attempted an
    access outside its buffers."""
    yield
    mode = request.config.getoption("--karma-lib")
    if mode not in ("bounds", "abbounds") or request.node.get_closest_marker("gpu") is None:
        return
    import ctypes
    import numpy as np
    from karma_amd import _lib
    paths = [_lib.BOUNDS_LIB_PATH] + ([_lib.ABBOUNDS_LIB_PATH] if mode == "abbounds" else [])
    for path in paths:
        if path != _lib.BOUNDS_LIB_PATH and not _lib.is_loaded(path):
            continue
        rep = np.zeros(4, np.uint64)
        L = _lib.load(path)
        assert L.karma_debug_bounds_report(rep.ctypes.data_as(ctypes.c_void_p), 1) == 0
        n, site, index, cap = (int(x) for x in rep)
        assert n == 0, (f"{os.path.basename(path)}: {n} out-of-bounds accesses; first: "
                        f"{_lib.KB_SITES.get(site, site)} (index {index}, cap {cap})")


@pytest.fixture(scope="session")
def vectors():
    with open(os.path.join(HERE, "golden", "crc32c_vectors.json")) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def records():
    with open(os.path.join(HERE, "golden", "crc32c_records.json")) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def karma_lib():
    """The engine library, built on demand (CPU build works without a GPU)."""
    from karma_amd import _lib
    if not os.path.exists(_lib.LIB_PATH):
        import subprocess
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "karma_amd", "csrc")], check=True)
    return _lib.lib()
