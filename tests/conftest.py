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


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (run with -m gpu on the GPU box)")


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
