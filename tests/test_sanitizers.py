"""Host code under AddressSanitizer + UBSan, and the CPU emulation of the device
WAL replay with bounds checks on every access.

`make -C karma_amd/csrc san` builds, with -fsanitize=address,undefined:
  build/san/host_logic_test  the library's host objects (capi, wal, wal_append, kfp, host_batch,
                             host_stage, host_crc32c, tables, rccl_comm) + tests/cpp/host_logic_test.cc
  build/san/wal_walk_emu     tests/cpp/wal_walk_emu.cc: the walk, resolve, gather and CRC-batch
                             addressing of wal_device.hip / wal.cc restated on the CPU
  build/san/dropin_test      tests/cpp/dropin_test.cc against host_crc32c.cc
"""
import os
import subprocess
import tempfile

import numpy as np
import pytest

import wal_images
import wal_model

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SAN = os.path.join(ROOT, "build", "san")
ENV = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:abort_on_error=1", UBSAN_OPTIONS="print_stacktrace=1")
CU = 256  # MI355X compute units: the planner's sub-range split for few segments


@pytest.fixture(scope="module")
def san_build():
    subprocess.run(["make", "-s", "-j8", "-C", os.path.join(ROOT, "karma_amd", "csrc"), "san"], check=True,
                   capture_output=True)
    return SAN


def test_host_logic_under_sanitizers(san_build):
    r = subprocess.run([os.path.join(san_build, "host_logic_test")], env=ENV, capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert "host_logic_test: ok" in r.stdout


def test_dropin_under_sanitizers(san_build):
    r = subprocess.run([os.path.join(san_build, "dropin_test")], env=ENV, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]


def _emulate(san_build, wal, seg, start, sub):
    with tempfile.NamedTemporaryFile(suffix=".wal", delete=False) as f:
        f.write(wal.tobytes())
        path = f.name
    try:
        r = subprocess.run([os.path.join(san_build, "wal_walk_emu"), path, str(seg), str(start), str(sub), str(CU)],
                           env=ENV, capture_output=True, text=True, timeout=300)
    finally:
        os.unlink(path)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = r.stdout.split()
    n, stop, status = int(lines[0]), int(lines[1]), int(lines[2])
    return [int(x) for x in lines[3: 3 + n]], stop, status


PLANS = {"split": 0, "split4k": 4096, "whole": 1 << 30}


def _check(san_build, wal, seg, start=0):
    want = wal_model.replay(wal.tobytes(), seg, start)
    for name, sub in PLANS.items():
        got = _emulate(san_build, wal, seg, start, sub)
        assert got == (list(want[0]), want[1], want[2]), (name, seg, start)


def test_emulated_walk_wal_looking_payloads(san_build):
    """Round 1's faulting test inputs: every walker and resolver access in bounds, and the
    result is scan_record's, from the start and from checkpoints."""
    wal, seg, rec = wal_images.wal_looking_payloads()
    for start in (0, int(rec[5]), int(rec[101]), int(rec[222])):
        _check(san_build, wal, seg, start)


@pytest.mark.parametrize("seg", [1 << 20, (256 << 10) + 4])
def test_emulated_walk_large_records(san_build, seg):
    wal, seg, rec = wal_images.large_records(seg)
    for start in (0, int(rec[3]), int(rec[len(rec) // 2])):
        _check(san_build, wal, seg, start)


@pytest.mark.parametrize("seg", [(64 << 10) + 12, 4096 + 4])
def test_emulated_walk_misaligned_segments(san_build, seg):
    wal, seg, rec = wal_images.segment_sizes(seg)
    _check(san_build, wal, seg, 0)
    k = len(rec) * 3 // 4
    wal[int(rec[k]) + 8] ^= 0x40  # a flipped payload byte: replay stops there
    _check(san_build, wal, seg, int(rec[1]))


@pytest.mark.parametrize("seg", [4096 + 4, 1 << 20])
def test_emulated_walk_uniform_runs(san_build, seg):
    """Runs of one size: the speculative header rounds; then a bad type inside a run."""
    wal, seg, rec, lens = wal_images.uniform_runs(seg)
    _check(san_build, wal, seg, 0)
    runs = np.nonzero((lens[1:-1] == lens[:-2]) & (lens[1:-1] == lens[2:]))[0] + 1
    k = int(runs[len(runs) // 2])
    wal[int(rec[k]) + 4] = 3
    _check(san_build, wal, seg, int(rec[2]))


def test_emulated_walk_randomized(san_build):
    inner = wal_images.inner_image()
    for case in range(8):
        wal, seg, start = wal_images.randomized(case, inner)
        _check(san_build, wal, seg, start)


def test_emulated_walk_zero_image_and_end(san_build):
    wal = np.zeros(4 * (64 << 10), np.uint8)
    _check(san_build, wal, 64 << 10, 0)
    assert _emulate(san_build, wal, 64 << 10, wal.nbytes, 0) == ([], wal.nbytes, wal_model.END)


@pytest.mark.parametrize("seg", [65536, 16384 + 4])
def test_emulated_walk_accepted_size0_records(san_build, seg):
    """Accepted size-0 records (stored CRC Value("\\0\\0\\0\\0")) advance the chain by 12 bytes
    (wal.cc:66, sivir.cc:38), across tile / sub-range edges and into the next segment
    (tests/wal_images.py stale_empty): the emulated walk matches scan_record, every access in
    bounds, from the start and from checkpoints on such records."""
    for seed in range(3):
        wal, heads = wal_images.stale_empty(seg, 6, 100 + seed)
        want = wal_model.replay(wal.tobytes(), seg)
        zs = [h for h in want[0] if int.from_bytes(wal[h + 4: h + 8].tobytes(), "little") == 0]
        assert zs
        for start in (0, zs[len(zs) // 2], zs[-1]):
            _check(san_build, wal, seg, start)
