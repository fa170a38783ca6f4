"""Host side of the boundary (no GPU needed): the library loads and exports what include/*.h
declares, crc32c::Extend / Value / Mask / Unmask match the reference golden vectors, the C++
drop-in compiles and links like Karma's callers, device entry points refuse to run without a
GPU (no CPU fallback), and the GF(2) combine identity the GPU combine kernels rely on holds."""
import ctypes
import os
import re
import subprocess

import numpy as np
import pytest

import karma_amd as K
from karma_amd import _lib
from golden_inputs import case_bytes, case_init

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared_symbols():
    names = set()
    for fn in os.listdir(os.path.join(ROOT, "include")):
        if fn.endswith(".h"):
            text = open(os.path.join(ROOT, "include", fn)).read()
            names |= set(re.findall(r"^\s*(?:const\s+)?[\w\s\*]+?\b(karma_\w+)\s*\(", text, flags=re.M))
    return names


def test_library_exports_every_declared_symbol(karma_lib):
    declared = _declared_symbols()
    assert declared == set(_lib.SIGNATURES), declared ^ set(_lib.SIGNATURES)
    for name in sorted(declared):
        assert hasattr(karma_lib, name), name
        assert name in _lib.SIGNATURES, f"{name} missing from karma_amd/_lib.py"
    out = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True, text=True, check=True)
    exported = {ln.split()[-1] for ln in out.stdout.splitlines() if " T " in ln}
    # the drop-in C++ symbol crc32c::Extend(unsigned, const char*, unsigned long)
    assert "_ZN6crc32c6ExtendEjPKcm" in exported
    assert declared <= exported
    # nothing but the ABI leaks out
    assert all(s.startswith("karma_") or s == "_ZN6crc32c6ExtendEjPKcm" for s in exported)


def test_abi_version_and_errors(karma_lib):
    assert karma_lib.karma_crc32c_abi_version() == 1
    assert karma_lib.karma_crc32c_strerror(0) == b"ok"
    assert karma_lib.karma_crc32c_strerror(-2) == b"no usable HIP device"


def test_host_extend_golden(vectors):
    for c in vectors["kat"]:
        assert K.Extend(case_init(c), case_bytes("kat", c)) == int(c["crc"], 16), c["name"]
    for c in vectors["pattern"]:
        if c["n"] <= (1 << 21):
            assert K.Value(case_bytes("pattern", c)) == int(c["crc"], 16)
    for c in vectors["splitmix"]:
        assert K.Extend(case_init(c), case_bytes("splitmix", c)) == int(c["crc"], 16)


def test_host_paths_agree_misaligned():
    rng = np.random.default_rng(11)
    data = rng.integers(0, 256, 20000, dtype=np.uint8)
    L = _lib.lib()
    for _ in range(500):
        off = int(rng.integers(0, 16))
        n = int(rng.integers(0, 19000))
        init = int(rng.integers(0, 1 << 32))
        a = L.karma_crc32c_extend_host(init, data.ctypes.data + off, n)
        b = L.karma_crc32c_extend_host_portable(init, data.ctypes.data + off, n)
        assert a == b


def test_mask_unmask(vectors):
    for m in vectors["mask"]:
        assert K.Mask(int(m["crc"], 16)) == int(m["masked"], 16)
        assert K.Unmask(int(m["masked"], 16)) == int(m["crc"], 16)
    assert K.kMaskDelta == 0xA282EAD8


def test_combine_identities():
    # Value(A||B) = Z_|B|(Value(A)) ^ Value(B);  Extend(c, D) = Z_|D|(c) ^ Value(D)
    rng = np.random.default_rng(2)
    for _ in range(200):
        a = rng.integers(0, 256, int(rng.integers(0, 3000)), dtype=np.uint8).tobytes()
        b = rng.integers(0, 256, int(rng.integers(0, 3000)), dtype=np.uint8).tobytes()
        assert K.Combine(K.Value(a), K.Value(b), len(b)) == K.Value(a + b)
        c = int(rng.integers(0, 1 << 32))
        assert K.Combine(c, K.Value(b), len(b)) == K.Extend(c, b)
    # large shifts (the multi-level combine of a 64 MiB stream uses Z_{unit*64^k})
    assert K.Combine(K.Value(b"x"), K.Value(b""), 0) == K.Value(b"x")


def test_dropin_cpp_links_against_engine(karma_lib, tmp_path):
    exe = tmp_path / "dropin_test"
    cmd = ["g++", "-std=c++20", "-O1", "-UNDEBUG", "-I", os.path.join(ROOT, "include"),
           os.path.join(ROOT, "tests", "cpp", "dropin_test.cc"), "-L", os.path.dirname(_lib.LIB_PATH),
           "-lkarma_crc32c", f"-Wl,-rpath,{os.path.dirname(_lib.LIB_PATH)}", "-o", str(exe)]
    subprocess.run(cmd, check=True)
    r = subprocess.run([str(exe)], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    assert "dropin_test: ok" in r.stdout
    # it resolved crc32c::Extend from libkarma_crc32c.so, not from a copy of crc32c.cc
    nm = subprocess.run(["nm", "-u", str(exe)], capture_output=True, text=True, check=True).stdout
    assert "_ZN6crc32c6ExtendEjPKcm" in nm


def _no_gpu():
    try:
        import torch
        return not torch.cuda.is_available()
    except Exception:
        return True


@pytest.mark.skipif(not _no_gpu(), reason="checks the no-device behaviour")
def test_device_entry_points_refuse_without_gpu(karma_lib):
    out = ctypes.c_uint32()
    buf = ctypes.create_string_buffer(64)
    st = karma_lib.karma_crc32c_batch_fixed(ctypes.addressof(buf), 16, 4, None, 0, ctypes.addressof(out), None)
    assert st == _lib.KARMA_E_NO_DEVICE
    st = karma_lib.karma_crc32c_stream(0, ctypes.addressof(buf), 64, ctypes.addressof(out), None)
    assert st == _lib.KARMA_E_NO_DEVICE
    assert b"no HIP device" in karma_lib.karma_crc32c_last_error()
    with pytest.raises(_lib.KarmaError):
        K.device_cu_count()


def test_invalid_arguments_rejected_before_device(karma_lib):
    # null output / data with records: KARMA_E_INVALID regardless of the device
    assert karma_lib.karma_crc32c_batch_fixed(None, 16, 4, None, 0, None, None) == _lib.KARMA_E_INVALID
    assert karma_lib.karma_crc32c_batch_ragged(None, None, None, 3, 0, None, 0, None, None) == _lib.KARMA_E_INVALID
    # zero records is a no-op success
    assert karma_lib.karma_crc32c_batch_fixed(None, 16, 0, None, 0, None, None) == 0


def test_python_batch_api_rejects_host_tensors():
    import torch
    with pytest.raises(ValueError):
        K.value_batch_fixed(torch.zeros(64, dtype=torch.uint8), 16)
    with pytest.raises(ValueError):
        K.extend_stream(0, torch.zeros(64, dtype=torch.uint8))


def test_wal_and_kfp_host_logic_without_gpu(karma_lib):
    """The structural half of the KFP layer runs on the host; with nothing to checksum it needs
    no device, and any device work (checksums, the WAL replay walk) refuses with
    KARMA_E_NO_DEVICE (no CPU fallback)."""
    import struct

    import numpy as np

    u64, sz, i32 = ctypes.c_uint64, ctypes.c_size_t, ctypes.c_int
    # KFP: a first frame whose size is over MAX_FRAME_SIZE stops before any CRC (frame.cc:70-73)
    buf = np.frombuffer(b"\xff\xff\xff\xff" + bytes(40), np.uint8).copy()
    n, used, why = sz(), u64(), i32()
    st = karma_lib.karma_kfp_parse_batch(buf.ctypes.data, None, buf.nbytes, 16, None, ctypes.byref(n),
                                         ctypes.byref(used), ctypes.byref(why), -1)
    assert st == 0 and (n.value, used.value, why.value) == (0, 0, 1)  # KARMA_KFP_BAD_SIZE
    # fewer than 20 bytes: wait for more (nullopt)
    st = karma_lib.karma_kfp_parse_batch(buf.ctypes.data, None, 19, 16, None, ctypes.byref(n), ctypes.byref(used),
                                         ctypes.byref(why), -1)
    assert st == 0 and (n.value, used.value, why.value) == (0, 0, 0)
    # a complete frame needs its CRC: refused without a device
    frame = struct.pack("<IBhBII", 24, 123, 1, 0, 0, 0) + b"abcd" + b"\0\0\0\0"
    fb = np.frombuffer(frame, np.uint8).copy()
    st = karma_lib.karma_kfp_parse_batch(fb.ctypes.data, None, fb.nbytes, 16, None, ctypes.byref(n),
                                         ctypes.byref(used), ctypes.byref(why), -1)
    assert st == _lib.KARMA_E_NO_DEVICE
    # WAL replay walks the headers on the device too: refused without one (no host walk)
    seg = 4096
    wal = np.zeros(2 * seg, np.uint8)
    wal[4] = 7
    nr, stop, status = u64(), u64(), i32()
    st = karma_lib.karma_wal_replay(wal.ctypes.data, None, wal.nbytes, seg, 0, ctypes.byref(nr), ctypes.byref(stop),
                                    ctypes.byref(status), None, 0, -1)
    assert st == _lib.KARMA_E_NO_DEVICE
    # replay from the end of the image has nothing to walk
    st = karma_lib.karma_wal_replay(wal.ctypes.data, None, wal.nbytes, seg, wal.nbytes, ctypes.byref(nr),
                                    ctypes.byref(stop), ctypes.byref(status), None, 0, -1)
    assert st == 0 and (nr.value, stop.value, status.value) == (0, wal.nbytes, 0)
    # invalid geometry is rejected before any device work
    assert karma_lib.karma_wal_replay(wal.ctypes.data, None, wal.nbytes, 3000, 0, ctypes.byref(nr),
                                      ctypes.byref(stop), ctypes.byref(status), None, 0, -1) == _lib.KARMA_E_INVALID


def test_wal_replay_dir_host_logic(karma_lib, tmp_path):
    """karma_wal_replay_dir's directory handling (wal::load_from_path, wal.cc:9-27) runs before any
    device work: files named by their decimal WAL offset, equal sizes, no gaps."""
    u64, i32 = ctypes.c_uint64, ctypes.c_int
    base, nr, stop, status = u64(), u64(), u64(), i32()

    def call(d, seg=0, start=0):
        return karma_lib.karma_wal_replay_dir(str(d).encode(), seg, start, ctypes.byref(base), ctypes.byref(nr),
                                              ctypes.byref(stop), ctypes.byref(status), None, 0, -1)

    assert call(tmp_path / "missing") == _lib.KARMA_E_IO
    empty = tmp_path / "empty"
    empty.mkdir()
    (empty / "not-a-segment").write_bytes(b"x")  # ignored: not a decimal name
    assert call(empty, start=7) == 0 and (nr.value, stop.value, status.value) == (0, 7, 0)
    seg = 4096
    ok = tmp_path / "ok"
    ok.mkdir()
    for off in (3 * seg, 4 * seg):
        (ok / str(off)).write_bytes(bytes(seg))
    (ok / "99").mkdir()  # a directory with a decimal name is not a segment
    assert call(ok, start=0) == _lib.KARMA_E_INVALID  # start before the first segment
    assert call(ok, start=3 * seg) == _lib.KARMA_E_NO_DEVICE  # valid: the walk needs the device
    assert call(ok, seg=seg, start=3 * seg) == _lib.KARMA_E_NO_DEVICE
    gap = tmp_path / "gap"
    gap.mkdir()
    for off in (0, 2 * seg):
        (gap / str(off)).write_bytes(bytes(seg))
    assert call(gap) == _lib.KARMA_E_INVALID
    sizes = tmp_path / "sizes"
    sizes.mkdir()
    (sizes / "0").write_bytes(bytes(seg))
    (sizes / str(seg)).write_bytes(bytes(seg // 2))
    assert call(sizes) == _lib.KARMA_E_INVALID
    assert karma_lib.karma_crc32c_strerror(_lib.KARMA_E_IO) == b"file I/O error"


def test_python_wal_api_refuses_without_gpu():
    """karma_amd.wal raises on device work without a GPU (no CPU fallback); replay from the end
    of an image needs none."""
    import numpy as np

    from karma_amd import wal as W
    img = np.zeros(2 * 4096, np.uint8)
    r = W.replay(img, 4096, start=img.nbytes)
    assert (len(r.records), r.stop, r.status) == (0, img.nbytes, W.END)
    with pytest.raises(K.KarmaError) as e:
        W.replay(img, 4096)
    assert e.value.status == _lib.KARMA_E_NO_DEVICE


def test_shipped_library_has_no_variant_knobs():
    """The shipped library reads no KARMA_* variant from the environment: a stray variable can
    never select a timing-only kernel (wrong CRCs) or change a plan."""
    with open(_lib.LIB_PATH, "rb") as f:
        blob = f.read()
    for knob in (b"KARMA_CRC_VARIANT", b"KARMA_RAGGED_VARIANT", b"KARMA_FOLD_MAX_K", b"KARMA_SPLIT_OVERDECOMPOSE",
                 b"KARMA_WALK_VARIANT", b"KARMA_WALK_SUB", b"KARMA_WAL_SMALL_MAX", b"KARMA_RAGGED_PLAN",
                 b"KARMA_RAGGED_EDGES", b"KARMA_LB_SEQ_MAX", b"KARMA_DIRECT_VARIANT", b"KARMA_FIXED_GRID_MULT",
                 b"KARMA_FINALIZE_PER_CU", b"KARMA_WAL_LIST_CRC", b"KARMA_SMALL_STAGED", b"KARMA_APPEND_CALL_BYTES", b"KARMA_WALK_DIRECT",
                 b"KARMA_RAGGED_DYN", b"KARMA_GATHER_PARTS", b"KARMA_SMALL_WHICH",
                 b"KARMA_STAGE_SKEW", b"KARMA_STAGE_R8", b"KARMA_SEGMENT_ONCE", b"KARMA_RAGGED_GRID",
                 b"KARMA_STAGE_TIMING", b"KARMA_STAGE_PAIR", b"KARMA_RAGGED_UNITS_MODE", b"KARMA_RAGGED_UNITS_FLAT",
                 b"KARMA_RAGGED_UNITS_TWICE", b"KARMA_RAGGED_UNITS_FIXEDLOOP", b"KARMA_SPEC_WIDE", b"KARMA_STAGE_WIDE", b"KARMA_SPEC_AL"):
        assert knob not in blob, knob


def test_library_never_page_locks_caller_memory():
    """Host buffers reach the device through the library's own pinned staging: the library does
    not import hipHostRegister at all (round 1's per-call register / unregister of caller pages is
    gone)."""
    out = subprocess.run(["nm", "-D", "--undefined-only", _lib.LIB_PATH], capture_output=True, text=True, check=True)
    imported = {ln.split()[-1].split("@")[0] for ln in out.stdout.splitlines() if ln.strip()}
    assert "hipHostRegister" not in imported and "hipHostUnregister" not in imported
