"""The CPU oracle (oracle/crc32c_port.c) against the golden vectors made by the reference's own
crc32c.cc (tests/golden/make_golden.py), and against the reference build when it is shipped."""
import numpy as np
import pytest

import oracle_lib
import synth
from golden_inputs import case_bytes, case_init, ragged_inputs


def test_known_answers(vectors):
    for c in vectors["kat"]:
        assert oracle_lib.extend(case_init(c), case_bytes("kat", c)) == int(c["crc"], 16), c["name"]


def test_check_value_and_rfc3720():
    assert oracle_lib.extend(0, b"123456789") == 0xE3069283
    iscsi = bytes.fromhex("01c000000000000000000000000000001400000000000400000000140000001828000000000000000200000000000000")
    assert oracle_lib.extend(0, iscsi) == 0xD9963A56


def test_pattern_vectors(vectors):
    for c in vectors["pattern"]:
        assert oracle_lib.extend(0, case_bytes("pattern", c)) == int(c["crc"], 16), (c["n"], c["start"])


def test_splitmix_vectors(vectors):
    for c in vectors["splitmix"]:
        assert oracle_lib.extend(case_init(c), case_bytes("splitmix", c)) == int(c["crc"], 16), c


def test_mask_vectors(vectors):
    port = oracle_lib.port()
    port.oracle_crc32c_mask.restype = port.oracle_crc32c_unmask.restype = oracle_lib._c.c_uint32
    port.oracle_crc32c_mask.argtypes = port.oracle_crc32c_unmask.argtypes = [oracle_lib._c.c_uint32]
    for m in vectors["mask"]:
        assert port.oracle_crc32c_mask(int(m["crc"], 16)) == int(m["masked"], 16)
        assert port.oracle_crc32c_unmask(int(m["masked"], 16)) == int(m["crc"], 16)


def test_fixed_records_fixture(records):
    g = records["fixed_4k"]
    got = oracle_lib.splitmix_fixed_crcs(g["seed"], g["rec_bytes"], 0, g["n_rec"])
    want = np.array([int(x, 16) for x in g["crc"]], dtype=np.uint32)
    assert np.array_equal(got, want)
    assert oracle_lib.extend(0, got.astype("<u4").tobytes()) == int(g["digest"], 16)


@pytest.mark.parametrize("key", ["ragged_replay_mix", "ragged_small_init", "ragged_tiny_unaligned"])
def test_ragged_fixtures(records, key):
    data, offs, lens, init, want = ragged_inputs(records[key])
    got = oracle_lib.ragged_crcs(data, offs, lens, init)
    assert np.array_equal(got, want)
    assert oracle_lib.extend(0, got.astype("<u4").tobytes()) == int(records[key]["digest"], 16)


def test_splitmix_generator_matches_fixture_stream():
    # the C generator (used for full-size GPU checks) and tests/synth.py agree byte for byte
    import ctypes
    buf = ctypes.create_string_buffer(4099)
    oracle_lib.port().oracle_splitmix_bytes(42, 13, buf, 4099)
    assert buf.raw[:4099] == synth.splitmix(42, 13, 4099)


def test_port_matches_reference_build():
    ref = oracle_lib.ref()
    if ref is None:
        pytest.skip("oracle/_ref not built (no /root/reference here)")
    rng = np.random.default_rng(3)
    data = rng.integers(0, 256, 70000, dtype=np.uint8)
    base = data.ctypes.data
    for _ in range(3000):
        off = int(rng.integers(0, 64))
        n = int(rng.choice([rng.integers(0, 70), rng.integers(0, 5000), rng.integers(0, 69000 - off)]))
        init = int(rng.integers(0, 1 << 32))
        a = oracle_lib.port().oracle_crc32c_extend(init, base + off, n)
        b = ref.ref_crc32c_extend(init, base + off, n)
        assert a == b, (off, n, init)
