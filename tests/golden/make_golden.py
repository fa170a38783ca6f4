#!/usr/bin/env python3
"""Generate tests/golden/*.json from the REFERENCE crc32c (test infrastructure).

Run in the build container (needs /root/reference):

    make -C oracle            # builds oracle/_ref/libkarma_ref_crc32c.so from
                              # /root/reference/karma-util/crc32c.cc + coding.cc
    python tests/golden/make_golden.py

Every expected value below is computed by the reference's own ``crc32c::Extend``
(karma-util/crc32c.cc:275-376) through oracle/ref_shim.cc.  Inputs are described by the
generators in tests/synth.py (or given inline as hex), so the fixtures stay small and the
GPU box can rebuild the bytes.  The committed JSON is data only; no reference source.
"""
from __future__ import annotations

import ctypes
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.dirname(HERE))
import synth  # noqa: E402

REF_SO = os.path.join(ROOT, "oracle", "_ref", "libkarma_ref_crc32c.so")


def load_ref():
    lib = ctypes.CDLL(REF_SO)
    lib.ref_crc32c_extend.restype = ctypes.c_uint32
    lib.ref_crc32c_extend.argtypes = [ctypes.c_uint32, ctypes.c_void_p, ctypes.c_size_t]
    lib.ref_crc32c_ragged_mt.restype = ctypes.c_int
    lib.ref_crc32c_ragged_mt.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                         ctypes.c_uint64, ctypes.c_void_p, ctypes.c_int]
    return lib


REF = None


def ext(init: int, data: bytes, misalign: int = 0) -> int:
    """Reference Extend over ``data`` placed at a buffer offset of ``misalign`` bytes."""
    buf = ctypes.create_string_buffer(b"\0" * misalign + data + b"\0" * 8, misalign + len(data) + 8)
    return REF.ref_crc32c_extend(init, ctypes.addressof(buf) + misalign, len(data))


def hx(v: int) -> str:
    return f"{v:08x}"


def kat_cases():
    iscsi = bytes.fromhex(
        "01c000000000000000000000000000001400000000000400000000140000001828000000000000000200000000000000")
    cases = []
    named = [
        ("empty", b""),
        ("check_123456789", b"123456789"),
        ("zeros_32", b"\x00" * 32),
        ("ones_32", b"\xff" * 32),
        ("ascending_32", bytes(range(32))),
        ("descending_32", bytes(range(31, -1, -1))),
        ("rfc3720_iscsi_read_pdu", iscsi),
        ("hello_world", b"hello world"),
        ("transport_header", b"I am header"),
        ("transport_body", b"I am body"),
    ]
    for name, data in named:
        cases.append({"name": name, "hex": data.hex(), "init": 0, "crc": hx(ext(0, data))})
    # streaming semantics: Extend(Value(A), B) == Value(A || B)  (frame.cc:56-57)
    a, b = b"hello ", b"world"
    cases.append({"name": "extend_hello_world", "hex": b.hex(), "init": ext(0, a), "crc": hx(ext(ext(0, a), b))})
    h, p = b"I am header", b"I am body"
    cases.append({"name": "frame_crc", "hex": p.hex(), "init": ext(0, h), "crc": hx(ext(ext(0, h), p))})
    mask = []
    for v in [0, 1, 0xE3069283, 0xFFFFFFFF, 0x12345678, 0xA282EAD8]:
        m = ((v >> 15) | (v << 17)) & 0xFFFFFFFF
        m = (m + 0xA282EAD8) & 0xFFFFFFFF
        mask.append({"crc": hx(v), "masked": hx(m)})
    return cases, mask


def pattern_cases():
    out = []
    lens = list(range(0, 301)) + [511, 512, 513, 1000, 1023, 1024, 1025, 2047, 2048, 2049, 4095, 4096, 4097,
                                  8191, 8192, 8193, 65535, 65536, 65537, 1 << 20, (1 << 20) + 13]
    for n in lens:
        data = synth.pattern(n)
        out.append({"n": n, "start": 0, "init": 0, "crc": hx(ext(0, data))})
    # start offsets shift the pattern; misalign exercises the reference prologue (crc32c.cc:323-329)
    for start in range(1, 17):
        for n in (4096, 100, 17):
            data = synth.pattern(n, start)
            out.append({"n": n, "start": start, "init": 0, "crc": hx(ext(0, data, misalign=start % 4))})
    n = 64 << 20
    out.append({"n": n, "start": 0, "init": 0, "crc": hx(ext(0, synth.pattern(n)))})
    return out


def splitmix_cases():
    out = []
    rng = np.random.default_rng(20261015)
    base = [(42, 0, 4096, 0), (42, 0, 65536, 0), (42, 0, 1 << 20, 0), (42, 0, 4096, 0xDEADBEEF),
            (42, 1000, 3096, 0)]
    for seed, off, n, init in base:
        out.append({"seed": seed, "off": off, "n": n, "init": hx(init), "crc": hx(ext(init, synth.splitmix(seed, off, n)))})
    # random (offset, length, init) triples, including unaligned offsets and tiny lengths
    for _ in range(400):
        seed = int(rng.integers(0, 1 << 63))
        off = int(rng.integers(0, 1 << 20))
        n = int(rng.choice([rng.integers(0, 64), rng.integers(0, 4096), rng.integers(0, 1 << 17)]))
        init = int(rng.integers(0, 1 << 32))
        out.append({"seed": seed, "off": off, "n": n, "init": hx(init), "crc": hx(ext(init, synth.splitmix(seed, off, n)))})
    return out


def fixed_records_case():
    """Config-2 shape at fixture size: 4 KiB records of splitmix(seed=42); first 2048 CRCs."""
    seed, rec, nrec = 42, 4096, 2048
    data = synth.splitmix(seed, 0, rec * nrec)
    crcs = [ext(0, data[i * rec:(i + 1) * rec]) for i in range(nrec)]
    # checksum of checksums: Value() over the little-endian u32 CRC array
    digest = ext(0, np.array(crcs, dtype="<u4").tobytes())
    return {"seed": seed, "rec_bytes": rec, "n_rec": nrec, "crc": [hx(c) for c in crcs], "digest": hx(digest)}


def ragged_case(seed_len: int, seed_data: int, count: int, lo: int, hi: int, header: int, with_init: bool):
    lens = synth.loguniform_lengths(seed_len, count, lo, hi)
    offs, arena = synth.ragged_layout(lens, header=header)
    data = np.frombuffer(synth.splitmix(seed_data, 0, arena + 16), dtype=np.uint8).copy()
    init = synth.splitmix_words(seed_len ^ 0x5A5A, 0, count).astype(np.uint32) if with_init else None
    out = np.zeros(count, dtype=np.uint32)
    REF.ref_crc32c_ragged_mt(data.ctypes.data, offs.ctypes.data, lens.ctypes.data,
                             init.ctypes.data if init is not None else None, count, out.ctypes.data, 8)
    digest = ext(0, out.astype("<u4").tobytes())
    return {"seed_len": seed_len, "seed_data": seed_data, "count": count, "lo": lo, "hi": hi, "header": header,
            "with_init": with_init, "arena_bytes": int(arena),
            "crc": [hx(int(c)) for c in out], "digest": hx(digest)}


def main():
    global REF
    REF = load_ref()
    kats, mask = kat_cases()
    doc = {
        "about": "CRC-32C golden vectors computed by the reference crc32c::Extend "
                 "(karma-util/crc32c.cc:275-376) built from /root/reference by oracle/Makefile; "
                 "inputs per tests/synth.py",
        "kat": kats,
        "mask": mask,
        "pattern": pattern_cases(),
        "splitmix": splitmix_cases(),
    }
    with open(os.path.join(HERE, "crc32c_vectors.json"), "w") as f:
        json.dump(doc, f, indent=0)
    recs = {
        "about": "per-record CRCs (reference crc32c::Value/Extend) for batched record fixtures",
        "fixed_4k": fixed_records_case(),
        "ragged_replay_mix": ragged_case(7, 11, 4096, 1, 65536, 8, False),
        "ragged_small_init": ragged_case(9, 13, 4096, 1, 300, 8, True),
        "ragged_tiny_unaligned": ragged_case(21, 23, 2048, 1, 40, 3, True),
    }
    with open(os.path.join(HERE, "crc32c_records.json"), "w") as f:
        json.dump(recs, f, indent=0)
    print("wrote", os.listdir(HERE))


if __name__ == "__main__":
    main()
