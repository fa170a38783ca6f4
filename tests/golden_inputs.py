"""Rebuild the input bytes a golden-vector case describes (test infrastructure)."""
from __future__ import annotations

import numpy as np

import synth


def case_bytes(kind: str, c: dict) -> bytes:
    if kind == "kat":
        return bytes.fromhex(c["hex"])
    if kind == "pattern":
        return synth.pattern(c["n"], c["start"])
    if kind == "splitmix":
        return synth.splitmix(c["seed"], c["off"], c["n"])
    raise ValueError(kind)


def case_init(c: dict) -> int:
    v = c.get("init", 0)
    return int(v, 16) if isinstance(v, str) else int(v)


def ragged_inputs(g: dict):
    lens = synth.loguniform_lengths(g["seed_len"], g["count"], g["lo"], g["hi"])
    offs, arena = synth.ragged_layout(lens, header=g["header"])
    data = synth.splitmix_np(g["seed_data"], 0, arena + 16).copy()
    init = synth.splitmix_words(g["seed_len"] ^ 0x5A5A, 0, g["count"]).astype(np.uint32) if g["with_init"] else None
    want = np.array([int(x, 16) for x in g["crc"]], dtype=np.uint32)
    return data, offs, lens, init, want
