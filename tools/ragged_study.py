#!/usr/bin/env python3
"""The ragged path against the fixed one, and builds of it against each other: times the units
kernel alone (karma_crc32c_time_next_units) and the whole call for several 4 GiB layouts, one
process, interleaved rounds.  Run on the GPU box from the repo root:

    python tools/ragged_study.py
    LIBS="grid=karma_amd/lib/libkarma_crc32c.so,units=tools/lib/libkarma_crc32c_nogrid.so" \\
        python tools/ragged_study.py

LIBS names the builds compared (name=path, comma-separated; default: the shipped library).  They
are loaded side by side (each keeps its own kernels and state; `name=path@KNOB=V;...` runs a build
with A/B knobs set, e.g. a timing form of the tools build, whose CRCs then differ), so every layout runs through
every build in the same process, rounds interleaved; every build's CRCs are compared with the
first one's.  Builds, not environment knobs: the tools build's extra kernels change the register
allocation of the kernels they share a file with.
"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import karma_amd as K  # noqa: E402
from karma_amd import _lib  # noqa: E402
import synth  # noqa: E402

LIBS = {}
KNOBS = {}  # name -> {knob: value}: name=path@KNOB=V;KNOB2=V2 runs that build with those A/B knobs set
_loaded = {}
for item in os.environ.get("LIBS", f"shipped={_lib.LIB_PATH}").split(","):
    name, _, path = item.partition("=")
    path, _, kn = path.partition("@")
    path = path if os.path.isabs(path) else os.path.join(ROOT, path)
    if path not in _loaded:
        _loaded[path] = _lib.load(path)
    LIBS[name] = _loaded[path]
    KNOBS[name] = dict(kv.split("=", 1) for kv in kn.replace("+", ";").split(";") if kv)


def set_knobs(name):
    for kv in KNOBS.values():
        for k in kv:
            os.environ.pop(k, None)
    os.environ.update(KNOBS.get(name, {}))
dev = torch.device("cuda:0")
GB = 4 << 30
RAW = GB + (64 << 20)  # config 3 arena = 4.01 GiB of payload + 8-B headers
raw = torch.empty(RAW, dtype=torch.uint8, device=dev)
K.fill_splitmix64(raw, 42)
torch.cuda.synchronize()
print("fill ok", hex(raw.data_ptr()), flush=True)
stream = torch.cuda.current_stream()
sh = stream.cuda_stream


def fixed_case(L, rec):
    n = GB // rec
    out = torch.empty(n, dtype=torch.uint32, device=dev)

    def run():
        set_knobs(None)
        _lib.check("fixed", L.karma_crc32c_batch_fixed(raw.data_ptr(), rec, n, None, 0, out.data_ptr(), sh))
    return run, n * rec, out


_dev_layouts = {}


def ragged_case(L, key, lens, offs, lib_name=None):
    if key not in _dev_layouts:
        end = int((offs.astype(np.uint64) + lens.astype(np.uint64)).max())
        assert end <= RAW, f"layout ends at {end} > buffer {RAW}"  # checked on the host before any launch
        _dev_layouts[key] = (torch.from_numpy(offs.astype(np.int64)).to(dev),
                             torch.from_numpy(lens.astype(np.int32)).to(dev), lens.size, int(lens.sum()))
    d_off, d_len, n, total = _dev_layouts[key]
    out = torch.empty(n, dtype=torch.uint32, device=dev)

    def run():
        set_knobs(lib_name)
        _lib.check("ragged", L.karma_crc32c_batch_ragged(raw.data_ptr(), d_off.data_ptr(), d_len.data_ptr(), n, total,
                                                         None, 0, out.data_ptr(), sh))
    return run, total, out


count = int(GB / (((65536 - 64) / np.log(1024)) + 8))
lens = synth.loguniform_lengths(7, count, 64, 65536)
offs, _ = synth.ragged_layout(lens, header=8)
srt = np.sort(lens)[::-1].copy()
o2, _ = synth.ragged_layout(srt, header=8)
layouts = {"aligned 4096": (np.full(GB // 4096, 4096, np.uint32), np.arange(GB // 4096, dtype=np.uint64) * 4096),
           "aligned 2048": (np.full(GB // 2048, 2048, np.uint32), np.arange(GB // 2048, dtype=np.uint64) * 2048),
           "config3": (lens, offs), "config3 sorted desc": (srt, o2)}
if os.environ.get("LAYOUTS"):  # a subset, e.g. LAYOUTS="aligned 4096,aligned 2048"
    layouts = {k: v for k, v in layouts.items() if k in os.environ["LAYOUTS"].split(",")}
cases = {}
first = next(iter(LIBS))
for lib_name, L in LIBS.items():  # (every build: its CRCs compared with the first build's)
    cases[f"fixed 4096 [{lib_name}]"] = (fixed_case(L, 4096), "fixed 4096")
for name, (ln, of) in layouts.items():
    for lib_name, L in LIBS.items():
        cases[f"ragged {name} [{lib_name}]"] = (ragged_case(L, name, ln, of, lib_name), name)

for name, ((run, nbytes, out), _) in cases.items():
    print("first call:", name, flush=True)
    run()
    torch.cuda.synchronize()
ref = {}
mism = {}
for name, ((run, nbytes, out), key) in cases.items():
    if key is None:
        continue
    got = out.cpu().numpy().copy()
    if key not in ref:
        ref[key] = got
    mism[name] = int((got != ref[key]).sum())
res = {k: ([], []) for k in cases}
for rnd in range(int(os.environ.get("ROUNDS", "5"))):
    for name, ((run, nbytes, out), _) in (cases.items() if rnd % 2 == 0 else reversed(list(cases.items()))):
        for _ in range(2):
            run()
        torch.cuda.synchronize()
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(10)]
        uev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(10)]
        for a, b in uev:
            a.record()
            b.record()
        torch.cuda.synchronize()
        lib_name = name[name.rindex("[") + 1:-1]
        for i in range(10):
            ev[i][0].record()
            LIBS[lib_name].karma_crc32c_time_next_units(uev[i][0].cuda_event, uev[i][1].cuda_event)
            run()
            ev[i][1].record()
        torch.cuda.synchronize()
        res[name][0].append(np.median([a.elapsed_time(b) for a, b in ev]))
        res[name][1].append(np.median([a.elapsed_time(b) for a, b in uev]))
for name, ((run, nbytes, out), _) in cases.items():
    call, units = np.median(res[name][0]), np.median(res[name][1])
    print(f"{name:40s} payload {nbytes / 2**30:5.2f} GiB  call {call:.4f} ms ({nbytes / call / 1e6:7.1f} GB/s, "
          f"{nbytes / call / 8e9:.3f})  units {units:.4f} ms ({nbytes / units / 1e6:7.1f} GB/s, {nbytes / units / 8e9:.3f})"
          + (f"  mismatches vs [{first}]: {mism[name]}" if name in mism else ""), flush=True)
