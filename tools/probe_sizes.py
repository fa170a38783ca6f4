"""HBM probe vs the fixed kernel over 1-16 GiB (per-launch overhead vs. streaming rate). GPU box."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch, karma_amd as K
x = torch.empty(16 << 30, dtype=torch.uint8, device="cuda")
o = torch.zeros(1, dtype=torch.uint32, device="cuda")
out = torch.empty(4 << 20, dtype=torch.uint32, device="cuda")
K.fill_splitmix64(x[: 16 << 30], 42)
torch.cuda.synchronize()
def t(fn, reps=10):
    for _ in range(3): fn()
    torch.cuda.synchronize()
    e = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
    for a, b in e:
        a.record(); fn(); b.record()
    torch.cuda.synchronize()
    return sorted(a.elapsed_time(b) for a, b in e)[reps // 2]
for g in (1, 2, 4, 8, 16):
    n = g << 30
    p = t(lambda: K.stream_probe(x[:n], o))
    k = t(lambda: K.value_batch_fixed(x[:n], 4096, out=out))
    print(f"{g:2d} GiB probe {p:.4f} ms ({p/g:.4f}/GiB)  fixed {k:.4f} ms ({k/g:.4f}/GiB)  ratio {p/k:.3f}", flush=True)
