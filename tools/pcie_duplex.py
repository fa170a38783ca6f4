"""tools/pcie_duplex.py -- what PCIe gives a host-memory WAL append.

Times, on one GPU, 4 MiB block copies between page-locked host buffers and HBM over 8
streams: H2D alone, D2H alone, and both directions at once (block k's D2H queued behind
block k's H2D on the same stream, as a device-framed append would).  Prints GB/s."""
import sys
import time

import torch


def main():
    total = int(sys.argv[1]) if len(sys.argv) > 1 else 196 << 20
    blk = int(sys.argv[2]) if len(sys.argv) > 2 else 4 << 20
    dev = torch.device("cuda", 0)
    h_src = torch.empty(total, dtype=torch.uint8).pin_memory()
    h_dst = torch.empty(total, dtype=torch.uint8).pin_memory()
    d_a = torch.empty(total, dtype=torch.uint8, device=dev)
    d_b = torch.empty(total, dtype=torch.uint8, device=dev)
    d_b.fill_(1)
    h_src.fill_(2)
    streams = [torch.cuda.Stream(dev) for _ in range(8)]
    nb = (total + blk - 1) // blk

    def run(h2d, d2h):
        for k in range(nb):
            s = streams[k % len(streams)]
            lo, hi = k * blk, min(total, (k + 1) * blk)
            with torch.cuda.stream(s):
                if h2d:
                    d_a[lo:hi].copy_(h_src[lo:hi], non_blocking=True)
                if d2h:
                    h_dst[lo:hi].copy_(d_b[lo:hi], non_blocking=True)
        torch.cuda.synchronize()

    for name, a, b in (("h2d", 1, 0), ("d2h", 0, 1), ("both", 1, 1)):
        for _ in range(3):
            run(a, b)
        reps = 10
        t0 = time.perf_counter()
        for _ in range(reps):
            run(a, b)
        dt = (time.perf_counter() - t0) / reps
        print(f"{name:5s} {total >> 20} MiB blocks {blk >> 10} KiB: {dt * 1e3:.3f} ms, "
              f"{total * (a + b) / dt / 1e9:.1f} GB/s total, {total / dt / 1e9:.1f} GB/s per direction", flush=True)


if __name__ == "__main__":
    main()
