import sys, os
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import numpy as np, torch
import karma_amd as K, oracle_lib
dev = torch.device("cuda:0")
rng = np.random.default_rng(5)
host = rng.integers(0, 256, size=(1 << 23) + 64, dtype=np.uint8)
dbuf = torch.from_numpy(host).to(dev)
size = (1 << 23) + 64
rng = np.random.default_rng(4)
lens = np.concatenate([rng.integers(0, 300000, 500), [size, size - 1, 1 << 20, 5, 0, 17, 1 << 22]]).astype(np.uint32)
offs = np.array([int(rng.integers(0, size - int(n) + 1)) for n in lens[:-7]] + [0, 1, size - (1 << 20), size - 5, size, size - 17, 3], dtype=np.uint64)
want = oracle_lib.ragged_crcs(host, offs, lens)
d_off = torch.from_numpy(offs.astype(np.int64)).to(dev); d_len = torch.from_numpy(lens.astype(np.int32)).to(dev)
for tl in [int(lens.sum()), None, int(lens.sum()), None]:
    got = K.extend_batch_ragged(dbuf, d_off, d_len, total_len=tl).cpu().numpy()
    print("total_len", tl, "mismatches", int((got != want).sum()))
for sub in [slice(0, 100), slice(500, 507), slice(0, 507)]:
    got = K.extend_batch_ragged(dbuf, d_off[sub], d_len[sub], total_len=int(lens[sub].sum())).cpu().numpy()
    print("sub", sub, "mismatches", int((got != want[sub]).sum()))
