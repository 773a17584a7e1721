"""Config-5 paged batches for profiling: a tree of N keys, one warm-up
batch, then K 1M-key batches (50 % overwrites, 50 % new) through the paged
layout, timing off.  Usage: python tools/prof_pages.py [N] [K]"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from riak_ensemble_amd import synctree_hip  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 100_000_000
K = int(sys.argv[2]) if len(sys.argv) > 2 else 5
B = 1_000_000
dev = torch.device('cuda', 0)
t = synctree_hip.DeviceTree()
seed = 0x5EED0005
for a in range(0, N, 10_000_000):
    m = min(10_000_000, N - a)
    k = bench._dev_keys(seed, a, m, dev, torch)
    v = bench._dev_values(torch.arange(a, a + m, dtype=torch.int64, device=dev), dev, torch)
    t.insert_int64_device(k.data_ptr(), v.data_ptr(), m, 17)
    del k, v
rng = np.random.default_rng(5)
for j in range(K + 1):
    old = torch.from_numpy(rng.integers(0, N, B // 2)).to(dev)
    k = torch.cat([bench._dev_keys_at(seed, old, dev, torch), bench._dev_keys(seed, N + j * B, B - B // 2, dev, torch)]).contiguous()
    seq = torch.cat([old + 1, torch.arange(N + j * B, N + j * B + (B - B // 2), device=dev)])
    v = bench._dev_values(seq, dev, torch).contiguous()
    t.insert_int64_device(k.data_ptr(), v.data_ptr(), B, 17)
torch.cuda.synchronize()
print('pages', t.page_stats(), 'entries', t.num_entries())
t.close()
