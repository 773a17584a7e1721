"""Entry accounting of the streaming path at scale: a tree of N int64 keys,
K+1 batches of 1M keys (half overwrites, half new) inserted twice, then the
entry count (before and after the fold) against the expected N + (K+1)*500K,
a verify and a sample of gets.  Usage: python tools/pages_count_check.py N K [csr]"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from riak_ensemble_amd import synctree_hip, _lib  # noqa: E402

N = int(sys.argv[1])
K = int(sys.argv[2])
B = 1_000_000
dev = torch.device('cuda', 0)
t = synctree_hip.DeviceTree()
if len(sys.argv) > 3 and sys.argv[3] == 'csr':
    t.debug_knob(_lib.ST_DBG_PAGES, -1)
if len(sys.argv) > 3 and sys.argv[3] == 'check':
    t.debug_knob(_lib.ST_DBG_PAGE_CHECK, 1)
seed = 0x5EED0005
for a in range(0, N, 10_000_000):
    m = min(10_000_000, N - a)
    k = bench._dev_keys(seed, a, m, dev, torch)
    v = bench._dev_values(torch.arange(a, a + m, dtype=torch.int64, device=dev), dev, torch)
    t.insert_int64_device(k.data_ptr(), v.data_ptr(), m, 17)
    del k, v
torch.cuda.synchronize()
print('built', t.num_entries(), flush=True)
rng = np.random.default_rng(5)
for rep in range(2):
    for j in range(K + 1):
        r2 = np.random.default_rng(100 + j)
        old = torch.from_numpy(r2.integers(0, N, B // 2)).to(dev)
        k = torch.cat([bench._dev_keys_at(seed, old, dev, torch), bench._dev_keys(seed, N + j * B, B - B // 2, dev, torch)])
        seq = torch.cat([old + 1, torch.arange(N + j * B, N + j * B + (B - B // 2), device=dev)])
        v = bench._dev_values(seq, dev, torch)
        uniq = torch.unique(k).numel()
        before = t.num_entries()
        t.insert_int64_device(k.contiguous().data_ptr(), v.contiguous().data_ptr(), B, 17)
        torch.cuda.synchronize()
        print('rep %d batch %d: uniq %d, entries %d -> %d (+%d), pages %s' % (rep, j, uniq, before, t.num_entries(),
              t.num_entries() - before, t.page_stats()), flush=True)
exp = N + (K + 1) * (B - B // 2)
print('expected', exp, 'paged count', t.num_entries(), flush=True)
print('verify', t.verify(), flush=True)
print('after fold', t.num_entries(), 'pages', t.page_stats(), flush=True)
t.close()
