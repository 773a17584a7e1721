"""Config-5 batch breakdown: a 100M-key tree (one partition = the whole
range), then per-kernel times (HIP events on the library's stream,
st_kernel_stats) over K timed 1M-key batches (50 % overwrites, 50 % new), then the wall
time of K more such batches with no per-kernel events.
Usage: python tools/part_breakdown.py [tree_keys] [batches] [csr|downN]
(csr: pages off; downN: st_debug_knob ST_DBG_PAGE_DOWN = N)"""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from riak_ensemble_amd import synctree_hip  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 100_000_000
K = int(sys.argv[2]) if len(sys.argv) > 2 else 30
B = 1_000_000
dev = torch.device('cuda', 0)
t = synctree_hip.DeviceTree()
if len(sys.argv) > 3 and sys.argv[3] == 'csr':   # pages off: every batch merged into the CSR
    from riak_ensemble_amd import _lib  # noqa: E402
    t.debug_knob(_lib.ST_DBG_PAGES, -1)
if len(sys.argv) > 3 and sys.argv[3].startswith('down'):   # which in-place merges shift down (pages.h)
    from riak_ensemble_amd import _lib  # noqa: E402
    t.debug_knob(_lib.ST_DBG_PAGE_DOWN, int(sys.argv[3][4:]))
seed = 0x5EED0005
for a in range(0, N, 10_000_000):
    m = min(10_000_000, N - a)
    k = bench._dev_keys(seed, a, m, dev, torch)
    v = bench._dev_values(torch.arange(a, a + m, dtype=torch.int64, device=dev), dev, torch)
    t.insert_int64_device(k.data_ptr(), v.data_ptr(), m, 17)
    del k, v
torch.cuda.synchronize()
rng = np.random.default_rng(5)
batches = []
for j in range(2 * K + 2):   # batches 0, 1 warm up (the second builds the pages), 2..K+1 timed with events, then K more without
    old = torch.from_numpy(rng.integers(0, N, B // 2)).to(dev)
    k = torch.cat([bench._dev_keys_at(seed, old, dev, torch), bench._dev_keys(seed, N + j * B, B - B // 2, dev, torch)])
    seq = torch.cat([old + 1, torch.arange(N + j * B, N + j * B + (B - B // 2), device=dev)])
    batches.append((k.contiguous(), bench._dev_values(seq, dev, torch).contiguous()))
torch.cuda.synchronize()
for k, v in batches[:2]:
    t.insert_int64_device(k.data_ptr(), v.data_ptr(), B, 17)
torch.cuda.synchronize()
names = ['key_segment', 'bucket', 'run_sort', 'mark_paths', 'segment_verify', 'verify_pos', 'level_verify',
         'path_status', 'key_status', 'merge_count', 'merge_write', 'merge_touched', 'mark_dirty', 'seg_perm',
         'segment_hash', 'level_rehash', 'pack_int64', 'page_build', 'page_plan', 'page_place', 'page_merge', 'page_fold']
t.set_timing(True)
t.kernel_stats('*reset*')
t0 = time.perf_counter()
for j in range(2, K + 2):
    k, v = batches[j]
    t.insert_int64_device(k.data_ptr(), v.data_ptr(), B, 17)
torch.cuda.synchronize()
el = (time.perf_counter() - t0) / K * 1e3
tot = 0.0
for nm in names:
    n, ms = t.kernel_stats(nm)
    if n:
        tot += ms
        print('%-16s %4d launches %9.3f ms/batch' % (nm, n // K, ms / K))
print('named kernels %.3f ms/batch, wall %.3f ms/batch (timing on)' % (tot / K, el))
t.set_timing(False)
t0 = time.perf_counter()
for j in range(K + 2, 2 * K + 2):   # fresh batches (half new keys), as the timed ones
    k, v = batches[j]
    t.insert_int64_device(k.data_ptr(), v.data_ptr(), B, 17)
torch.cuda.synchronize()
print('wall %.3f ms/batch (timing off), entries %d, pages (on, batches, builds, folds, moved slots) %s' % ((time.perf_counter() - t0) / K * 1e3, t.num_entries(), t.page_stats()))
t.close()
