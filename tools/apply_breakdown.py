"""Config-3 exchange apply by kernel: A and B2 = A with 1,000+ keys' Seq
advanced (as bench.py's compare leg), a fresh copy of A applies B2's newer
values (st_exchange_apply: compare + select + one batched insert/3); per-kernel
HIP-event times of the apply, its wall time, and the same for a second apply
after the first (nothing left to take).  Usage: python tools/apply_breakdown.py"""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from riak_ensemble_amd import synctree_hip  # noqa: E402

N = 10_000_000
dev = torch.device('cuda', 0)
keys_d = bench._dev_keys(0x5EED0001, 0, N, dev, torch)
vals_d = bench._dev_values(torch.arange(N, dtype=torch.int64, device=dev), dev, torch)
a = synctree_hip.DeviceTree()
a.insert_int64_device(keys_d.data_ptr(), vals_d.data_ptr(), N, 17)
pres, _ = a.level_entries(6)
segs = np.nonzero(pres)[0][::1000].tolist()
imgs = a.exchange_get_batch(6, segs)
mut2 = [(k, v[:-1] + bytes([v[-1] + 1])) for k, v in ((img[0][0], img[0][1]) for img in imgs) if v[-1] < 255]
b2 = synctree_hip.DeviceTree()
b2.insert_int64_device(keys_d.data_ptr(), vals_d.data_ptr(), N, 17)
b2.insert_batch([k for k, _ in mut2], [v for _, v in mut2])
names = ['cmp_walk', 'diff_apply', 'seg_voff', 'tile_build', 'clamp_runs', 'key_segment', 'bucket', 'run_sort', 'mark_paths', 'segment_verify', 'level_verify',
         'path_status', 'key_status', 'merge_count', 'merge_write', 'merge_touched', 'mark_dirty', 'seg_perm',
         'segment_hash', 'level_rehash', 'pack_int64', 'page_build', 'page_plan', 'page_place', 'page_merge']
for rep in range(3):
    ta = synctree_hip.DeviceTree()
    ta.insert_int64_device(keys_d.data_ptr(), vals_d.data_ptr(), N, 17)
    assert ta.exchange_plan(b2)[0] == 'ok'
    torch.cuda.synchronize()
    ta.set_timing(True)
    ta.kernel_stats('*reset*')
    t0 = time.perf_counter()
    r = ta.exchange_apply(b2)
    torch.cuda.synchronize()
    el = (time.perf_counter() - t0) * 1e3
    assert r[0] == 'ok' and ta.top_hash() == b2.top_hash(), r
    tot = 0.0
    print('apply %d: wall %.3f ms (timing on), %d keys taken' % (rep, el, r[1]['applied']))
    for nm in names:
        c, ms = ta.kernel_stats(nm)
        if c:
            tot += ms
            print('  %-16s %3d launches %8.3f ms' % (nm, c, ms))
    print('  named kernels %.3f ms' % tot)
    ta.close()
