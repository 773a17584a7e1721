"""The repair path (riak_ensemble_peer_tree do_repair, peer_tree.erl:264-277)
and the first rehash after an insert batch on a 10M-key tree, by phase:
wall time of each C-ABI call (delete_node / insert / rehash) and the kernels
each one launched (HIP events on the library stream).
Usage: python tools/repair_breakdown.py [keys] [reps]"""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from riak_ensemble_amd import synctree_hip, workload  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
R = int(sys.argv[2]) if len(sys.argv) > 2 else 10
NAMES = ['bucket', 'clamp_runs', 'key_segment', 'key_status', 'level_rehash', 'level_verify', 'mark_dirty',
         'mark_paths', 'merge_count', 'merge_write', 'ov_flush', 'page_build', 'page_fold', 'page_merge', 'page_plan',
         'path_status', 'rehash_fused', 'run_sort', 'seg_perm', 'segment_hash', 'segment_verify', 'small',
         'tile_build', 'verify_pos']
keys = workload.keys_int63(N, workload.SEED)
vals = workload.obj_hash_values(N)
kd = torch.from_numpy(keys).cuda()
vd = torch.from_numpy(vals).cuda()
torch.cuda.synchronize()
t = synctree_hip.DeviceTree()
t.insert_int64_device(kd.data_ptr(), vd.data_ptr(), N, 17)
t.rehash()
t.sync()
H1 = t.height + 1
segs = t.segments_of([int(k) for k in keys[:(R + 2) * 7:7]])


def phases(label, calls):
    """calls: [(name, fn)]; R reps: median wall per call, then one timed rep."""
    walls = {nm: [] for nm, _ in calls}
    for r in range(R):
        torch.cuda.synchronize()
        for nm, fn in calls:
            t0 = time.perf_counter()
            fn(r)
            t.sync()
            walls[nm].append(time.perf_counter() - t0)
    t.set_timing(True)
    t.kernel_stats('*reset*')
    for nm, fn in calls:
        fn(R)
    t.sync()
    ks = {}
    for k in NAMES:
        n, ms = t.kernel_stats(k)
        if n:
            ks[k] = (n, ms)
    t.set_timing(False)
    tot = 0.0
    for nm, _ in calls:
        w = sorted(walls[nm])
        med = w[len(w) // 2] * 1e3
        tot += med
        print('%-10s %-12s median %.3f ms (min %.3f)' % (label, nm, med, w[0] * 1e3))
    print('%-10s total        %.3f ms' % (label, tot))
    for k, (n, ms) in ks.items():
        print('%-10s   kernel %-16s %3d launches %.3f ms' % (label, k, n, ms))


phases('repair', [('delete_node', lambda r: t.delete_node(H1, segs[r])), ('rehash', lambda r: t.rehash())])
rng = np.random.default_rng(7)
small = [([int(x) for x in rng.integers(0, 1 << 62, 1000)], [b'\x00' * 17] * 1000) for _ in range(R + 1)]
phases('mut1000', [('insert', lambda r: t.insert_batch(*small[r])), ('rehash', lambda r: t.rehash())])
big = []
for r in range(R + 1):
    k = torch.from_numpy(rng.integers(0, 1 << 62, 100_000)).cuda()
    big.append((k, torch.zeros((100_000, 17), dtype=torch.uint8, device='cuda')))
torch.cuda.synchronize()
phases('mut100k', [('insert', lambda r: t.insert_int64_device(big[r][0].data_ptr(), big[r][1].data_ptr(), 100_000, 17)),
                   ('rehash', lambda r: t.rehash())])
t.close()
