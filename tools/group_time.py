"""Config-4 group rehash time (E trees x N keys, keys generated on the device
as bench.py does): ms per st_rehash_group by HIP events and by wall clock.
Usage: python tools/group_time.py [E] [N] [reps]"""
import os
import sys
import time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import bench
from riak_ensemble_amd import synctree_hip, workload

E = int(sys.argv[1]) if len(sys.argv) > 1 else 512
N = int(sys.argv[2]) if len(sys.argv) > 2 else 1_000_000
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 5
dev = torch.device('cuda', 0)
vals = bench._dev_values(torch.arange(N, dtype=torch.int64, device=dev), dev, torch)
trees = []
for e in range(E):
    k = bench._dev_keys(workload.SEED ^ (e + 1), 0, N, dev, torch)
    t = synctree_hip.DeviceTree()
    t.insert_int64_device(k.data_ptr(), vals.data_ptr(), N, 17)
    trees.append(t)
torch.cuda.synchronize()
synctree_hip.rehash_group(trees)
top = [t.top_hash() for t in trees[:4]]
trees[0].set_timing(True)
trees[0].kernel_stats('*reset*')
t0 = time.perf_counter()
for _ in range(reps):
    synctree_hip.rehash_group(trees)
torch.cuda.synchronize()
wall = (time.perf_counter() - t0) / reps * 1e3
n, ms = trees[0].kernel_stats('rehash_group')
assert [t.top_hash() for t in trees[:4]] == top
print('group %d x %d: kernel %.3f ms, wall %.3f ms per rehash' % (E, N, ms / max(n, 1), wall), flush=True)
