"""Profile helper: config-4 shape (E ensembles x N keys) group rehash."""
import sys
import os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from riak_ensemble_amd import synctree_hip, workload

E = int(sys.argv[1]) if len(sys.argv) > 1 else 32
N = int(sys.argv[2]) if len(sys.argv) > 2 else 1_000_000
trees = []
for e in range(E):
    k = torch.from_numpy(workload.keys_int63(N, workload.SEED ^ (e + 1))).cuda()
    v = torch.from_numpy(workload.obj_hash_values(N)).cuda()
    t = synctree_hip.DeviceTree()
    t.insert_int64_device(k.data_ptr(), v.data_ptr(), N, 17)
    trees.append(t)
torch.cuda.synchronize()
for _ in range(5):
    synctree_hip.rehash_group(trees)
torch.cuda.synchronize()
print('ok')
