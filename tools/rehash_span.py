"""Fused rehash time on a 10M-key tree: GPU span of K back-to-back launches
on the tree's stream (two events, none per launch), min of R rounds.
Usage: python tools/rehash_span.py [keys] [K] [R]"""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from riak_ensemble_amd import synctree_hip, workload
n = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
K = int(sys.argv[2]) if len(sys.argv) > 2 else 200
R = int(sys.argv[3]) if len(sys.argv) > 3 else 5
k = torch.from_numpy(workload.keys_int63(n)).cuda()
v = torch.from_numpy(workload.obj_hash_values(n)).cuda()
torch.cuda.synchronize()
t = synctree_hip.DeviceTree()
t.insert_int64_device(k.data_ptr(), v.data_ptr(), n, 17)
for _ in range(3):
    t.rehash()
t.sync()
s = torch.cuda.Stream()
t.set_stream(s.cuda_stream)
res = []
for r in range(R):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(K):
        t.rehash()
    e1.record(s)
    e1.synchronize()
    res.append(e0.elapsed_time(e1) / K * 1e3)
t.set_stream(0)
print('rehash span us/launch: min %.2f all %s (lib %s)' % (min(res), [round(x, 2) for x in res], os.environ.get('ST_LIB', 'default')))
