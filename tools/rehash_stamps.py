"""Phase stamps of the fused rehash kernel (run with ST_LEVEL_STAMPS=1)."""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from riak_ensemble_amd import synctree_hip, workload
n = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
k = torch.from_numpy(workload.keys_int63(n)).cuda()
v = torch.from_numpy(workload.obj_hash_values(n)).cuda()
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 4
torch.cuda.synchronize()
t = synctree_hip.DeviceTree()
t.insert_int64_device(k.data_ptr(), v.data_ptr(), n, 17)
for i in range(reps):   # the first hashes from the segments (no tiles yet), the rest run the fused kernel
    print('--- rehash', i, file=sys.stderr, flush=True)
    t.rehash()
    t.sync()
