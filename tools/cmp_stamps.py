"""GPU box diagnostic: config-3 compare (10M keys, every 1000th non-empty
segment differs) with the compare walk's per-wave phase stamps
(ST_CMP_STAMPS=1) and the kernel times."""
import os
import sys
import time

os.environ.setdefault('ST_CMP_STAMPS', '1')
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
from riak_ensemble_amd import synctree_hip, workload

n = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
step = int(sys.argv[2]) if len(sys.argv) > 2 else 1000
keys_d = torch.from_numpy(workload.keys_int63(n, workload.SEED)).cuda()
vals_d = torch.from_numpy(workload.obj_hash_values(n)).cuda()
a = synctree_hip.DeviceTree()
a.insert_int64_device(keys_d.data_ptr(), vals_d.data_ptr(), n, 17)
b = synctree_hip.DeviceTree()
b.insert_int64_device(keys_d.data_ptr(), vals_d.data_ptr(), n, 17)
pres, _ = a.level_entries(a.height + 1)
segs = np.nonzero(pres)[0][::step].tolist()
imgs = a.exchange_get_batch(a.height + 1, segs)
mut = [(img[0][0], bytes([(img[0][1][0] + 1) % 256]) + img[0][1][1:]) for img in imgs]
for i in range(0, len(mut), 4096):
    b.insert_batch([k for k, _ in mut[i:i + 4096]], [v for _, v in mut[i:i + 4096]])
for _ in range(3):
    nd = a.compare_device(b)
print('diffs', nd, 'expected', len(segs), flush=True)
a.set_timing(True)
a.kernel_stats('*reset*')
reps = 20
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(reps):
    a.compare_device(b)
torch.cuda.synchronize()
print('ms/compare %.4f' % ((time.perf_counter() - t0) / reps * 1e3),
      {k: round(a.kernel_stats(k)[1] / reps, 4) for k in ('cmp_walk',)}, flush=True)
print('visited', a.compare_stats())
