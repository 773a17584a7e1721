"""Per-key insert/get latency on a 100k-key device tree;
run under rocprofv3 --kernel-trace --stats to see where a single call goes."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from riak_ensemble_amd import synctree_hip, workload  # noqa: E402

n = 100_000
keys = workload.keys_int63(n, workload.SEED ^ 0x100)
vals = workload.obj_hash_values(n)
t = synctree_hip.DeviceTree()
t.insert_int64(keys, vals)
t.rehash()
kl = [int(k) for k in keys[:50]]
for what in ('get', 'insert'):
    t0 = time.perf_counter()
    for k in kl:
        if what == 'get':
            t.get_batch([k])
        else:
            t.insert_batch([k], [b'\x00' * 17])
    print(what, round((time.perf_counter() - t0) / len(kl) * 1e6, 1), 'us/call', flush=True)
