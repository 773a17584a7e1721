"""Per-key get/2 and insert/3 latency through the single-key C-ABI calls
(st_get1 / st_insert1) on a 100k-key device tree, checked against the C
restatement; median / p90 / mean over N calls and the k_small kernel alone
(HIP events).  Usage: python tools/perkey_lat.py [N]"""
import os
import sys
import time

import numpy as np

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, R)
sys.path.insert(0, os.path.join(R, 'oracle'))
import oracle_c as C  # noqa: E402
from riak_ensemble_amd import synctree_hip, workload  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 2000
n = 100_000
keys = workload.keys_int63(n, workload.SEED ^ 0x100)
vals = workload.obj_hash_values(n)
t = synctree_hip.DeviceTree()
t.insert_int64(keys, vals)
t.rehash()
ora = C.OTree()
ora.bulk_load_int64(keys, vals)
rng = np.random.default_rng(5)
kl = [int(keys[i]) for i in rng.integers(0, n, N)]
t.get1(kl[0])
res = {}
for what in ('get', 'insert'):
    lat = []
    for i, k in enumerate(kl):
        v = (i + 1).to_bytes(17, 'big')
        t0 = time.perf_counter()
        r = t.get1(k) if what == 'get' else t.insert1(k, v)
        lat.append(time.perf_counter() - t0)
        if what == 'get':
            assert r == ora.get(k), (i, r, ora.get(k))
        else:
            assert r is None, r
            ora.insert(k, v)
    lat = np.array(lat) * 1e6
    res[what] = (np.median(lat), np.percentile(lat, 90), lat.mean())
    print('%-6s median %.1f  p90 %.1f  mean %.1f us/call (%d calls)' % (what, *res[what], N), flush=True)
assert t.top_hash() == ora.top_hash()
for what in ('get', 'insert'):
    t.set_timing(True)
    t.kernel_stats('*reset*')
    for i, k in enumerate(kl[:200]):
        t.get1(k) if what == 'get' else t.insert1(k, (i + 7).to_bytes(17, 'big'))
    launches, ms = t.kernel_stats('small')
    t.set_timing(False)
    print('%-6s k_small kernel %.1f us (HIP events, %d launches)' % (what, ms / max(launches, 1) * 1e3, launches))
t.close()
print('RESULT ok')
