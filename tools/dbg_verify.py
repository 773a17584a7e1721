"""Replays stress_small trial 0 geometry (16, 2^20) without extra trees and
verifies after every step; prints the first step whose insert batch leaves
the device tree inconsistent (diagnostic)."""
import os, sys
import numpy as np
R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, R)
sys.path.insert(0, os.path.join(R, 'oracle'))
import oracle_c as C
from riak_ensemble_amd import synctree_hip, workload


def _val(seq):
    return bytes([0]) + (1).to_bytes(8, 'big') + seq.to_bytes(8, 'big')


tn, W, S = 0, 16, 1 << 20
n = 20000
keys = workload.keys_int63(n, workload.SEED ^ (0x51 + tn))
vals = workload.obj_hash_values(n)
dev = synctree_hip.DeviceTree(W, S)
ora = C.OTree(W, S)
dev.insert_int64(keys, vals)
ora.bulk_load_int64(keys, vals)
rng = np.random.default_rng(tn)
extra = workload.keys_int63(4000, workload.SEED ^ (0x52 + tn))
seq = n
for step in range(120):
    m = int(rng.integers(1, 17))
    ks, vs = [], []
    for _ in range(m):
        k = int(keys[rng.integers(0, n)]) if rng.random() < 0.5 else int(extra[rng.integers(0, len(extra))])
        seq += 1
        ks.append(k)
        vs.append(_val(seq))
    st = dev.insert_batch(ks, vs)
    for k, v in zip(ks, vs):
        ora.insert(k, v)
    topok = dev.top_hash() == ora.top_hash()
    probe = [ks[0], int(keys[rng.integers(0, n)]), int(extra[rng.integers(0, len(extra))])]
    g = dev.get_batch(probe)
    vok = dev.verify()
    print('step', step, 'm', len(ks), 'st_ok', all(x is None for x in st), 'top', topok, 'verify', vok,
          'get', g == [ora.get(k) for k in probe], flush=True)
    if not vok or not topok:
        segs = [ora.segment_of(k) for k in ks]
        print('  segments', segs, 'dup keys', len(set(ks)) != len(ks), flush=True)
        for lvl in range(1, ora.height + 2):
            pa, ha = dev.level_entries(lvl)
            pb, hb = ora.level_entries(lvl)
            d = np.nonzero((pa != pb) | np.any(ha != hb, axis=1))[0]
            print('  level', lvl, 'differing buckets', d[:10], flush=True)
        break
    if step % 30 == 29:
        if step % 60 == 29:
            dev.rehash()
