"""Debug: K1 variant vs oracle on small trees (full and dirty rehash)."""
import os
import sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..'))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', 'oracle'))
import numpy as np
import oracle_c as C
from riak_ensemble_amd import synctree_hip

def cmp(dt, ot, tag):
    pa, ha = dt.level_entries(6)
    pb, hb = ot.level_entries(6)
    bad = np.nonzero((pa != pb) | (ha != hb).any(axis=1))[0]
    print(tag, 'mismatching segments:', len(bad), bad[:10].tolist())
    for s in bad[:5].tolist():
        node = ot.node(6, s)
        print('   seg', s, 'n', len(node), 'bytes', sum(len(v) for _, v in node), 'dev present', pa[s], 'orc present', pb[s])

keys = list(range(1, 101))
vals = [(k * 10).to_bytes(8, 'big') for k in keys]
ot = C.OTree()
for k, v in zip(keys, vals):
    ot.insert(k, v)
dt = synctree_hip.DeviceTree()
for k, v in zip(keys, vals):
    dt.insert_batch([k], [v])
cmp(dt, ot, 'per-key inserts')
dt2 = synctree_hip.DeviceTree()
dt2.insert_batch(keys, vals)
cmp(dt2, ot, 'one batch')
dt2.rehash()
cmp(dt2, ot, 'batch+full rehash')
dt.rehash()
cmp(dt, ot, 'per-key + full rehash')
