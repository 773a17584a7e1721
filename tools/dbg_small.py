import sys, os
sys.path.insert(0, '/root/repo'); sys.path.insert(0, '/root/repo/oracle')
import numpy as np
import oracle_c as C
from riak_ensemble_amd import synctree_hip, workload
def _val(seq, epoch=1):
    return bytes([0]) + epoch.to_bytes(8, 'big') + seq.to_bytes(8, 'big')
W, S = 16, 1 << 20
n = 20000
keys = workload.keys_int63(n, workload.SEED ^ 0x51)
vals = workload.obj_hash_values(n)
dev = synctree_hip.DeviceTree(W, S)
ora = C.OTree(W, S)
dev.insert_int64(keys, vals); ora.bulk_load_int64(keys, vals)
rng = np.random.default_rng(7)
extra = workload.keys_int63(4000, workload.SEED ^ 0x52)
seq = n
for step in range(120):
    m = int(rng.integers(1, 17))
    ks, vs = [], []
    for _ in range(m):
        k = int(keys[rng.integers(0, n)]) if rng.random() < 0.5 else int(extra[rng.integers(0, len(extra))])
        seq += 1; ks.append(k); vs.append(_val(seq))
    if rng.random() < 0.2:
        ks.append(ks[0]); seq += 1; vs.append(_val(seq)); ks, vs = ks[-16:], vs[-16:]
    before_top = dev.top_hash()
    st = dev.insert_batch(ks, vs)
    for k, v in zip(ks, vs): ora.insert(k, v)
    if not all(x is None for x in st):
        print('step', step, 'n', len(ks), 'st', st, 'segs', [ora.segment_of(k) for k in ks], flush=True)
        print('dev top', dev.top_hash().hex(), 'ora top', ora.top_hash().hex(), flush=True)
        break
    if dev.top_hash() != ora.top_hash():
        print('top mismatch at step', step, 'n', len(ks), flush=True); break
    probe = [ks[0], int(keys[rng.integers(0, n)]), int(extra[rng.integers(0, len(extra))])]
    g = dev.get_batch(probe); e = [ora.get(k) for k in probe]
    if g != e: print('get mismatch', step, g, e, flush=True); break
    if step % 30 == 29:
        if step % 60 == 29: dev.rehash()
        else: assert dev.verify()
print('done', step)
