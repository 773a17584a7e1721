"""Replays test_small_inserts_and_gets_interleaved[(4, 4096)] and prints the
first divergence (diagnostic)."""
import os, sys
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'oracle'))
import oracle_c as C
from riak_ensemble_amd import synctree_hip, workload


def _val(seq, epoch=1):
    return bytes([0]) + epoch.to_bytes(8, 'big') + seq.to_bytes(8, 'big')


for rep in range(3):
    W, S = 4, 4096
    n = 20000
    keys = workload.keys_int63(n, workload.SEED ^ 0x51)
    vals = workload.obj_hash_values(n)
    dev = synctree_hip.DeviceTree(W, S)
    ora = C.OTree(W, S)
    assert dev.insert_int64(keys, vals) == 0
    ora.bulk_load_int64(keys, vals)
    print('rep', rep, 'top ok', dev.top_hash() == ora.top_hash(), 'verify', dev.verify(), flush=True)
    rng = np.random.default_rng(7)
    extra = workload.keys_int63(4000, workload.SEED ^ 0x52)
    seq = n
    bad = False
    for step in range(120):
        m = int(rng.integers(1, 17))
        ks, vs = [], []
        for _ in range(m):
            if rng.random() < 0.5:
                k = int(keys[rng.integers(0, n)])
            else:
                k = int(extra[rng.integers(0, len(extra))])
            seq += 1
            ks.append(k)
            vs.append(_val(seq))
        if rng.random() < 0.2:
            ks.append(ks[0])
            seq += 1
            vs.append(_val(seq))
            ks, vs = ks[-16:], vs[-16:]
        vb = dev.verify()
        st = dev.insert_batch(ks, vs)
        if not all(x is None for x in st):
            print('step', step, 'n', len(ks), 'verify-before', vb, 'st', st, 'verify-after', dev.verify(), flush=True)
            print('segments', [ora.segment_of(k) for k in ks], flush=True)
            bad = True
            break
        for k, v in zip(ks, vs):
            ora.insert(k, v)
        if dev.top_hash() != ora.top_hash():
            print('top differs at step', step, flush=True)
            bad = True
            break
        probe = [ks[0], int(keys[rng.integers(0, n)]), int(extra[rng.integers(0, len(extra))])]
        if dev.get_batch(probe) != [ora.get(k) for k in probe]:
            print('get differs at step', step, flush=True)
        if step % 30 == 29:
            if step % 60 == 29:
                dev.rehash()
                print('rehash at', step, 'top ok', dev.top_hash() == ora.top_hash(), flush=True)
            else:
                print('verify at', step, dev.verify(), flush=True)
    print('rep', rep, 'bad' if bad else 'ok', flush=True)
    dev.close()
