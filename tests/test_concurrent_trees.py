"""Different tree handles used at the same time from different threads
(SURVEY §8b threading contract: one gen_server per tree, many trees running
concurrently -- src/riak_ensemble_peer_tree.erl:58-59; the NIF runs them on
dirty schedulers).  Every thread owns two device trees and drives bulk and
per-key inserts, gets, rehash, verify and compare on them while the other
threads do the same; each thread checks its trees against its own C
restatement (oracle/, the checker only).  ctypes releases the GIL, so the
library calls of the threads overlap, including the device-memory cache they
share."""
import threading

import numpy as np
import pytest

from riak_ensemble_amd import workload


def _vals(seqs):
    v = np.zeros((len(seqs), 17), np.uint8)
    v[:, 8] = 1
    v[:, 9:17] = np.array(seqs, '>u8').view(np.uint8).reshape(-1, 8)
    return v


def _worker(tid, rounds, C, synctree_hip, errors):
    try:
        geom = [(16, 1 << 20), (16, 1 << 16), (4, 4096)][tid % 3]
        W, S = geom
        rng = np.random.default_rng(100 + tid)
        n = 30000 if S >= 1 << 16 else 3000
        keys = workload.keys_int63(n, workload.SEED ^ (0x700 + tid))
        vals = workload.obj_hash_values(n)
        for r in range(rounds):
            a, b = synctree_hip.DeviceTree(W, S), synctree_hip.DeviceTree(W, S)
            oa, ob = C.OTree(W, S), C.OTree(W, S)
            try:
                assert a.insert_int64(keys, vals) == 0 and b.insert_int64(keys, vals) == 0
                oa.bulk_load_int64(keys, vals)
                ob.bulk_load_int64(keys, vals)
                seq = n
                for step in range(20):
                    m = int(rng.integers(1, 40))
                    ks = [int(keys[i]) for i in rng.integers(0, n, m)]
                    vs = _vals(list(range(seq, seq + m)))
                    seq += m
                    tgt, otgt = (a, oa) if step % 2 else (b, ob)
                    if m <= 16:
                        st = tgt.insert_batch(ks, [bytes(v) for v in vs])
                        assert all(x is None for x in st), st
                    else:
                        assert tgt.insert_int64(np.array(ks, np.int64), vs) == 0
                    for k, v in zip(ks, vs):
                        otgt.insert(k, bytes(v))
                    probe = ks[:3]
                    assert tgt.get_batch(probe) == [otgt.get(k) for k in probe]
                    if step % 7 == 6:
                        tgt.rehash()
                        assert tgt.verify()
                    assert tgt.top_hash() == otgt.top_hash(), (tid, r, step)
                got = a.compare(b)
                assert got[0] == 'ok'
                exp = oa.compare(ob)
                assert [(k, v) for _, k, v in got[1]] == exp, (tid, r)
            finally:
                a.close()
                b.close()
    except Exception as e:   # reported by the main thread
        errors.append((tid, repr(e)))


@pytest.mark.gpu
def test_trees_driven_from_concurrent_threads():
    import oracle_c as C
    from riak_ensemble_amd import synctree_hip
    errors = []
    ths = [threading.Thread(target=_worker, args=(i, 3, C, synctree_hip, errors)) for i in range(4)]
    for th in ths:
        th.start()
    for th in ths:
        th.join()
    assert not errors, errors
