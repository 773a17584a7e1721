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


def _inserter(b, keys, vals, errors, started, done):
    """B's owner: inserts keys into B one call at a time (the per-key path,
    into B's overlay) and in 20-key batches (the bulk path: a CSR merge that
    frees and replaces B's device buffers)."""
    import time
    try:
        started.wait(30)
        i = 0
        while i < len(keys):
            time.sleep(0.0005)
            if (i // 10) % 3 == 2 and i + 20 <= len(keys):
                assert b.insert_int64(keys[i:i + 20], vals[i:i + 20]) == 0
                i += 20
            else:
                assert b.insert1(int(keys[i]), bytes(vals[i])) is None
                i += 1
    except Exception as e:
        errors.append(('inserter', repr(e)))
    finally:
        done.set()


@pytest.mark.gpu
def test_exchange_reads_remote_under_its_lock_while_owner_inserts():
    """The exchange process reads the REMOTE tree while the remote's owner
    keeps inserting into it (riak_ensemble_exchange.erl:72-81 reads it only
    through the remote peer_tree, peer_tree.erl:58-59,155-157): st_compare /
    st_exchange_plan(A, B) take B's owner lock, so every result equals the
    reference compare of A against B as it stood between two of the owner's
    inserts -- never a torn state, never a fault."""
    import oracle_c as C
    from riak_ensemble_amd import synctree_hip
    N, M, T = 100_000, 160, 40
    keys = workload.keys_int63(N, workload.SEED ^ 0x1CE)
    vals = workload.obj_hash_values(N)
    bumped = vals.copy()
    idx_b = np.arange(0, N - M, 997)
    idx_b = idx_b[vals[idx_b, 16] < 255][:T]            # T keys B holds with Seq + 1 (valid_obj_hash takes them)
    bumped[idx_b, 16] += 1
    a, b = synctree_hip.DeviceTree(), synctree_hip.DeviceTree()
    assert a.insert_int64(keys, vals) == 0
    assert b.insert_int64(keys[:N - M], bumped[:N - M]) == 0
    oa = C.OTree().bulk_load_int64(keys, vals)
    ob = C.OTree().bulk_load_int64(keys[:N - M], bumped[:N - M])
    exp0 = oa.compare(ob)                                # B before any of the owner's inserts
    assert len(exp0) == T + M
    late = [int(k) for k in keys[N - M:]]
    pos = {k: i for i, k in enumerate(late)}

    def expected(i):                                     # B after the owner's first i inserts
        gone = set(late[:i])
        return [d for d in exp0 if d[0] not in gone]

    errors, started, done = [], threading.Event(), threading.Event()
    th = threading.Thread(target=_inserter, args=(b, keys[N - M:], vals[N - M:], errors, started, done))
    seen = []
    th.start()
    try:
        it = 0
        while not done.is_set() or it < 4:
            if it % 2 == 0:
                got = a.compare(b)
                assert got[0] == 'ok', got[:2]
                lst = [(k, v) for _, k, v in got[1]]
                remaining = [k for k, (va, vb) in lst if vb == '$none']
                i = M - len(remaining)
                assert lst == expected(i), 'compare saw a state of B that never existed (i=%d)' % i
            else:
                st, info = a.exchange_plan(b)
                assert st == 'ok' and info['take'] == T, (st, info)
                i = M - (info['diffs'] - T)
                assert 0 <= i <= M
            seen.append(i)
            started.set()
            it += 1
    finally:
        th.join()
    assert not errors, errors
    assert seen == sorted(seen), 'B went back in time: %s' % seen[:50]
    assert seen[-1] == M and len(set(seen)) > 2, seen   # the reader overlapped the owner's inserts
    a.close()
    b.close()
