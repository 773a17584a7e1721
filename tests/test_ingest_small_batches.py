"""Regression test for the small-batch bulk ingest.

insert/3 batches of 1-16 keys merged through the BULK ingest (key -> segment,
radix sort, per-segment runs, merge count/scan/write into a new CSR, dirty-path
rehash; synctree.erl:189-209 applied per key in batch order) into a freshly
bulk-loaded 20,000-key tree of 2^20 segments -- the case that intermittently
dropped CSR entries in round 2.  The sequence mirrors tools/stress_small.py
(three geometries per seed, trees created and destroyed in turn, so the device
allocator recycles the previous trees' memory), and every step is checked
against the C restatement (oracle/, the checker only): the top hash after
every batch, a probe of gets, and at the end every key and every level.
"""
import numpy as np
import pytest

from riak_ensemble_amd import workload


def _vals(seqs):
    v = np.zeros((len(seqs), 17), np.uint8)
    v[:, 8] = 1                                             # Epoch = 1
    v[:, 9:17] = np.array(seqs, '>u8').view(np.uint8).reshape(-1, 8)
    return v


def _run(tn, W, S, steps, C, synctree_hip):
    n = 20000 if S >= 4096 else 3000
    keys = workload.keys_int63(n, workload.SEED ^ (0x51 + tn))
    vals = workload.obj_hash_values(n)
    dev = synctree_hip.DeviceTree(W, S)
    ora = C.OTree(W, S)
    try:
        assert dev.insert_int64(keys, vals) == 0
        ora.bulk_load_int64(keys, vals)
        assert dev.top_hash() == ora.top_hash(), 'seed %d geom %s: bulk load' % (tn, (W, S))
        rng = np.random.default_rng(tn)
        extra = workload.keys_int63(4000, workload.SEED ^ (0x52 + tn))
        seq = n
        model = {int(k) for k in keys}
        for step in range(steps):
            m = int(rng.integers(1, 17))
            ks = [int(keys[rng.integers(0, n)]) if rng.random() < 0.5 else int(extra[rng.integers(0, len(extra))])
                  for _ in range(m)]
            seqs = list(range(seq + 1, seq + m + 1))
            seq += m
            vs = _vals(seqs)
            # the bulk path for every batch size (st_insert_int64 never takes the per-key kernel)
            assert dev.insert_int64(np.array(ks, np.int64), vs) == 0
            for k, v in zip(ks, vs):
                ora.insert(k, bytes(v))
                model.add(k)
            where = 'seed %d geom %s step %d (%d keys)' % (tn, (W, S), step, m)
            assert dev.top_hash() == ora.top_hash(), where
            probe = [ks[0], int(keys[rng.integers(0, n)]), int(extra[rng.integers(0, len(extra))])]
            assert dev.get_batch(probe) == [ora.get(k) for k in probe], where
            if step % 30 == 29:
                if step % 60 == 29:
                    dev.rehash()
                else:
                    assert dev.verify(), where
                assert dev.num_entries() == ora.num_entries(), where
        allk = sorted(model)
        assert dev.get_batch(allk) == [ora.get(k) for k in allk], 'seed %d geom %s: final keys' % (tn, (W, S))
        for lvl in range(1, ora.height + 2):
            pa, ha = dev.level_entries(lvl)
            pb, hb = ora.level_entries(lvl)
            assert (pa == pb).all() and (ha == hb).all(), 'seed %d geom %s: level %d' % (tn, (W, S), lvl)
        assert dev.verify()
    finally:
        dev.close()


@pytest.mark.gpu
def test_small_batches_bulk_ingest_into_large_tree():
    import oracle_c as C
    from riak_ensemble_amd import synctree_hip
    for tn in range(4):
        for W, S in [(16, 1 << 20), (4, 4096), (16, 16)]:
            _run(tn, W, S, 60, C, synctree_hip)
