"""int64 batches with long and short runs of one segment:
st_insert_int64 sorts a segment's run of <= 4 keys in registers (a sorting
network on (key, batch index)) and longer runs in memory; either way the last
writer of a key wins (synctree.erl:189-209 applied per key in batch order).
Small segment counts make runs long; keys repeat inside a batch and include
the int64 extremes (the sign-flipped big-endian order).  Every batch goes
through the bulk ingest -- into the CSR first, then through the pages once the
tree is 32 x the batch -- and is checked against the C restatement (oracle/,
the checker only): top hash, every key's value, every level.
"""
import numpy as np
import pytest

from riak_ensemble_amd import workload


def _vals(seqs):
    v = np.zeros((len(seqs), 17), np.uint8)
    v[:, 8] = 1
    v[:, 9:17] = np.array(seqs, '>u8').view(np.uint8).reshape(-1, 8)
    return v


def _skewed(n, rng):
    """95 % of the keys small, 5 % near 2^62: inside a segment the first and
    last keys span the outliers, so the positions' interpolation guesses far
    off and its bisection finishes from either side of the window."""
    small = rng.choice(10_000_000, n - n // 20, replace=False).astype(np.int64)
    big = (np.int64(1) << 62) + rng.choice(1 << 40, n // 20, replace=False).astype(np.int64)
    return np.concatenate([small, big])


@pytest.mark.gpu
@pytest.mark.parametrize('W,S,n0,batch,skew', [(16, 256, 20000, 600, False), (4, 64, 4000, 120, False),
                                               (16, 16, 2000, 60, False), (16, 256, 20000, 600, True)])
def test_int64_runs_last_writer_wins(W, S, n0, batch, skew):
    import oracle_c as C
    from riak_ensemble_amd import synctree_hip
    rng = np.random.default_rng(S)
    if skew:
        base = _skewed(n0, rng)
    else:
        base = workload.keys_int63(n0, workload.SEED ^ (0x77 + S)).astype(np.int64)
    base[:4] = [np.iinfo(np.int64).min, np.iinfo(np.int64).max, -1, 0]
    pool = np.concatenate([base, -base[4:200]])                 # negative keys too
    dev = synctree_hip.DeviceTree(W, S)
    ora = C.OTree(W, S)
    try:
        seq = 0
        vals = _vals(range(1, n0 + 1))
        assert dev.insert_int64(base, vals) == 0
        ora.bulk_load_int64(base, vals)
        seq = n0
        model = {int(k) for k in base}
        for step in range(12):
            # a few hot keys repeated many times (runs longer than 4) and a spread of others
            hot = pool[rng.integers(0, len(pool), 3)]
            ks = np.concatenate([np.repeat(hot, rng.integers(2, 9, 3)),
                                 pool[rng.integers(0, len(pool), batch - 40)]]).astype(np.int64)
            ks = ks[rng.permutation(len(ks))]
            seqs = range(seq + 1, seq + len(ks) + 1)
            seq += len(ks)
            vs = _vals(seqs)
            assert dev.insert_int64(ks, vs) == 0
            for k, v in zip(ks, vs):
                ora.insert(int(k), bytes(v))
                model.add(int(k))
            assert dev.top_hash() == ora.top_hash(), 'step %d' % step
        allk = sorted(model)
        assert dev.num_entries() == ora.num_entries()
        assert dev.get_batch(allk) == [ora.get(k) for k in allk]
        for lvl in range(1, ora.height + 2):
            pa, ha = dev.level_entries(lvl)
            pb, hb = ora.level_entries(lvl)
            assert (pa == pb).all() and (ha == hb).all(), 'level %d' % lvl
        assert dev.page_stats()[1] > 0, 'no batch went through the pages'
    finally:
        dev.close()
