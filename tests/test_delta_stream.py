"""Streaming insert batches through the delta CSR (SURVEY §8d
config 5): a batch much smaller than the tree merges into the delta, every
segment's content is the merged view of its base run and its delta run, and
the delta folds into the base past its limit.  Every batch is checked against
the C restatement of insert/3 (synctree.erl:189-209, sequential inserts, last
writer wins): top hash after every batch, every level's entries, entry
counts, and after folding the segments themselves (get, compare).  The fold
limit is lowered (st_debug_knob ST_DBG_DELTA_LIMIT) so the tests cross it
several times.  Needs an MI355X."""
import numpy as np
import pytest

import oracle_c as C
from riak_ensemble_amd import _lib, synctree_hip, workload

pytestmark = pytest.mark.gpu


def _levels(dev, ora):
    for lvl in range(1, dev.height + 2):
        pa, ha = dev.level_entries(lvl)
        pb, hb = ora.level_entries(lvl)
        assert (pa == pb).all(), 'presence differs at level %d' % lvl
        assert (ha[pa == 1] == hb[pb == 1]).all(), 'hashes differ at level %d' % lvl


def _obj(seqs, epoch=1):
    v = np.zeros((len(seqs), 17), np.uint8)
    v[:, 8] = epoch
    v[:, 9:17] = np.array(seqs, '>u8').view(np.uint8).reshape(-1, 8)
    return v


@pytest.mark.parametrize('segments,n0,batch,limit', [
    (1 << 16, 300_000, 4_000, 30_000),     # H = 4: folds every ~7 batches
    (1 << 20, 1_000_000, 20_000, 150_000),  # H = 5, the config-5 geometry at 1/100 scale
])
def test_int_keys_stream_through_delta(segments, n0, batch, limit):
    rng = np.random.default_rng(segments ^ n0)
    keys = workload.keys_int63(n0 + 40 * batch, workload.SEED ^ 0xDE17A)
    dev = synctree_hip.DeviceTree(16, segments)
    ora = C.OTree(16, segments)
    assert dev.insert_int64(keys[:n0], _obj(range(n0))) == 0
    ora.bulk_load_int64(keys[:n0], _obj(range(n0)))
    dev.debug_knob(_lib.ST_DBG_DELTA_LIMIT, limit)
    nxt = n0
    for b in range(30):
        old = rng.integers(0, nxt, batch // 2)                 # overwrites (Seq + 1), some repeated in the batch
        new = np.arange(nxt, nxt + batch - batch // 2)
        nxt += len(new)
        idx = rng.permutation(np.concatenate([old, new]))
        ks = keys[idx]
        vs = _obj(idx + 1 + b, epoch=2)
        assert dev.insert_int64(ks, vs) == 0
        assert ora.insert_int64_seq(ks, vs) == 0
        assert dev.top_hash() == ora.top_hash(), 'top hash differs after batch %d' % b
        assert dev.num_entries() == ora.num_entries(), b
        if b % 6 == 5:
            _levels(dev, ora)
    dl_n, dl_new, folds = dev.delta_stats()
    assert folds >= 2, (dl_n, dl_new, folds)               # the limit was crossed (and the delta refilled)
    assert dl_n > 0
    _levels(dev, ora)
    # reads fold the delta first: the segments themselves are the reference's
    probe = [int(k) for k in keys[rng.integers(0, nxt, 300)]]
    assert dev.get_batch(probe) == [ora.get(k) for k in probe]
    assert dev.delta_stats()[0] == 0
    assert dev.verify()
    dev.rehash()
    _levels(dev, ora)
    dev.close()


def _rand_bin(rng, lo, hi):
    return bytes(rng.integers(0, 256, int(rng.integers(lo, hi + 1)), dtype=np.uint8))


def test_variable_keys_and_values_through_delta():
    """Binary keys of 1..24 bytes and values of 0..40 bytes (empty values and
    values shorter than a 16-byte chunk: several merged-view pieces inside one
    chunk), with a delta limit crossed twice."""
    rng = np.random.default_rng(77)
    S = 4096
    dev, ora = synctree_hip.DeviceTree(16, S), C.OTree(16, S)
    base = {}
    while len(base) < 20_000:
        base[_rand_bin(rng, 1, 24)] = _rand_bin(rng, 0, 40)
    ks = list(base)
    st = dev.insert_batch(ks, [base[k] for k in ks])
    assert all(x is None for x in st)
    ora.bulk_load(ks, [base[k] for k in ks])
    dev.debug_knob(_lib.ST_DBG_DELTA_LIMIT, 1500)
    for b in range(12):
        bk = [ks[i] for i in rng.integers(0, len(ks), 300)] + [_rand_bin(rng, 1, 24) for _ in range(300)]
        bv = [_rand_bin(rng, 0, 40) for _ in bk]
        st = dev.insert_batch(bk, bv)
        assert all(x is None for x in st)
        for k, v in zip(bk, bv):
            ora.insert(k, v)
        ks.extend(bk[300:])
        assert dev.top_hash() == ora.top_hash(), 'top hash differs after batch %d' % b
        assert dev.num_entries() == ora.num_entries()
    assert dev.delta_stats()[2] >= 2
    _levels(dev, ora)
    probe = ks[::97]
    assert dev.get_batch(probe) == [ora.get(k) for k in probe]
    dev.close()


@pytest.mark.parametrize('delta', [True, False], ids=['delta', 'default_merge'])
def test_corrupted_segment_rejects_streamed_keys(delta):
    """A corrupted segment (corrupt/2, synctree.erl:241-247) met by a streamed
    batch: its keys are refused with {corrupted, Level, Bucket} and the rest
    are inserted, as sequential insert/3 calls would do.  With the delta
    enabled (ST_DBG_DELTA_LIMIT 0 = auto limit) the batch lands in the delta;
    with the default merge (delta off) nothing does."""
    S, n0 = 1 << 16, 200_000
    keys = workload.keys_int63(n0 + 5000, workload.SEED ^ 0xC0)
    vals = _obj(range(n0 + 5000))
    dev, ora = synctree_hip.DeviceTree(16, S), C.OTree(16, S)
    assert dev.insert_int64(keys[:n0], vals[:n0]) == 0
    ora.bulk_load_int64(keys[:n0], vals[:n0])
    if delta:
        dev.debug_knob(_lib.ST_DBG_DELTA_LIMIT, 0)
    # one streamed batch first (the delta holds entries), then corrupt a key's segment
    assert dev.insert_int64(keys[n0:n0 + 2000], vals[n0:n0 + 2000]) == 0
    ora.insert_int64_seq(keys[n0:n0 + 2000], vals[n0:n0 + 2000])
    victim = int(keys[7])
    dev.corrupt(victim)
    ora.corrupt(victim)
    seg = ora.segment_of(victim)
    same = [int(k) for k in keys[:n0] if ora.segment_of(int(k)) == seg][:3]
    fresh = [int(k) for k in keys[n0 + 2000:n0 + 2500]]
    bk = same + fresh
    bv = [bytes(v) for v in _obj(range(9000, 9000 + len(bk)), epoch=3)]
    exp = []
    for k, v in zip(bk, bv):
        r = ora.insert(k, v)
        exp.append(None if r is ora else r)
    assert any(e is not None for e in exp)
    assert dev.insert_batch(bk, bv) == exp
    if delta:
        assert dev.delta_stats()[0] > 0                       # the streamed batch went to the delta
    else:
        assert dev.delta_stats()[0] == 0                      # default: merged into the base
    assert dev.top_hash() == ora.top_hash()
    _levels(dev, ora)
    assert dev.get_batch(bk[:50]) == [ora.get(k) for k in bk[:50]]
    dev.close()
