"""Parity at the BASELINE.json configuration sizes (configs 2-5), through the
C-ABI, against the C restatement (oracle/, the checker only).

* config 2: a 10M-key tree, full rehash (K1 + K2), every level's entries and
  the top hash bit-exact (synctree.erl:489-543).
* config 3: two 10M-key trees, every 1000th non-empty segment's first value
  bumped (test/synctree_intercepts.erl:96-104) plus keys only the remote tree
  holds; the full ordered diff list equals the oracle's compare/3
  (synctree.erl:372-417, Keys ++ Acc order), for every filter.
* config 5: a 100M-key tree partitioned by segment range over G = 1, 2, 4, 8
  partitions taking 1M-key write batches (50 % overwrites, 50 % new keys);
  the combined top hash and the owned level entries equal sequential oracle
  inserts (synctree.erl:189-209).
* config 4: a group of 512 ensembles x 1M keys (one GPU's share of 4096)
  rehashed as one device batch; every tree's top hash and a sample's upper
  levels equal the oracle's.

Inputs: splitmix64 keys masked to 63 bits (riak_ensemble_amd/workload.py),
17-byte ObjHash values <<0, Epoch:64, Seq:64>> (riak_ensemble_peer.erl:1717-1724).
"""
import concurrent.futures as cf

import numpy as np
import pytest

from riak_ensemble_amd import workload

N10M = 10_000_000
SEED = workload.SEED


def _keys(seed, n, start=0):
    """splitmix64(seed + i) masked to 63 bits (duplicates allowed: last writer wins)."""
    return (workload.splitmix64(seed, n, start) & np.uint64(0x7FFFFFFFFFFFFFFF)).astype(np.int64)


def _level_parity(dev, ora, levels):
    for lvl in levels:
        pa, ha = dev.level_entries(lvl)
        pb, hb = ora.level_entries(lvl)
        assert (pa == pb).all(), 'presence differs at level %d' % lvl
        assert (ha[pa == 1] == hb[pb == 1]).all(), 'hashes differ at level %d' % lvl


@pytest.fixture(scope='module')
def big():
    import oracle_c as C
    from riak_ensemble_amd import synctree_hip
    keys = _keys(SEED, N10M)
    vals = workload.obj_hash_values(N10M)
    ora = C.OTree().bulk_load_int64(keys, vals)
    dev = synctree_hip.DeviceTree()
    assert dev.insert_int64(keys, vals) == 0
    yield keys, vals, ora, dev
    dev.close()


@pytest.mark.gpu
def test_config2_rehash_10m_every_level(big):
    keys, vals, ora, dev = big
    # the batched insert's own dirty-path rehash ...
    assert dev.top_hash() == ora.top_hash()
    # ... and the full rehash (K1 tiles + level kernels), twice
    for _ in range(2):
        dev.rehash()
        assert dev.top_hash() == ora.top_hash()
        _level_parity(dev, ora, range(1, dev.height + 2))
    assert dev.verify() and dev.verify(upper=True)


@pytest.mark.gpu
def test_config3_compare_10m_ordered_diff(big):
    import oracle_c as C
    from riak_ensemble_amd import synctree_hip
    keys, vals, ora, dev = big
    pres, _ = ora.level_entries(dev.height + 1)
    segs = np.nonzero(pres)[0][::1000]
    bumped = []
    for s in segs.tolist():
        k, v = ora.node(dev.height + 1, int(s))[0]
        bumped.append((k, bytes([(v[0] + 1) % 256]) + v[1:]))
    extra_k = _keys(SEED ^ 0x3, 200)
    extra_v = workload.obj_hash_values(200, epoch=2)
    remote = synctree_hip.DeviceTree()
    assert remote.insert_int64(keys, vals) == 0
    st = remote.insert_batch([k for k, _ in bumped] + [int(k) for k in extra_k],
                             [v for _, v in bumped] + [bytes(v) for v in extra_v])
    assert all(s is None for s in st)
    orb = C.OTree().bulk_load_int64(keys, vals)
    for k, v in bumped:
        orb.insert(k, v)
    orb.insert_int64_seq(extra_k, extra_v)
    assert remote.top_hash() == orb.top_hash()
    for filt, opts in ((0, ()), (1, ('local_only',)), (2, ('remote_only',))):
        exp = ora.compare(orb, opts)
        r = dev.compare(remote, filt)
        assert r[0] == 'ok'
        got = [(k, vv) for _, k, vv in r[1]]
        assert len(got) == len(exp)
        assert got == exp, 'ordered diff differs (filter %s)' % (opts,)
        assert dev.compare_device(remote, filt) == len(exp)
    # and the other direction
    exp = orb.compare(ora)
    r = remote.compare(dev)
    assert [(k, vv) for _, k, vv in r[1]] == exp
    remote.close()


class _Local:
    def __init__(self, rank, world):
        self.rank, self.world = rank, world

    def get_rank(self, group=None):
        return self.rank

    def get_world_size(self, group=None):
        return self.world


def _combine(parts):
    rows = []
    for p in parts:
        pres, hashes = p.tree.level_entries(2)
        a, b = p.b2
        rows.append(np.concatenate([pres[a:b, None], hashes[a:b]], axis=1))
    rows = np.concatenate(rows)
    for p in parts:
        p.tree.combine_upper(rows[:, 0].copy(), rows[:, 1:].copy())


@pytest.mark.gpu
def test_config5_partitioned_streaming_100m():
    """BASELINE config 5 at its size: a 100M-key tree partitioned by segment
    range over G = 1, 2, 4, 8 partitions (one process here; the same
    st_set_partition + level-2 all-gather + st_combine_upper path as the
    G-rank run), two 1M-key write batches (50 % overwrites, 50 % new keys)
    through the insert path with its dirty-path rehash; after every batch
    the combined top hash equals the oracle's sequential inserts
    (ot_apply_int64_batch, pinned against insert_int64_seq in test_oracle),
    and at the end every partition's owned level-2/3/6 entries and a full
    rehash agree."""
    import torch
    import oracle_c as C
    from riak_ensemble_amd import synctree_hip, parallel
    N = 100_000_000
    seed = 0x5EED0005
    keys = _keys(seed, N)
    vals = workload.obj_hash_values(N)
    rng = np.random.default_rng(5)
    batches = []
    B = 1_000_000
    for j in range(2):
        old = rng.integers(0, N, B // 2)
        k = np.concatenate([keys[old], _keys(seed, B - B // 2, N + j * B)])
        seq = np.concatenate([old + 1, np.arange(N + j * B, N + j * B + (B - B // 2))]).astype(np.uint64)
        v = np.zeros((B, 17), np.uint8)
        v[:, 8] = 1
        v[:, 9:17] = seq.astype('>u8').view(np.uint8).reshape(B, 8)
        batches.append((k, v))
    ora = C.OTree().bulk_load_int64_par(keys, vals)
    tops, lv = [], {}
    for k, v in batches:
        ora.apply_int64_batch(k, v)
        tops.append(ora.top_hash())
    for lvl in (2, 3, 6):
        lv[lvl] = ora.level_entries(lvl)
    del ora
    kd = torch.from_numpy(keys).cuda()
    vd = torch.from_numpy(vals.reshape(-1)).cuda()
    torch.cuda.synchronize()   # the library reads device inputs on its own stream
    for G in (1, 2, 4, 8):
        parts = [parallel.PartitionedTree(synctree_hip.DeviceTree(), _Local(r, G)) for r in range(G)]
        for p in parts:
            assert p.tree.insert_int64_device(kd.data_ptr(), vd.data_ptr(), N, 17) == 0
        torch.cuda.synchronize()
        _combine(parts)
        for j, (k, v) in enumerate(batches):
            for p in parts:
                assert p.tree.insert_int64(k, v) == 0
            _combine(parts)
            assert all(p.top_hash() == tops[j] for p in parts), 'G=%d batch %d' % (G, j)
        for p in parts:
            for lvl in (2, 3, 6):
                pa, ha = p.tree.level_entries(lvl)
                pb, hb = lv[lvl]
                m = len(pa) // G
                sl = slice(p.rank * m, (p.rank + 1) * m)
                assert (pa[sl] == pb[sl]).all() and (ha[sl] == hb[sl]).all(), 'G=%d level %d' % (G, lvl)
        for p in parts:     # a full rehash of every partition reproduces the same top hash
            p.tree.rehash()
        _combine(parts)
        assert all(p.top_hash() == tops[-1] for p in parts)
        for p in parts:
            p.tree.close()


@pytest.mark.gpu
def test_config4_group_512_ensembles_1m():
    """BASELINE config 4's per-GPU share at its size: 512 ensembles x 1M keys
    (4096 over 8 GPUs) rehashed as ONE device batch (st_rehash_group); every
    tree's top hash equals the oracle's, the upper levels of a sample too."""
    import oracle_c as C
    from riak_ensemble_amd import synctree_hip
    E, n = 512, 1_000_000
    vals = workload.obj_hash_values(n)

    def oracle(e):
        o = C.OTree().bulk_load_int64_par(_keys(SEED ^ (e + 1), n), vals, 1)
        r = (o.top_hash(), o.level_entries(2) if e % 64 == 0 else None, o.level_entries(3) if e % 64 == 0 else None)
        del o
        return r

    with cf.ThreadPoolExecutor(16) as ex:
        fut = [ex.submit(oracle, e) for e in range(E)]
        trees = []
        for e in range(E):
            t = synctree_hip.DeviceTree()
            assert t.insert_int64(_keys(SEED ^ (e + 1), n), vals) == 0
            trees.append(t)
        exp = [f.result() for f in fut]
    synctree_hip.rehash_group(trees)
    for e, (t, (top, l2, l3)) in enumerate(zip(trees, exp)):
        assert t.top_hash() == top, 'ensemble %d' % e
        if l2 is not None:
            for lvl, (pb, hb) in ((2, l2), (3, l3)):
                pa, ha = t.level_entries(lvl)
                assert (pa == pb).all() and (ha == hb).all()
    # per-tree rehash agrees with the batch
    for t in trees[:4]:
        t.rehash()
    assert [t.top_hash() for t in trees[:4]] == [e[0] for e in exp[:4]]
    for t in trees:
        t.close()
