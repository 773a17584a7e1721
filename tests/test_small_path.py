"""The per-key latency path: insert/3 and get/2 batches of
up to 16 keys served by one fused kernel (k_small) with an overlay of changed
segments that every other entry point merges into the CSR first.  Checked
against the C restatement (oracle/, the checker only) after every step, with
bulk operations interleaved (rehash, compare, exchange_get, snapshot, big
insert batches), corruption (synctree.erl:189-227, 302-320) and the fallback
to the bulk path (segments larger than the kernel rewrites)."""
import numpy as np
import pytest

from riak_ensemble_amd import workload


def _val(seq, epoch=1):
    return bytes([0]) + epoch.to_bytes(8, 'big') + seq.to_bytes(8, 'big')


@pytest.mark.gpu
@pytest.mark.parametrize('geom', [(16, 1 << 20), (4, 4096), (16, 16)])
def test_small_inserts_and_gets_interleaved(geom):
    import oracle_c as C
    from riak_ensemble_amd import synctree_hip
    W, S = geom
    n = 20000 if S >= 4096 else 3000
    keys = workload.keys_int63(n, workload.SEED ^ 0x51)
    vals = workload.obj_hash_values(n)
    dev = synctree_hip.DeviceTree(W, S)
    ora = C.OTree(W, S)
    assert dev.insert_int64(keys, vals) == 0
    ora.bulk_load_int64(keys, vals)
    assert dev.top_hash() == ora.top_hash()
    rng = np.random.default_rng(7)
    extra = workload.keys_int63(4000, workload.SEED ^ 0x52)
    seq = n
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
        if rng.random() < 0.2:          # a duplicate key inside the batch: last writer wins
            ks.append(ks[0])
            seq += 1
            vs.append(_val(seq))
            ks, vs = ks[-16:], vs[-16:]
        st = dev.insert_batch(ks, vs)
        assert all(x is None for x in st), st
        for k, v in zip(ks, vs):
            ora.insert(k, v)
        assert dev.top_hash() == ora.top_hash(), 'step %d' % step
        probe = [ks[0], int(keys[rng.integers(0, n)]), int(extra[rng.integers(0, len(extra))])]
        assert dev.get_batch(probe) == [ora.get(k) for k in probe]
        if step % 30 == 29:             # a bulk operation merges the overlay
            if step % 60 == 29:
                dev.rehash()
            else:
                assert dev.verify()
            assert dev.top_hash() == ora.top_hash()
            assert dev.num_entries() == ora.num_entries()
    # exchange_get of a few segments and a compare against a bulk-built copy
    segs = sorted({ora.segment_of(int(k)) for k in extra[:20]})
    assert dev.exchange_get_batch(ora.height + 1, segs) == [ora.node(ora.height + 1, s) for s in segs]
    for lvl in range(1, ora.height + 2):
        pa, ha = dev.level_entries(lvl)
        pb, hb = ora.level_entries(lvl)
        assert (pa == pb).all() and (ha == hb).all()
    dev.close()


@pytest.mark.gpu
def test_small_path_corruption_and_notfound():
    import oracle_c as C
    from riak_ensemble_amd import synctree_hip
    n = 5000
    keys = workload.keys_int63(n, workload.SEED ^ 0x53)
    vals = workload.obj_hash_values(n)
    dev = synctree_hip.DeviceTree()
    ora = C.OTree()
    dev.insert_int64(keys, vals)
    ora.bulk_load_int64(keys, vals)
    # get on an empty tree: undefined top => notfound
    empty = synctree_hip.DeviceTree()
    assert empty.get_batch([1, 2, 3]) == ['notfound'] * 3
    assert empty.insert_batch([5], [b'x']) == [None]
    assert empty.get_batch([5, 6]) == [b'x', 'notfound']
    empty.close()
    # raw corruption of one segment (a bumped value, no rehash)
    k0 = int(keys[10])
    s0 = ora.segment_of(k0)
    node = ora.node(ora.height + 1, s0)
    bad = [(node[0][0], bytes([node[0][1][0] ^ 1]) + node[0][1][1:])] + node[1:]
    dev.store_node(ora.height + 1, s0, bad)
    ora.store_segment(s0, bad)
    k1 = int(keys[11])
    got = dev.insert_batch([k0, k1], [_val(1, 9), _val(2, 9)])
    exp = [ora.insert(k0, _val(1, 9)), ora.insert(k1, _val(2, 9))]
    assert got[0] == exp[0] and got[0][0] == 'corrupted'
    assert got[1] is None and not isinstance(exp[1], tuple)
    assert dev.get_batch([k0, k1, 12345]) == [ora.get(k0), ora.get(k1), ora.get(12345)]
    assert dev.top_hash() == ora.top_hash()
    # a bulk rehash repairs the inner levels; then the segment verifies again
    dev.rehash()
    ora.rehash()
    assert dev.get_batch([k0]) == [ora.get(k0)]
    assert dev.top_hash() == ora.top_hash()
    dev.close()


@pytest.mark.gpu
def test_small_path_falls_back_for_big_segments():
    """A segment larger than the kernel rewrites (1024 entries) takes the bulk
    path: same results."""
    import oracle_c as C
    from riak_ensemble_amd import synctree_hip
    n = 40000          # 16 segments of ~2500 entries
    keys = workload.keys_int63(n, workload.SEED ^ 0x54)
    vals = workload.obj_hash_values(n)
    dev = synctree_hip.DeviceTree(16, 16)
    ora = C.OTree(16, 16)
    dev.insert_int64(keys, vals)
    ora.bulk_load_int64(keys, vals)
    for i in range(20):
        k = int(keys[i * 7])
        assert dev.insert_batch([k], [_val(i, 3)]) == [None]
        ora.insert(k, _val(i, 3))
        assert dev.top_hash() == ora.top_hash()
    assert dev.get_batch([int(keys[0]), int(keys[7])]) == [ora.get(int(keys[0])), ora.get(int(keys[7]))]
    dev.close()


@pytest.mark.gpu
def test_single_key_entry_points():
    """st_get1 / st_insert1 (the NIF's per-key calls) agree with the batch
    calls and with the C restatement, corruption included."""
    import oracle_c as C
    from riak_ensemble_amd import synctree_hip
    n = 5000
    keys = workload.keys_int63(n, workload.SEED ^ 0x57)
    vals = workload.obj_hash_values(n)
    dev = synctree_hip.DeviceTree()
    ora = C.OTree()
    assert dev.get1(5) == 'notfound'   # empty tree
    dev.insert_int64(keys, vals)
    ora.bulk_load_int64(keys, vals)
    for i in range(0, 200, 7):
        k = int(keys[i])
        assert dev.get1(k) == ora.get(k) == dev.get_batch([k])[0]
        assert dev.insert1(k, _val(i, 4)) is None
        ora.insert(k, _val(i, 4))
        assert dev.top_hash() == ora.top_hash()
    assert dev.insert1(('t', 1), b'\x00x') is None            # a term key
    assert dev.get1(('t', 1)) == b'\x00x'
    assert dev.get1(123456789) == ora.get(123456789) == 'notfound'
    k0 = int(keys[3])
    s0 = ora.segment_of(k0)
    node = ora.node(ora.height + 1, s0)
    bad = [(node[0][0], bytes([node[0][1][0] ^ 1]) + node[0][1][1:])] + node[1:]
    dev.store_node(ora.height + 1, s0, bad)
    ora.store_segment(s0, bad)
    assert dev.insert1(k0, _val(9, 9)) == ora.insert(k0, _val(9, 9))
    assert dev.get1(k0) == ora.get(k0)
    with pytest.raises(TypeError):
        dev.insert1(k0, 'not a binary')
    dev.close()


@pytest.mark.gpu
def test_per_key_requests_of_many_trees_in_one_launch():
    """st_insert1_multi / st_get1_multi: per-key insert/3 and get/2 requests
    of many trees (riak_ensemble_peer_tree.erl:224-246, every peer tree of a
    node taking puts at once) served by ONE launch over all the trees, a
    workgroup per tree -- the same results as the per-tree calls in request
    order, checked against one C restatement per tree: statuses (including
    {corrupted, L, B} from a corrupted segment), gets, top hashes."""
    import oracle_c as C
    from riak_ensemble_amd import synctree_hip, workload
    rng = np.random.default_rng(2024)
    geoms = [(16, 1 << 16), (16, 1 << 20), (4, 4096)]
    T, n0 = 24, 20_000
    devs, oras, keys = [], [], []
    for i in range(T):
        W, S = geoms[i % 3]
        k = workload.keys_int63(n0, workload.SEED ^ (0x3000 + i))
        v = workload.obj_hash_values(n0)
        d = synctree_hip.DeviceTree(W, S)
        assert d.insert_int64(k, v) == 0
        o = C.OTree(W, S).bulk_load_int64(k, v)
        devs.append(d); oras.append(o); keys.append([int(x) for x in k])
    # one corrupted segment in tree 5: requests into it are refused
    victim = keys[5][11]
    devs[5].corrupt(victim)
    oras[5].corrupt(victim)
    same = [k for k in keys[5] if oras[5].segment_of(k) == oras[5].segment_of(victim) and k != victim][:2]
    seq = 10 ** 6
    for r in range(12):
        m = int(rng.integers(40, 160))
        tix = [int(x) for x in rng.integers(0, T, m)]
        tix[:4] = [3, 3, 3, 3] * 1               # a tree repeated within the launch
        if r % 3 == 0:
            tix += [7] * 20                       # more than 16 requests for one tree: two launches
        ks, vs = [], []
        for t in tix:
            if rng.random() < 0.5:
                ks.append(keys[t][int(rng.integers(0, len(keys[t])))])
            else:
                nk = int(rng.integers(0, 1 << 62))
                keys[t].append(nk)
                ks.append(nk)
            seq += 1
            vs.append(bytes([0]) + (3).to_bytes(8, 'big') + seq.to_bytes(8, 'big'))
        if r == 4:
            tix += [5, 5]
            ks += same
            vs += [b'\x00' * 17, b'\x00' * 17]
        got = synctree_hip.insert1_multi([devs[t] for t in tix], ks, vs)
        exp = []
        for t, k, v in zip(tix, ks, vs):
            res = oras[t].insert(k, v)
            exp.append(None if res is oras[t] else res)
        assert got == exp, r
        if r == 4:
            assert exp[-1] is not None and exp[-1][0] == 'corrupted'
        probe_t = [int(x) for x in rng.integers(0, T, 200)]
        probe_k = [keys[t][int(rng.integers(0, len(keys[t])))] for t in probe_t]
        want = [oras[t].get(k) for t, k in zip(probe_t, probe_k)]
        assert synctree_hip.get1_multi([devs[t] for t in probe_t], probe_k) == want, r
        if r == 0:   # a value buffer too small: ST_ERANGE reports the size, the retry gets it all
            assert synctree_hip.get1_multi([devs[t] for t in probe_t], probe_k, vcap=16) == want
        for t in range(T):
            assert devs[t].top_hash() == oras[t].top_hash(), (r, t)
    for d in devs:
        d.close()
