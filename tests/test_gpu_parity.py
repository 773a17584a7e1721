"""Parity of the HIP product path (libsynctree_hip.so via riak_ensemble_amd.synctree)
with the CPU restatements (oracle/) and the golden fixtures.  Bit-exact
everywhere: segment ids, every level's entries, top hashes, ordered diff
lists, corruption tuples.  Needs an MI355X."""
import json
import os
import random

import numpy as np
import pytest

import oracle_c as C
import synctree_ref as R
from riak_ensemble_amd import synctree as S
from riak_ensemble_amd import synctree_hip, workload

pytestmark = pytest.mark.gpu

GOLD = json.load(open(os.path.join(os.path.dirname(__file__), 'golden', 'synctree_golden.json')))


def dec_key(d):
    if d['t'] == 'int':
        return int(d['v'])
    if d['t'] == 'atom':
        return d['v']
    return bytes.fromhex(d['v'])


def dec_val(v):
    return v['atom'] if isinstance(v, dict) else bytes.fromhex(v)


def dec_diff(lst):
    return [(dec_key(k), (dec_val(a), dec_val(b))) for k, (a, b) in lst]


def dec_result(r):
    if isinstance(r, dict) and 'tuple' in r:
        return tuple(r['tuple'])
    if isinstance(r, dict):
        return r['atom']
    return bytes.fromhex(r)


def build(n, width='default', segments='default'):
    """test/synctree_pure.erl:70-80 on the device path."""
    t = S.new(None, width, segments)
    for k in range(n, 0, -1):
        t = S.insert(k, (k * 10).to_bytes(8, 'big'), t)
    return t


def assert_levels_equal(dev, orc):
    """Every level's recorded entries, device vs C oracle."""
    for lvl in range(1, orc.height + 2):
        pa, ha = dev.modstate.level_entries(lvl)
        pb, hb = orc.level_entries(lvl)
        assert (pa == pb).all(), 'presence differs at level %d' % lvl
        assert (ha[pa == 1] == hb[pb == 1]).all(), 'hashes differ at level %d' % lvl


# ------------------------------------------------------------------ key -> segment
def test_segments_match_golden():
    t = S.new()
    assert t.modstate.segments_of(list(range(1, 101))) == GOLD['segments_int_1_100']
    keys = [dec_key(k) for k, _ in GOLD['segments_misc']]
    assert t.modstate.segments_of(keys) == [s for _, s in GOLD['segments_misc']]


# ------------------------------------------------------------------ synctree_pure
def test_pure_basic():
    """test/synctree_pure.erl:28-37"""
    t = build(100)
    assert S.get(42, t) == (420).to_bytes(8, 'big')
    t2 = S.insert(42, (42).to_bytes(8, 'big'), t)
    assert S.get(42, t2) == (42).to_bytes(8, 'big')
    assert t2.top_hash.hex() == GOLD['basic']['top_after']
    # the stale record t holds the old top hash: the reference reports corruption
    assert S.get(42, t) == dec_result(GOLD['basic']['get42_stale_record'])


def test_pure_corrupt():
    """test/synctree_pure.erl:43-54"""
    g = GOLD['corrupt']
    t = build(10)
    assert S.get(4, t) == dec_result(g['get4'])
    t2 = S.corrupt(4, t)
    assert S.get(4, t2) == dec_result(g['get4_corrupt'])
    assert S.insert(4, b'\x01', t2) == dec_result(g['insert_into_corrupt'])
    assert S.verify(t2) == g['verify_corrupt']
    assert S.verify_upper(t2) == g['verify_upper_corrupt']
    t3 = S.rehash(t2)
    assert S.get(4, t3) == 'notfound'
    assert t3.top_hash.hex() == g['top_rehashed']
    assert S.verify(t3) is True


def test_pure_exchange():
    """test/synctree_pure.erl:60-68"""
    t1, t2 = build(50), build(40)
    res = S.local_compare(t1, t2)
    assert sorted(res, key=lambda d: d[0]) == R.expected_diff(50, 10)
    assert res == dec_diff(GOLD['exchange_50_40'])
    assert S.local_compare(t2, t1) == dec_diff(GOLD['exchange_40_50'])


def test_remote_exact_order_device_and_generic():
    """test/synctree_remote.erl:37-39: exact order, through the device compare
    and through message-passing funs (the generic level loop)."""
    a, b = build(10), build(6)
    assert S.compare(S.height(a), S.direct_exchange(a), S.direct_exchange(b)) == R.expected_diff(10, 4)
    calls = []

    def remote(op, arg):
        calls.append(op)
        if op == 'exchange_get':
            return S.exchange_get(arg[0], arg[1], b)
        return 'ok'
    assert S.compare(S.height(a), S.direct_exchange(a), remote) == R.expected_diff(10, 4)
    assert 'start_exchange_level' in calls


def test_top_hashes_and_levels_build():
    for n, h in GOLD['top_build'].items():
        assert build(int(n)).top_hash.hex() == h
    t = build(100)
    assert_levels_equal(t, C.build(100))
    for lvl, nodes in GOLD['levels_build_100'].items():
        lvl = int(lvl)
        bks = [int(b) for b in nodes]
        imgs = S.exchange_get_batch(lvl, bks, t)
        for b, img in zip(bks, imgs):
            exp = nodes[str(b)]
            if lvl <= t.height:
                assert [[c, h.hex()] for c, h in img] == exp
            else:
                assert [[{'t': 'int', 'v': str(k)}, v.hex()] for k, v in img] == exp


# ------------------------------------------------------------------ randomized golden cases
def _dev_tree(case, entries, batch):
    t = S.new(None, case['width'], case['segments'])
    kv = [(dec_key(k), bytes.fromhex(v)) for k, v in entries]
    if batch:
        t, st = S.insert_batch(kv, t)
        assert all(s is None for s in st)
    else:
        for k, v in kv:
            t = S.insert(k, v, t)
    return t


@pytest.mark.parametrize('batch', [False, True])
@pytest.mark.parametrize('idx', range(len(GOLD['random_cases'])))
def test_random_case_golden(idx, batch):
    case = GOLD['random_cases'][idx]
    ta = _dev_tree(case, case['a'], batch)
    tb = _dev_tree(case, case['b_ops'], batch)
    top = ta.top_hash
    assert (top if isinstance(top, str) else top.hex()) == case['top_a']
    top = tb.top_hash
    assert (top if isinstance(top, str) else top.hex()) == case['top_b']
    assert S.local_compare(ta, tb) == dec_diff(case['diff_all'])
    for opt, key in (('local_only', 'diff_local_only'), ('remote_only', 'diff_remote_only')):
        got = S.compare(S.height(ta), S.direct_exchange(ta), S.direct_exchange(tb), None, [opt])
        assert got == dec_diff(case[key])
        # the generic (callback) level loop agrees with the device K3
        gen = S._compare_generic(S.height(ta), S.direct_exchange(ta), S.direct_exchange(tb), None, opt)
        assert gen == got
    for lvl, nodes in case['levels_a'].items():
        lvl = int(lvl)
        bks = [int(b) for b in nodes]
        for b, img in zip(bks, S.exchange_get_batch(lvl, bks, ta)):
            exp = nodes[str(b)]
            if lvl <= ta.height:
                assert [[c, h.hex()] for c, h in img] == exp
            else:
                assert img == [(dec_key(k), bytes.fromhex(v)) for k, v in exp]
    assert S.verify(ta) and S.verify(tb)
    if ta.height > 0:
        assert S.verify_upper(ta)
    for k, v in case['a'][:10]:
        assert S.get(dec_key(k), ta) == bytes.fromhex(v)


def test_both_filters_crash():
    t = build(3)
    with pytest.raises(S.SynctreeCrash):
        S.compare(S.height(t), S.direct_exchange(t), S.direct_exchange(t), None, ['local_only', 'remote_only'])


def test_bad_geometry():
    for w, s in [(16, 1000), (3, 9), (16, 8)]:
        with pytest.raises(S.SynctreeCrash):
            S.new(None, w, s)


def test_empty_trees():
    a, b = S.new(), S.new()
    assert S.top_hash(a) == 'undefined'
    assert S.get(1, a) == 'notfound'
    assert S.local_compare(a, b) == []
    assert S.verify(a) and S.verify_upper(a)
    b = S.insert(7, b'x', b)
    assert S.local_compare(a, b) == [(7, ('$none', b'x'))]
    assert S.local_compare(b, a) == [(7, (b'x', '$none'))]
    a = S.rehash(a)
    assert S.top_hash(a) == 'undefined'
    assert S.exchange_get(0, 0, a) == [(0, 'undefined')]


def test_height0_and_width2():
    for w, s in [(2, 1), (16, 16), (2, 2), (4, 1 << 10)]:
        keys = list(range(-20, 40)) + [b'', b'a', 'atom']
        vals = [bytes([i % 256]) * (i % 5) for i in range(len(keys))]
        d = S.new(None, w, s)
        o = C.OTree(w, s)
        for k, v in zip(keys, vals):
            d = S.insert(k, v, d)
            o.insert(k, v)
        assert d.top_hash == o.top_hash()
        assert_levels_equal(d, o)
        for k, v in zip(keys, vals):
            assert S.get(k, d) == v


# ------------------------------------------------------------------ corruption parity
def _corrupt_value(v):
    return bytes([(v[0] + 1) % 256]) + v[1:]


@pytest.mark.parametrize('geom', [(4, 256), (16, 4096), (16, 1 << 20)])
def test_raw_corruption_parity(geom):
    """test/synctree_intercepts.erl:96-104 mutations written through the raw
    backend (Mod:store), then every read path compared with the C oracle."""
    w, s = geom
    rng = random.Random(3)
    keys = list(range(1, 120))
    d = S.new(None, w, s)
    o = C.OTree(w, s)
    for k in keys:
        v = bytes(rng.randrange(256) for _ in range(17))
        d = S.insert(k, v, d)
        o.insert(k, v)
    H = d.height
    # corrupt_segment: first value's first byte of one segment
    seg = o.segment_of(keys[5])
    node = o.node(H + 1, seg)
    bad = [(node[0][0], _corrupt_value(node[0][1]))] + node[1:]
    d = S.m_flush(S.m_batch(('put', (H + 1, seg), bad), d))
    o.store_segment(seg, bad)
    # corrupt_upper: two levels above the segment of another key
    lvl = H - 1
    seg2 = o.segment_of(keys[40])
    b2 = seg2 >> (d.shift * (H + 1 - lvl))
    nd = o.node(lvl, b2)
    bad2 = [(nd[0][0], _corrupt_value(nd[0][1]))] + nd[1:]
    d = S.m_flush(S.m_batch(('put', (lvl, b2), bad2), d))
    o.store_inner(lvl, b2, bad2)
    for k in keys + [1000, 1001, b'zz']:
        assert S.get(k, d) == o.get(k), k
    assert S.verify(d) == o.verify()
    assert S.verify_upper(d) == o.verify_upper()
    # exchange against a clean tree: the reference crashes in orddict_delta
    clean_d, clean_o = S.new(None, w, s), C.OTree(w, s)
    for k in keys:
        clean_d = S.insert(k, b'z', clean_d)
        clean_o.insert(k, b'z')
    exp = o.compare(clean_o)
    assert exp[0] == 'crash'
    with pytest.raises(S.SynctreeCrash) as ei:
        S.local_compare(d, clean_d)
    assert repr(exp[2]) in str(ei.value)
    # inserts: rejected on corrupted paths, applied elsewhere
    for k in keys[:30] + [5000, 5001]:
        r = S.insert(k, b'q', d)
        e = o.insert(k, b'q')
        if isinstance(e, tuple):
            assert r == e
        else:
            assert not isinstance(r, tuple)
            d = r
    assert d.top_hash == o.top_hash()
    assert_levels_equal(d, o)
    # repair as riak_ensemble_peer_tree does (peer_tree.erl:264-277): delete + rehash
    d = S.m_flush(S.m_batch(('delete', (H + 1, seg)), d))
    o.delete_node(H + 1, seg)
    d = S.rehash(d)
    o.rehash()
    assert d.top_hash == o.top_hash()
    assert_levels_equal(d, o)
    assert S.verify(d) and o.verify()
    d = S.rehash_upper(d)
    o.rehash_upper()
    assert d.top_hash == o.top_hash()


def test_batch_duplicates_last_writer_wins():
    rng = random.Random(9)
    keys = [rng.randrange(0, 5000) for _ in range(3000)] + [b'k%d' % (i % 37) for i in range(200)]
    vals = [bytes(rng.randrange(256) for _ in range(rng.randrange(0, 40))) for _ in keys]
    d, st = S.insert_batch(list(zip(keys, vals)), S.new())
    assert all(s is None for s in st)
    o = C.OTree()
    for k, v in zip(keys, vals):
        o.insert(k, v)
    assert d.top_hash == o.top_hash()
    assert_levels_equal(d, o)
    # a second batch into the existing tree (merge path)
    keys2 = [rng.randrange(0, 8000) for _ in range(2000)]
    vals2 = [bytes([rng.randrange(256)]) * 17 for _ in keys2]
    d, st = S.insert_batch(list(zip(keys2, vals2)), d)
    for k, v in zip(keys2, vals2):
        o.insert(k, v)
    assert d.top_hash == o.top_hash()
    assert_levels_equal(d, o)
    assert S.get_batch([k for k in keys2[:50]], d) == [o.get(k) for k in keys2[:50]]


def test_stale_record_semantics():
    """ETS-backed records share nodes but not the top_hash field."""
    r = R.new()
    d = S.new()
    for k in range(1, 20):
        r = R.insert(k, b'v%d' % k, r)
        d = S.insert(k, b'v%d' % k, d)
    r_old, d_old = r, d
    r = R.insert(5, b'new', r)
    d = S.insert(5, b'new', d)
    for k in (5, 6, 100):
        assert S.get(k, d_old) == R.get(k, r_old)
        assert S.get(k, d) == R.get(k, r)
    assert S.insert(7, b'x', d_old) == R.insert(7, b'x', r_old)


# ------------------------------------------------------------------ bench-shaped sizes
def _bench_tree(n, vlen=17):
    keys = workload.keys_int63(n)
    vals = workload.obj_hash_values(n) if vlen == 17 else workload.test_values(keys)
    dt = synctree_hip.DeviceTree()
    assert dt.insert_int64(keys, vals) == 0
    ot = C.OTree().bulk_load_int64(keys, vals)
    return keys, vals, dt, ot


@pytest.mark.parametrize('n', [1000, 100_000, 1_000_000])
def test_bench_shaped_build_parity(n):
    keys, vals, dt, ot = _bench_tree(n)
    assert dt.top_hash() == ot.top_hash()
    for lvl in range(1, 7):
        pa, ha = dt.level_entries(lvl)
        pb, hb = ot.level_entries(lvl)
        assert (pa == pb).all() and (ha == hb).all()
    if n == 1000:
        assert dt.top_hash().hex() == GOLD['splitmix_1000']['top']
    # rehash of a device-resident tree reproduces the same hashes
    dt.rehash()
    assert dt.top_hash() == ot.top_hash()
    assert dt.verify() and dt.verify(upper=True)


def test_exchange_corrupt_segments_1m():
    """Config 3 shape at 1M keys: B = A with every 1000th non-empty segment's
    first value bumped and rehashed; the diff is exactly those keys, in
    reference order."""
    n = 1_000_000
    keys, vals, da, oa = _bench_tree(n)
    db = synctree_hip.DeviceTree()
    db.insert_int64(keys, vals)
    ob = C.OTree().bulk_load_int64(keys, vals)
    present, _ = oa.level_entries(6)
    segs = np.nonzero(present)[0][::1000]
    for s in segs.tolist():
        node = ob.node(6, s)
        bad = [(node[0][0], _corrupt_value(node[0][1]))] + node[1:]
        ob.store_segment(s, bad)
        db.store_node(6, s, bad)
    ob.rehash()
    db.rehash()
    assert db.top_hash() == ob.top_hash()
    exp = oa.compare(ob)
    assert len(exp) == len(segs)
    r = da.compare(db)
    assert r[0] == 'ok'
    assert [(k, vv) for _, k, vv in r[1]] == exp
    assert da.compare_device(db) == len(segs)
    # A2 = A with segs[3] corrupted WITHOUT rehash (inconsistent): the frontier
    # of A2 vs B reaches segs[3], whose verification fails -> the reference
    # crashes in orddict_delta there (local side)
    da2 = synctree_hip.DeviceTree()
    da2.insert_int64(keys, vals)
    oa2 = C.OTree().bulk_load_int64(keys, vals)
    node = oa.node(6, int(segs[3]))
    bad = [(node[0][0], _corrupt_value(_corrupt_value(node[0][1])))] + node[1:]
    da2.store_node(6, int(segs[3]), bad)
    oa2.store_segment(int(segs[3]), bad)
    exp = oa2.compare(ob)
    assert exp == ('crash', 'local', ('corrupted', 6, int(segs[3])))
    r = da2.compare(db)
    assert r == ('corrupted', 'local', ('corrupted', 6, int(segs[3])))
    # an identical-top pair never descends (level 0 equal): no crash, no diffs
    assert da2.compare(da)[0] == 'ok' and oa2.compare(oa) == []
