"""term_to_binary keys (synctree.erl:261-268): tuples,
lists, maps, floats and integers outside int64.  The host passes
term_to_binary(Key) (ST_KEY_TERM); the library derives an order-preserving
record (riak_ensemble_amd/csrc/term_key.h) whose memcmp order is Erlang term
order, and hashes term_to_binary(Key) -- or <<Key:64>> for an integer -- for
the segment.

CPU: the record order against the Python restatement's term order
(oracle/synctree_ref.py term_key, the checker) over random nested terms;
ETF round trips.  GPU: trees of mixed keys built through the device path
against synctree_ref (top hash, every level's entries, get, exchange_get,
ordered compare), through both the small-batch and the bulk path."""
import random

import numpy as np
import pytest

import synctree_ref as R
from riak_ensemble_amd import terms


def rand_atom(rng):
    pool = ['a', 'b', 'ab', 'abc', 'z', 'é', 'ñandú', 'xÿ', '中', 'true', '', 'a\u0000b']
    return rng.choice(pool) if rng.random() < 0.7 else ''.join(rng.choice('abcxyz') for _ in range(rng.randint(1, 6)))


def rand_term(rng, depth=0):
    r = rng.random()
    leaf = depth >= 3 or r < 0.55
    if leaf:
        k = rng.randrange(9)
        if k == 0:
            return rng.randint(-300, 300)
        if k == 1:
            return rng.choice([(1 << 63) - 1, -(1 << 63), (1 << 31), -(1 << 31) - 1, 0])
        if k == 2:   # bignums, both signs
            return rng.choice([1, -1]) * rng.randint(1 << 63, 1 << rng.choice([64, 70, 100, 200]))
        if k == 3:   # non-integral floats
            return rng.choice([-1, 1]) * (rng.randint(0, 1 << 20) + rng.choice([0.5, 0.25, 0.1, 1e-9]))
        if k == 4:   # floats beyond int64 (integral)
            return rng.choice([-1.0, 1.0]) * 2.0 ** rng.randint(64, 300) * (1 + rng.random())
        if k == 5:
            return rand_atom(rng)
        if k == 6:
            return bytes(rng.choice([0, 1, 97, 255]) for _ in range(rng.randint(0, 5)))
        if k == 7:
            return []
        return rng.randint(0, 255)
    if r < 0.7:
        return tuple(rand_term(rng, depth + 1) for _ in range(rng.randint(0, 4)))
    if r < 0.8:   # a map; keys compare exactly (1 and 1.0 are two keys)
        pool = [1, 1.0, 2, 0.5, -3, 'a', (1,), (1.0,), b'k']
        pairs = [(rng.choice(pool) if rng.random() < 0.5 else rand_term(rng, depth + 1), rand_term(rng, depth + 1))
                 for _ in range(rng.randint(0, 4))]
        return terms.Map(pairs)
    if rng.random() < 0.3:   # a "string"
        return [rng.randint(0, 255) for _ in range(rng.randint(1, 5))]
    return [rand_term(rng, depth + 1) for _ in range(rng.randint(1, 4))]


def distinct_terms(n, seed):
    rng = random.Random(seed)
    out, seen = [], set()
    while len(out) < n:
        t = rand_term(rng)
        k = repr(R.term_key(t))
        if k in seen:
            continue
        seen.add(k)
        out.append(t)
    return out


def test_etf_round_trip_and_parts():
    for t in distinct_terms(500, 1):
        b = terms.term_to_binary(t)
        assert b == R.term_to_binary(t), t        # two independent restatements agree
        assert terms.binary_to_term(b) == t
        kt, kb = terms.key_parts(t)
        assert terms.key_from_parts(kt, kb) == t


def test_key_record_order_is_erlang_term_order():
    """memcmp order of the library's key records (st_key_record: host code,
    no device) == Erlang term order of the restatement, for nested terms of
    every supported type, plain keys included."""
    ts = distinct_terms(3000, 2) + [0, -1, 1, 255, 256, 'a', b'a', (), [], [[]], {0: 1}.get(0), 1.5, -1.5]
    uniq = {}
    for t in ts:
        uniq.setdefault(repr(R.term_key(t)), t)
    ts = list(uniq.values())
    by_erlang = sorted(ts, key=R.term_key)
    by_record = sorted(ts, key=terms.order_key)
    bad = [(a, b) for a, b in zip(by_erlang, by_record) if a != b or type(a) != type(b)]
    assert not bad, bad[:5]
    # the order part (terms.order_sk) decides too, and Erlang-equal numbers
    # (==: 1 and 1.0, nested or not, bignums and big integral floats, 0 and
    # -0.0) have EQUAL order parts -- one key for orddict:store/erase,
    # lists:keyfind and orddict_delta
    assert sorted(ts, key=terms.order_sk) == by_record
    eq_pairs = [(1, 1.0), (0, -0.0), (-7, -7.0), ((1, 'a'), (1.0, 'a')), ([2, [3]], [2.0, [3.0]]),
                (1 << 70, float(1 << 70)), (-(1 << 80), -float(1 << 80)), ((1 << 63) - 1024, float((1 << 63) - 1024))]
    for a, b in eq_pairs:
        assert R.term_key(a) == R.term_key(b)
        assert terms.order_sk(a) == terms.order_sk(b), (a, b)
    for a, b in [(1, 1.5), (1.5, 2), ((1, 'a'), (1.5, 'a')), (-1, -0.5)]:
        assert (terms.order_sk(a) < terms.order_sk(b)) == (R.term_key(a) < R.term_key(b)), (a, b)
    # plain-domain keys keep their short records
    assert terms.order_key(5) == bytes([0x10, 0x80, 0, 0, 0, 0, 0, 0, 5])
    assert terms.order_key('ab') == b'\x20ab'
    assert terms.order_key(b'ab') == b'\x50ab'


def test_map_keys_order_and_equality():
    """Maps (synctree.erl:261-268 sends them through term_to_binary): ordered
    by size, then keys in map-key order, then values (ERTS term comparison);
    map keys compare exactly -- #{1 => a} and #{1.0 => a} are different keys,
    and every integer key sorts before every float key -- while values compare
    with ==, so #{a => 1} and #{a => 1.0} are one key."""
    M = terms.Map
    ms = [M({}), M({'a': 1}), M({'a': 1.0}), M({1: 'a'}), M([(1.0, 'a')]), M({2: 'a'}), M([(0.5, 'a')]),
          M({'a': 1, 'b': 2}), M([(1, 'x'), (1.0, 'y')]), M({(1,): 0}), M([((1.0,), 0)]), M({'a': M({1: 2})}),
          M({'a': M([(1.0, 2)])}), M({b'k': [1, 2]}), M({'z': (1, 2)}), M([(3, 'a'), (-3, 'a')]),
          M({1 << 70: 'a'}), M([(2.0 ** 70, 'a')])]
    near = [(9,), (9, 9, 9, 9), [], [1], 'atom', b'bin', 7, 7.5]
    ts = ms + near
    by_erlang = sorted(ts, key=R.term_key)
    by_record = sorted(ts, key=terms.order_sk)   # (stable: the two == maps keep their order)
    assert [repr(x) for x in by_erlang] == [repr(x) for x in by_record]
    # the documented rules, spelled out
    ok = terms.order_sk
    assert ok(M({1: 'a'})) < ok(M([(1.0, 'a')]))              # integer key before float key
    assert ok(M({2: 'a'})) < ok(M([(0.5, 'a')]))              # ... whatever their values
    assert ok(M({1 << 70: 'a'})) < ok(M([(2.0 ** 70, 'a')]))
    assert ok(M({'z': 0})) < ok(M({'a': 1, 'b': 2}))          # size first
    assert ok(M({'a': 1})) == ok(M({'a': 1.0}))               # values compare with ==
    assert ok(M({'a': M({1: 2})})) != ok(M({'a': M([(1.0, 2)])}))   # a map value's keys: exact
    assert ok((9,)) < ok(M({})) < ok([])                      # tuple < map < nil
    for a, b in [(M({'a': 1}), M({'a': 1.0})), (M({'a': (1, 2.0)}), M({'a': (1.0, 2)}))]:
        assert R.term_key(a) == R.term_key(b)
    assert R.term_key(M({1: 'a'})) != R.term_key(M([(1.0, 'a')]))
    # term_to_binary writes a map's pairs in map-key order (a flatmap)
    assert terms.term_to_binary(M([(1.0, 'a'), (2, 'b'), ('c', 1)])) == (
        b'\x83t\x00\x00\x00\x03' + b'a\x02' + b'd\x00\x01b' + b'F' + __import__('struct').pack('>d', 1.0) +
        b'd\x00\x01a' + b'd\x00\x01c' + b'a\x01')
    assert terms.binary_to_term(terms.term_to_binary(M([(1, 'a'), (1.0, 'b')]))) == M([(1, 'a'), (1.0, 'b')])


def test_term_key_rejects_outside_domain():
    with pytest.raises(TypeError):
        terms.key_parts(True)
    with pytest.raises(TypeError):
        terms.key_parts({1, 2})   # a Python set: no Erlang term
    with pytest.raises(TypeError):
        terms.key_parts(object())
    # pids, refs, ports and funs stay outside the device key domain (ST_EINVAL)
    import ctypes
    from riak_ensemble_amd import _lib as L
    n = ctypes.c_uint64()
    pid = b'\x83' + bytes([88, 100, 0, 13]) + b'nonode@nohost' + bytes(12)   # NEW_PID_EXT
    assert L.load().st_key_record(3, pid, len(pid), None, 0, ctypes.byref(n)) == L.ST_EINVAL
    from riak_ensemble_amd import _lib
    # a malformed ETF is refused by the library (ST_EINVAL)
    with pytest.raises(ValueError):
        import ctypes
        n = ctypes.c_uint64()
        _lib.check(_lib.load().st_key_record(3, b'\x83\x68\x02\x61', 4, None, 0, ctypes.byref(n)), 'st_key_record')


def test_bignum_segment_is_low_64_bits():
    """ensure_binary(Integer) = <<Key:64>> even for bignums: the segment of
    2^64 + 5 is the segment of 5 (synctree.erl:261-262)."""
    assert R.get_segment((1 << 64) + 5, 1 << 20) == R.get_segment(5, 1 << 20)
    assert R.get_segment(-(1 << 64) - 1, 1 << 20) == R.get_segment(-1, 1 << 20)


# ------------------------------------------------------------------ GPU
def _ref_tree(keys, vals, width, segments):
    t = R.new(b'ref', width, segments)
    for k, v in zip(keys, vals):
        t = R.insert(k, v, t)
    return t


def _val(i):
    return bytes([0]) + (1).to_bytes(8, 'big') + i.to_bytes(8, 'big')


@pytest.mark.gpu
@pytest.mark.parametrize('geom,n,batch', [((16, 256), 3000, 4096), ((16, 256), 600, 16), ((16, 1 << 20), 2000, 4096),
                                          ((4, 64), 800, 7)])
def test_term_keys_device_parity(geom, n, batch):
    from riak_ensemble_amd import synctree_hip
    W, S = geom
    keys = distinct_terms(n, 10 + n) + [5, -7, 'atom', b'bin', (1 << 64) + 5, 5.5]
    vals = [_val(i) for i in range(len(keys))]
    ref = _ref_tree(keys, vals, W, S)
    dev = synctree_hip.DeviceTree(W, S)
    for i in range(0, len(keys), batch):
        st = dev.insert_batch(keys[i:i + batch], vals[i:i + batch])
        assert all(x is None for x in st)
    assert dev.top_hash() == R.top_hash(ref)
    H = R.height(ref)
    for lvl in range(1, H + 2):
        buckets = list(range(min(W ** (lvl - 1), 4096)))
        got = dev.exchange_get_batch(lvl, buckets)
        exp = [R.exchange_get(lvl, b, ref) for b in buckets]
        assert got == exp, 'level %d' % lvl
    probe = keys[::7] + [(9, 9, 9), [1, 2, 3, 4, 5, 6], -(1 << 99)]
    assert dev.get_batch(probe) == [R.get(k, ref) for k in probe]
    # compare against a modified copy: diff order = descending segment, ascending Erlang term order
    keys2 = keys[: n // 2] + distinct_terms(200, 99)
    vals2 = [_val(i + 7) for i in range(len(keys2))]
    ref2 = _ref_tree(keys2, vals2, W, S)
    dev2 = synctree_hip.DeviceTree(W, S)
    dev2.insert_batch(keys2, vals2)
    res = dev.compare(dev2)
    assert res[0] == 'ok'
    assert [(k, v) for _, k, v in res[1]] == R.local_compare(ref, ref2)
    dev.close()
    dev2.close()


def _same_segment_pairs(S, want):
    """(integer-form, float-form) key pairs that hash to one segment of S."""
    out = []
    for k in range(1, 5000):
        for a, b in ((k, float(k)), ((k, 'x'), (float(k), 'x'))):
            if R.get_segment(a, S) == R.get_segment(b, S):
                out.append((a, b))
        if len(out) >= want:
            break
    return out


@pytest.mark.gpu
@pytest.mark.parametrize('bulk', [False, True])
def test_equal_numbers_are_one_key(bulk):
    """1 and 1.0 (and {1,x} / {1.0,x}) in one segment are ONE key, as the
    reference's orddict:store (synctree.erl:206: the later key form and value
    replace the entry), lists:keyfind in get (:342-348) and orddict_delta
    (riak_ensemble_util.erl:120-125, K1 reported) treat them; corrupt/2's
    orddict:erase removes either form.  Device vs synctree_ref, through the
    per-key kernel and the bulk ingest."""
    from riak_ensemble_amd import synctree_hip
    W, S = 4, 64
    pairs = _same_segment_pairs(S, 6)
    assert len(pairs) >= 4
    ref = R.new(b'ref', W, S)
    dev = synctree_hip.DeviceTree(W, S)
    filler = [(i * 7919, _val(i)) for i in range(40)]
    first = [(a, _val(100 + j)) for j, (a, _) in enumerate(pairs)]
    second = [(b, _val(200 + j)) for j, (_, b) in enumerate(pairs)]
    for k, v in filler + first + second:
        ref = R.insert(k, v, ref)
    if bulk:   # one bulk batch: last writer wins among == keys
        kv = filler + first + second
        assert all(x is None for x in dev.insert_batch([k for k, _ in kv], [v for _, v in kv]))
    else:      # one key per call (the per-key kernel)
        for k, v in filler + first + second:
            assert dev.insert_batch([k], [v]) == [None]
    assert dev.top_hash() == R.top_hash(ref)
    segs = sorted({R.get_segment(a, S) for a, _ in pairs})
    got = dev.exchange_get_batch(R.height(ref) + 1, segs)
    exp = [R.exchange_get(R.height(ref) + 1, s, ref) for s in segs]
    assert got == exp
    assert all(type(k) is type(e) for g, x in zip(got, exp) for (k, _), (e, _) in zip(g, x))   # the float form is stored
    probe = [a for a, _ in pairs] + [b for _, b in pairs]
    assert dev.get_batch(probe) == [R.get(k, ref) for k in probe]
    assert dev.get_batch(probe) == [v for _, v in second] * 2
    # orddict_delta: the integer form here, the float form there, different values
    ref2 = R.new(b'ref2', W, S)
    dev2 = synctree_hip.DeviceTree(W, S)
    for k, v in filler + first:
        ref2 = R.insert(k, v, ref2)
    dev2.insert_batch([k for k, _ in filler + first], [v for _, v in filler + first])
    res = dev2.compare(dev)
    assert res[0] == 'ok'
    got, exp = [(k, v) for _, k, v in res[1]], R.local_compare(ref2, ref)
    assert got == exp and len(exp) == len(pairs)
    assert [repr(k) for k, _ in got] == [repr(k) for k, _ in exp]   # K1: the local (integer) form
    # corrupt/2 with the other form erases the entry
    a0, b0 = pairs[0]
    dev.corrupt(a0)
    ref = R.corrupt(a0, ref)
    assert dev.get_batch([b0]) == [R.get(b0, ref)]
    dev.close()
    dev2.close()


@pytest.mark.gpu
def test_compare_long_common_key_prefixes():
    """The compare merge-join orders keys by a 12-byte order prefix and falls
    back to the staged bytes on a tie: binary keys sharing 11..40 leading
    bytes, keys that are prefixes of other keys, and values differing only in
    their last byte, against synctree_ref's local_compare."""
    from riak_ensemble_amd import synctree_hip
    W, S = 4, 16
    stem = bytes(range(65, 105))
    keys = []
    for cut in (10, 11, 12, 13, 20, 40):
        for tail in (b'', b'\x00', b'\x01', b'\xff', b'\x00\x00', b'ab'):
            keys.append(stem[:cut] + tail)
    keys = list(dict.fromkeys(keys))
    vals = [_val(i) for i in range(len(keys))]
    keys2 = keys[::2] + [stem[:12] + b'zz', stem + b'\x00\x01']
    vals2 = [(v[:-1] + bytes([v[-1] ^ 1])) if i % 3 == 0 else v for i, v in enumerate(vals[::2])] + [_val(900), _val(901)]
    ref, ref2 = _ref_tree(keys, vals, W, S), _ref_tree(keys2, vals2, W, S)
    dev, dev2 = synctree_hip.DeviceTree(W, S), synctree_hip.DeviceTree(W, S)
    dev.insert_batch(keys, vals)
    dev2.insert_batch(keys2, vals2)
    for a, b, ra, rb in ((dev, dev2, ref, ref2), (dev2, dev, ref2, ref)):
        res = a.compare(b)
        assert res[0] == 'ok'
        assert [(k, v) for _, k, v in res[1]] == R.local_compare(ra, rb)
    dev.close()
    dev2.close()


def test_map_keys_outside_the_restated_etf_are_refused(monkeypatch):
    """ERTS writes a hashmap (> 32 pairs) in its hash order and, from OTP 26,
    a flatmap's atom keys in atom-index order: neither byte string can be
    restated, so such a key (whose segment is md5 of those bytes,
    synctree.erl:251-268) is refused rather than silently put in another
    segment than the Erlang peer's.  The NIF passes ERTS's own bytes."""
    big = terms.Map([(i, i) for i in range(33)])
    with pytest.raises(TypeError):
        terms.term_to_binary(big)
    with pytest.raises(R.ErlangCrash):
        R.term_to_binary(big)
    ok = terms.Map([(i, i) for i in range(32)])
    assert terms.term_to_binary(ok) == R.term_to_binary(ok)
    two_atoms = terms.Map([('a', 1), ('b', 2)])
    assert terms.term_to_binary(two_atoms, atoms='latin1') == R.term_to_binary(two_atoms)
    monkeypatch.setattr(R, 'ETF_ATOMS', 'utf8')
    with pytest.raises(TypeError):
        terms.term_to_binary(two_atoms, atoms='utf8')
    with pytest.raises(R.ErlangCrash):
        R.term_to_binary(two_atoms)
    one_atom = terms.Map([('a', 1), (2, 2)])
    assert terms.term_to_binary(one_atom, atoms='utf8') == R.term_to_binary(one_atom)
