"""Segment-pair shapes of the device compare (k_cmp_walk)
against the C restatement of compare/3..5 (synctree.erl:354-449,
riak_ensemble_util.erl:115-141 orddict_delta): the staged first pair of a
wave's list (<= 63 entries and <= 1 KB of keys a side) and every fallback
next to it -- a side with no entries (local-only / remote-only segments),
segments of more than 63 entries, key runs over 1 KB, empty values, many
differing segments per wave, and both filters.  Needs an MI355X."""
import numpy as np
import pytest

import oracle_c as C
from riak_ensemble_amd import _lib, synctree_hip

pytestmark = pytest.mark.gpu

FILTERS = [((), _lib.ST_FILTER_ALL), (('local_only',), _lib.ST_FILTER_LOCAL_ONLY),
           (('remote_only',), _lib.ST_FILTER_REMOTE_ONLY)]


def _rand_bin(rng, lo, hi):
    return bytes(rng.integers(0, 256, int(rng.integers(lo, hi + 1)), dtype=np.uint8))


def _pair(segments, base, a_only, b_only, changed, rng):
    """A = base + a_only; B = base (values of `changed` replaced) + b_only."""
    ka = list(base) + list(a_only)
    va = [base[k] for k in base] + [a_only[k] for k in a_only]
    kb, vb = [], []
    for k, v in base.items():
        kb.append(k)
        vb.append(changed.get(k, v))
    kb += list(b_only)
    vb += [b_only[k] for k in b_only]
    da, db = synctree_hip.DeviceTree(16, segments), synctree_hip.DeviceTree(16, segments)
    oa, ob = C.OTree(16, segments), C.OTree(16, segments)
    assert all(x is None for x in da.insert_batch(ka, va))
    assert all(x is None for x in db.insert_batch(kb, vb))
    oa.bulk_load(ka, va)
    ob.bulk_load(kb, vb)
    assert da.top_hash() == oa.top_hash() and db.top_hash() == ob.top_hash()
    return da, db, oa, ob


def _check(da, db, oa, ob):
    for opts, filt in FILTERS:
        exp = oa.compare(ob, opts)
        got = da.compare(db, filt)
        assert got[0] == 'ok', got
        assert [(k, vv) for _, k, vv in got[1]] == exp, opts
        assert da.compare_device(db, filt) == len(exp)
        # and the other way round (the remote side's shapes become local)
        exp_r = ob.compare(oa, opts)
        got_r = db.compare(da, filt)
        assert [(k, vv) for _, k, vv in got_r[1]] == exp_r, ('reverse', opts)


@pytest.mark.parametrize('segments,nkeys,klen,vlen', [
    (4096, 20_000, (1, 24), (0, 40)),     # ~5 entries a segment: the staged pair
    (256, 20_000, (1, 24), (0, 40)),      # ~78 a segment: over 63 entries, the fallback
    (4096, 12_000, (60, 120), (17, 17)),  # long keys: several segments over 1 KB of keys
    (65536, 30_000, (8, 8), (0, 0)),      # empty values only
])
def test_compare_segment_shapes(segments, nkeys, klen, vlen):
    rng = np.random.default_rng(segments * 7 + nkeys)
    base = {}
    while len(base) < nkeys:
        base[_rand_bin(rng, *klen)] = _rand_bin(rng, *vlen)
    keys = list(base)
    o = C.OTree(16, segments)
    segs = {}
    for k in keys:
        segs.setdefault(o.segment_of(k), []).append(k)
    occupied = sorted(segs)
    pick = rng.permutation(len(occupied))
    # whole segments only on one side, values changed in others, single new keys
    a_seg = [occupied[i] for i in pick[:40]]
    b_seg = [occupied[i] for i in pick[40:80]]
    a_only = {k: base.pop(k) for s in a_seg for k in segs[s]}
    b_only = {k: base.pop(k) for s in b_seg for k in segs[s]}
    changed = {}
    for i in pick[80:400]:
        for k in segs[occupied[i]][:2]:
            if k in base:
                changed[k] = _rand_bin(rng, *vlen) + b'\x01'
    for _ in range(150):
        a_only[_rand_bin(rng, *klen)] = _rand_bin(rng, *vlen)
        b_only[_rand_bin(rng, *klen)] = _rand_bin(rng, *vlen)
    da, db, oa, ob = _pair(segments, base, a_only, b_only, changed, rng)
    _check(da, db, oa, ob)
    da.close()
    db.close()


def test_compare_many_diff_segments_per_wave():
    """Every segment differs (a wave lists more than 32 items: no staged
    pair), then one differing segment per 50 (one or two a wave)."""
    rng = np.random.default_rng(5)
    S = 65536
    keys = [int(x) for x in rng.choice(1 << 40, 60_000, replace=False)]
    vals = [bytes(_rand_bin(rng, 17, 17)) for _ in keys]
    o = C.OTree(16, S)
    for every in (1, 50):
        seg_of = {k: o.segment_of(k) for k in keys}
        hit = sorted(set(seg_of.values()))[::every]
        hit = set(hit)
        vb, done = [], set()
        for k, v in zip(keys, vals):
            s = seg_of[k]
            if s in hit and s not in done:
                done.add(s)
                vb.append(v[:-1] + bytes([v[-1] ^ 0x5a]))
            else:
                vb.append(v)
        da, db = synctree_hip.DeviceTree(16, S), synctree_hip.DeviceTree(16, S)
        oa, ob = C.OTree(16, S), C.OTree(16, S)
        assert all(x is None for x in da.insert_batch(keys, vals))
        assert all(x is None for x in db.insert_batch(keys, vb))
        oa.bulk_load(keys, vals)
        ob.bulk_load(keys, vb)
        exp = oa.compare(ob)
        assert len(exp) == len(hit)
        _check(da, db, oa, ob)
        da.close()
        db.close()
