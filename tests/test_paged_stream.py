"""Streaming insert batches through the paged segment layout (DESIGN.md
§3.3): an insert/3 batch much smaller than the tree
rewrites only the tails of the segments it touches inside per-segment pages
with slack, moves a segment that outgrew its page to the append region, and
rebuilds the pages when the moves fill that region; any other call folds the
pages back into the canonical CSR.  Every batch is checked against the C or
Python restatement of insert/3 (synctree.erl:189-209, sequential inserts,
last writer wins): top hash and entry count after every batch, every level's
entries, and after folding the segments themselves (get, compare).  Small
slack (st_debug_knob ST_DBG_PAGES) makes the tests cross moves and rebuilds;
ST_DBG_PAGE_DOWN = 2 makes every in-place merge that fits shift the entries
before its insert positions down into the page's head slack (1: when that
moves fewer bytes; the default, 0, never shifts down).
Needs an MI355X."""
import numpy as np
import pytest

import oracle_c as C
import synctree_ref as R
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


@pytest.mark.parametrize('segments,n0,batch,slack,check,down', [
    (1 << 16, 300_000, 4_000, 1, True, 0),      # H = 4, minimal slack: moves every batch, rebuilds
    (1 << 16, 300_000, 4_000, 25, True, 0),     # the default slack
    (1 << 20, 1_000_000, 20_000, 2, True, 0),   # H = 5, the config-5 geometry at 1/100 scale
    (4096, 500_000, 6_000, 25, True, 0),        # H = 3, ~120 entries a segment: pieces of kilobytes
    (1 << 16, 300_000, 4_000, 2, False, 0),     # the production merge (no checked stores), rebuilds and deletes
    (4096, 500_000, 6_000, 25, True, 2),        # every in-place merge that fits shifts down (head slack)
    (1 << 16, 300_000, 4_000, 2, False, 2),     # ... in the unchecked merge, with rebuilds
    (4096, 500_000, 6_000, 25, True, 1),        # down when that moves fewer bytes
])
def test_int_keys_stream_through_pages(segments, n0, batch, slack, check, down):
    rng = np.random.default_rng(segments ^ n0 ^ slack)
    keys = workload.keys_int63(n0 + 40 * batch, workload.SEED ^ 0xDE17A)
    dev = synctree_hip.DeviceTree(16, segments)
    ora = C.OTree(16, segments)
    assert dev.insert_int64(keys[:n0], _obj(range(n0))) == 0
    ora.bulk_load_int64(keys[:n0], _obj(range(n0)))
    dev.debug_knob(_lib.ST_DBG_PAGES, slack)
    dev.debug_knob(_lib.ST_DBG_PAGE_CHECK, 1 if check else 0)   # every page store bounds-checked, every page validated
    dev.debug_knob(_lib.ST_DBG_PAGE_DOWN, down)
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
    on, batches, builds, folds, moved, touched = dev.page_stats()
    assert touched > 0
    assert on == 1 and batches == 30 and folds == 0, dev.page_stats()
    assert moved > 0
    if slack <= 2:
        assert builds >= 2, dev.page_stats()                  # the append region filled and the pages were rebuilt
    _levels(dev, ora)
    # reads fold the pages first: the segments themselves are the reference's
    probe = [int(k) for k in keys[rng.integers(0, nxt, 300)]]
    assert dev.get_batch(probe) == [ora.get(k) for k in probe]
    assert dev.page_stats()[0] == 0 and dev.page_stats()[3] == 1
    assert dev.num_entries() == ora.num_entries()
    assert dev.verify()
    dev.rehash()
    _levels(dev, ora)
    # streaming again after the fold, then the full rehash straight after
    for b in range(3):
        idx = rng.integers(0, nxt, batch)
        assert dev.insert_int64(keys[idx], _obj(idx + 100, epoch=3)) == 0
        ora.insert_int64_seq(keys[idx], _obj(idx + 100, epoch=3))
    assert dev.page_stats()[0] == 1
    dev.rehash()   # the first full rehash after the batches hashes the pages' segments: no fold
    assert dev.page_stats()[0] == 1
    assert dev.top_hash() == ora.top_hash()
    _levels(dev, ora)
    # the repair path (riak_ensemble_peer_tree.erl:264-277): delete segment
    # nodes of a paged tree (the pages just empty them), then rehash/1 twice
    # (from the segments, then the tiled fused kernel)
    idx = rng.integers(0, nxt, batch)
    dev.debug_knob(_lib.ST_DBG_PAGES, slack)   # pages from this batch on (not only from the second of a run)
    assert dev.insert_int64(keys[idx], _obj(idx + 200, epoch=4)) == 0
    ora.insert_int64_seq(keys[idx], _obj(idx + 200, epoch=4))
    assert dev.page_stats()[0] == 1
    H1 = dev.height + 1
    for k in keys[idx[:3]]:
        seg = ora.segment_of(int(k))
        dev.delete_node(H1, seg)
        ora.delete_node(H1, seg)
    assert dev.page_stats()[0] == 1 and dev.num_entries() == ora.num_entries()
    ora.rehash()
    for _ in range(2):
        dev.rehash()
        assert dev.top_hash() == ora.top_hash()
    _levels(dev, ora)
    assert dev.get_batch([int(k) for k in keys[idx[:20]]]) == [ora.get(int(k)) for k in keys[idx[:20]]]
    dev.close()


def _same_segment_pairs(S, want):
    """(integer, float) key pairs that hash to one segment of S."""
    out = []
    for k in range(1, 20000):
        if R.get_segment(k, S) == R.get_segment(float(k), S):
            out.append((k, float(k)))
            if len(out) >= want:
                break
    return out


def _rand_bin(rng, lo, hi):
    return bytes(rng.integers(0, 256, int(rng.integers(lo, hi + 1)), dtype=np.uint8))


@pytest.mark.parametrize('slack,down', [(1, 0), (25, 0), (1, 2), (25, 2)])
def test_variable_keys_and_values_through_pages(slack, down):
    """Binary keys of 1..24 bytes and values of 0..40 bytes: overwrites that
    grow and shrink a value (tails moving right and left inside a page),
    empty values, segments outgrowing their pages."""
    rng = np.random.default_rng(77 + slack)
    S = 4096
    dev, ora = synctree_hip.DeviceTree(16, S), C.OTree(16, S)
    base = {}
    while len(base) < 20_000:
        base[_rand_bin(rng, 1, 24)] = _rand_bin(rng, 0, 40)
    ks = list(base)
    st = dev.insert_batch(ks, [base[k] for k in ks])
    assert all(x is None for x in st)
    ora.bulk_load(ks, [base[k] for k in ks])
    dev.debug_knob(_lib.ST_DBG_PAGES, slack)
    dev.debug_knob(_lib.ST_DBG_PAGE_CHECK, 1)   # every page store bounds-checked, every page validated
    dev.debug_knob(_lib.ST_DBG_PAGE_DOWN, down)
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
    assert dev.page_stats()[1] == 12 and dev.page_stats()[4] > 0
    _levels(dev, ora)
    probe = ks[::97]
    assert dev.get_batch(probe) == [ora.get(k) for k in probe]
    dev.close()


@pytest.mark.parametrize('down', [0, 2])
def test_uniform_pages_turning_mixed(down):
    """Int keys with 17-byte values: every page is UNIFORM (one key length,
    one value length: only its first and end offset slots are kept, pages.h).
    Batches that put a longer value, a shorter value or a binary key into
    such pages turn them mixed (their offsets are written first), interleaved with
    uniform batches; every batch against the C restatement of insert/3."""
    rng = np.random.default_rng(2024)
    S, n0 = 1 << 16, 300_000
    keys = workload.keys_int63(n0 + 200_000, workload.SEED ^ 0x0FF5E7)
    dev, ora = synctree_hip.DeviceTree(16, S), C.OTree(16, S)
    assert dev.insert_int64(keys[:n0], _obj(range(n0))) == 0
    ora.bulk_load_int64(keys[:n0], _obj(range(n0)))
    dev.debug_knob(_lib.ST_DBG_PAGES, 3)
    dev.debug_knob(_lib.ST_DBG_PAGE_CHECK, 1)
    dev.debug_knob(_lib.ST_DBG_PAGE_DOWN, down)
    nxt = n0
    for b in range(16):
        if b % 4 == 3:   # a mixed batch: other value lengths, term keys, overwrites of uniform entries
            old = [int(k) for k in keys[rng.integers(0, nxt, 200)]]
            bk = old + [b'k-%d-%d' % (b, j) for j in range(100)] + [int(k) for k in keys[nxt:nxt + 100]]
            nxt += 100
            bv = [_rand_bin(rng, 0, 40) for _ in bk]
            assert all(x is None for x in dev.insert_batch(bk, bv))
            for k, v in zip(bk, bv):
                ora.insert(k, v)
        else:            # a uniform batch: int keys, 17-byte values
            old = rng.integers(0, nxt, 2000)
            new = np.arange(nxt, nxt + 2000)
            nxt += 2000
            idx = rng.permutation(np.concatenate([old, new]))
            assert dev.insert_int64(keys[idx], _obj(idx + 7 + b, epoch=5)) == 0
            assert ora.insert_int64_seq(keys[idx], _obj(idx + 7 + b, epoch=5)) == 0
        assert dev.top_hash() == ora.top_hash(), 'top hash differs after batch %d' % b
        assert dev.num_entries() == ora.num_entries(), b
    assert dev.page_stats()[0] == 1 and dev.page_stats()[3] == 0
    _levels(dev, ora)
    probe = [int(k) for k in keys[rng.integers(0, nxt, 300)]]
    assert dev.get_batch(probe) == [ora.get(k) for k in probe]   # folds the pages (offsets from the stride)
    assert dev.verify()
    _levels(dev, ora)
    dev.close()


@pytest.mark.parametrize('down', [0, 2])
def test_equal_numbers_through_pages(down):
    """1 and 1.0 are ONE key (synctree.erl:206 orddict:store compares with
    ==): a streamed float form replaces the integer entry with a longer key
    record, and the integer form replaces it back -- key byte shifts of both
    signs inside a page.  Device vs synctree_ref (term keys)."""
    rng = np.random.default_rng(11)
    W, S = 4, 64
    ref = R.new(b'ref', W, S)
    dev = synctree_hip.DeviceTree(W, S)
    ks = list(range(3000))
    vs = [_rand_bin(rng, 0, 20) for _ in ks]
    for k, v in zip(ks, vs):
        ref = R.insert(k, v, ref)
    assert all(x is None for x in dev.insert_batch(ks, vs))
    dev.debug_knob(_lib.ST_DBG_PAGES, 5)
    dev.debug_knob(_lib.ST_DBG_PAGE_CHECK, 1)
    dev.debug_knob(_lib.ST_DBG_PAGE_DOWN, down)
    pairs = [(a, b) for a, b in _same_segment_pairs(S, 40) if isinstance(a, int) and a < 3000]
    assert len(pairs) >= 10
    for b in range(8):
        pick = [int(x) for x in rng.integers(0, 3000, 30)]
        same = [p[b % 2 == 0] for p in pairs[b % 3::3]]   # the float form, then the integer form back
        bk = same + pick + [('t', b, j) for j in range(10)]
        bv = [_rand_bin(rng, 0, 30) for _ in bk]
        assert all(x is None for x in dev.insert_batch(bk, bv))
        for k, v in zip(bk, bv):
            ref = R.insert(k, v, ref)
        assert dev.top_hash() == R.top_hash(ref), b
    assert dev.page_stats()[1] == 8
    segs = list(range(S))
    got = dev.exchange_get_batch(R.height(ref) + 1, segs)
    exp = [R.exchange_get(R.height(ref) + 1, s, ref) for s in segs]
    assert got == exp
    assert [repr(k) for g in got for k, _ in g] == [repr(k) for x in exp for k, _ in x]   # the stored form
    dev.close()


@pytest.mark.parametrize('pages', [True, False], ids=['pages', 'csr_merge'])
def test_corrupted_segment_rejects_streamed_keys(pages):
    """A corrupted segment (corrupt/2, synctree.erl:241-247) met by a streamed
    batch: its keys are refused with {corrupted, Level, Bucket} and the rest
    are inserted, as sequential insert/3 calls would do -- through the pages
    (the default) and with the pages off (every batch merged into the CSR)."""
    S, n0 = 1 << 16, 200_000
    keys = workload.keys_int63(n0 + 5000, workload.SEED ^ 0xC0)
    vals = _obj(range(n0 + 5000))
    dev, ora = synctree_hip.DeviceTree(16, S), C.OTree(16, S)
    assert dev.insert_int64(keys[:n0], vals[:n0]) == 0
    ora.bulk_load_int64(keys[:n0], vals[:n0])
    dev.debug_knob(_lib.ST_DBG_PAGE_CHECK, 1)
    dev.debug_knob(_lib.ST_DBG_PAGES, 0 if pages else -1)   # pages (from the first streamed batch) or none
    # a streamed batch, then corrupt a key's segment (corrupt/2 folds the pages)
    assert dev.insert_int64(keys[n0:n0 + 2000], vals[n0:n0 + 2000]) == 0
    ora.insert_int64_seq(keys[n0:n0 + 2000], vals[n0:n0 + 2000])
    assert dev.page_stats()[0] == (1 if pages else 0)
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
    if pages:
        dev.debug_knob(_lib.ST_DBG_PAGES, 0)   # corrupt/2 folded the pages: back on from this batch
    assert dev.insert_batch(bk, bv) == exp
    assert dev.page_stats()[0] == (1 if pages else 0)
    assert dev.top_hash() == ora.top_hash()
    _levels(dev, ora)
    assert dev.get_batch(bk[:50]) == [ora.get(k) for k in bk[:50]]
    dev.close()


def test_checked_mode_refuses_a_page_outside_its_capacity():
    """The checked mode (ST_DBG_PAGE_CHECK) against the defect class of round
    5's paged-merge fault (a page left pointing past its capacity, then
    indexed by the next batch's positions kernel): a poisoned page
    (ST_DBG_PAGE_POISON) is refused before the batch reads it -- ST_EDEVICE,
    the tree in error -- instead of an access outside the page arrays."""
    S, n0 = 1 << 16, 200_000
    keys = workload.keys_int63(n0 + 20_000, workload.SEED ^ 0x9015)
    dev = synctree_hip.DeviceTree(16, S)
    assert dev.insert_int64(keys[:n0], _obj(range(n0))) == 0
    dev.debug_knob(_lib.ST_DBG_PAGES, 10)
    dev.debug_knob(_lib.ST_DBG_PAGE_CHECK, 1)
    assert dev.insert_int64(keys[n0:n0 + 4000], _obj(range(4000))) == 0
    assert dev.page_stats()[0] == 1
    victim = dev.segments_of([int(keys[n0 + 5000])])[0]
    dev.debug_knob(_lib.ST_DBG_PAGE_POISON, victim)
    with pytest.raises(_lib.DeviceError, match='page check before the batch'):
        dev.insert_int64(keys[n0 + 4000:n0 + 8000], _obj(range(4000)))
    with pytest.raises(_lib.DeviceError):
        dev.top_hash()   # the tree refuses reads after a device error
    dev.close()
