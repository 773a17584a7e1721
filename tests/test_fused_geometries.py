"""The fused full rehash (k_rehash_fused: K1 + every inner level in one launch)
at every geometry it serves -- W = 16, H = 3..6 (4096 .. 2^24 segments) --
dense and sparse (empty segments, empty level-H nodes, empty windows), alone
(16 waves per window) and as a group (8 waves per window, two windows per
CU), every level's entries against the C restatement of synctree.erl:489-543.
Needs an MI355X."""
import numpy as np
import pytest

import oracle_c as C
from riak_ensemble_amd import synctree_hip, workload

pytestmark = pytest.mark.gpu


def _level_parity(dev, ora):
    assert dev.top_hash() == ora.top_hash()
    for lvl in range(1, dev.height + 2):
        pa, ha = dev.level_entries(lvl)
        pb, hb = ora.level_entries(lvl)
        assert (pa == pb).all(), 'presence differs at level %d' % lvl
        assert (ha[pa == 1] == hb[pb == 1]).all(), 'hashes differ at level %d' % lvl


def _pair(segments, n, seed, window_gaps=False):
    keys = workload.keys_int63(n, seed)
    if window_gaps:   # keep only keys outside every other window: whole empty windows
        ora0 = C.OTree(16, segments)
        segs = np.array([ora0.segment_of(int(k)) for k in keys.tolist()], np.int64)
        keys = keys[(segs // 4096) % 2 == 0]
    vals = workload.obj_hash_values(len(keys))
    ora = C.OTree(16, segments).bulk_load_int64(keys, vals)
    dev = synctree_hip.DeviceTree(16, segments)
    assert dev.insert_int64(keys, vals) == 0
    return dev, ora


@pytest.mark.parametrize('segments,n', [
    (4096, 60_000),          # H = 3: one window, no levels above it
    (4096, 900),             # H = 3, sparse: empty segments and level-H nodes
    (1 << 16, 1_000_000),    # H = 4: 16 windows, one level above
    (1 << 16, 20_000),       # H = 4, sparse
    (1 << 20, 300_000),      # H = 5, sparse (the config-4 shape is 1M keys)
    (1 << 24, 2_000_000),    # H = 6: 4096 windows, three levels above
])
def test_fused_rehash_geometry(segments, n):
    dev, ora = _pair(segments, n, workload.SEED ^ segments ^ n)
    assert dev.height == ora.height
    for _ in range(2):   # the first full rehash after the inserts hashes from the CSR, the second is the fused one
        dev.rehash()
        _level_parity(dev, ora)
    assert dev.verify() and dev.verify(upper=True)
    dev.close()


def test_fused_rehash_empty_windows():
    dev, ora = _pair(1 << 20, 200_000, workload.SEED ^ 77, window_gaps=True)
    for _ in range(2):   # the first full rehash after the inserts hashes from the CSR, the second is the fused one
        dev.rehash()
        _level_parity(dev, ora)
    dev.close()


def test_group_rehash_mixed_density():
    """st_rehash_group: trees of one geometry with different densities in ONE
    launch (8-wave windows, two per CU); each tree equals its own oracle."""
    pairs = [_pair(1 << 16, n, workload.SEED ^ (n + 5)) for n in (500_000, 3_000, 40_000, 1)]
    synctree_hip.rehash_group([d for d, _ in pairs])
    for dev, ora in pairs:
        _level_parity(dev, ora)
    synctree_hip.rehash_group([d for d, _ in pairs])   # self-resetting counters: again
    for dev, ora in pairs:
        _level_parity(dev, ora)
        dev.close()


@pytest.mark.parametrize('segments,skip', [(1 << 20, 37), (1 << 16, 15)])
def test_mailbox_timeout_is_a_device_error(segments, skip):
    """A window root's mailbox entry that never arrives (fault injection:
    st_debug_knob ST_DBG_SKIP_MAIL) must not become a stale entry hashed into
    the top hash: the bounded wait raises the tree's device-error word, the
    call that waits for the launch reports ST_EDEVICE, reads are refused, and
    a clean full rehash makes the tree readable again with the right hashes."""
    from riak_ensemble_amd import _lib
    dev, ora = _pair(segments, 100_000, workload.SEED ^ 0xB0B ^ segments)
    dev.rehash()
    _level_parity(dev, ora)
    dev.debug_knob(_lib.ST_DBG_SKIP_MAIL, skip)
    dev.rehash()                      # asynchronous: the launch is enqueued
    with pytest.raises(_lib.DeviceError, match='mailbox'):
        dev.sync()                    # the call that waits reports it
    with pytest.raises(_lib.DeviceError):
        dev.top_hash()                # no top hash from a tree in error
    with pytest.raises(_lib.DeviceError):
        dev.level_entries(2)
    # the per-key path right after a faulted rehash: k_small must not read
    # the invalid upper levels (get/2, insert/3 report the device error)
    probe = int(workload.keys_int63(1, workload.SEED ^ 0xB0B ^ segments)[0])
    for op in (lambda: dev.get1(probe), lambda: dev.insert1(probe, b'x' * 17)):
        dev.debug_knob(_lib.ST_DBG_SKIP_MAIL, -1)
        dev.rehash()                  # clean: the tree is readable again
        assert dev.get1(probe) == ora.get(probe)
        dev.debug_knob(_lib.ST_DBG_SKIP_MAIL, skip)
        dev.rehash()                  # faulted, and not waited for
        with pytest.raises(_lib.DeviceError, match='mailbox'):
            op()
        with pytest.raises(_lib.DeviceError):
            dev.get1(probe)           # and the tree stays in error
    dev.debug_knob(_lib.ST_DBG_SKIP_MAIL, -1)
    dev.rehash()                      # a clean full rehash clears the error
    dev.sync()
    _level_parity(dev, ora)
    # the group rehash hands no window root over through a mailbox (its
    # levels above level H are launches of their own, k_level16_group): the
    # knob leaves it untouched, and both trees get their oracle's levels
    other, ora2 = _pair(segments, 50_000, workload.SEED ^ 0xB0C ^ segments)
    dev.debug_knob(_lib.ST_DBG_SKIP_MAIL, skip)
    synctree_hip.rehash_group([other, dev])
    _level_parity(dev, ora)
    _level_parity(other, ora2)
    dev.debug_knob(_lib.ST_DBG_SKIP_MAIL, -1)
    synctree_hip.rehash_group([other, dev])
    _level_parity(dev, ora)
    _level_parity(other, ora2)
    dev.close()
    other.close()
