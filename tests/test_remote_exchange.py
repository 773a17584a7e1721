"""Streaming exchange across a process boundary (SURVEY §8f rank 3;
riak_ensemble_amd/remote.py).  The remote tree lives in another process; the
local side runs synctree:compare/3 (src/synctree.erl:372-417) with a remote
fun that sends ONE start_exchange_level request per level and serves the
level's exchange_get calls from the reply (test/synctree_remote.erl:25-66).

CPU: the protocol against the Python restatement on both sides (oracle/, the
checker), including the exact order of test/synctree_remote.erl:37-39.
GPU: device trees on both sides -- the remote process answers each level with
one batched device call -- against the C restatement's compare, with filters,
single-bucket fallback and a corrupted remote (the reference's
function_clause in orddict_delta)."""
import numpy as np
import pytest

import synctree_ref as R
from riak_ensemble_amd import remote, workload


class _RefTree:
    """Remote tree for the CPU test: the Python restatement (checker)."""

    def __init__(self, n):
        self.t = R.build(n)

    def exchange_get_batch(self, level, buckets):
        return [R.exchange_get(level, b, self.t) for b in buckets]


def _ref_tree(n):
    return _RefTree(n)


def test_streaming_protocol_exact_order_cpu():
    from riak_ensemble_amd import synctree as S
    a = R.build(10)

    def local(op, arg):
        return R.exchange_get(arg[0], arg[1], a) if op == 'exchange_get' else 'ok'

    with remote.RemoteTree(_ref_tree, (6,)) as rt:
        got = S.compare(R.height(a), local, rt.fun)
        levels = list(rt.levels)
        requests = rt.requests
    assert got == R.expected_diff(10, 4)          # test/synctree_remote.erl:37-39
    assert [lvl for lvl, _ in levels] == list(range(R.height(a) + 2))
    assert requests == len(levels)                # one message per level, no per-bucket calls
    assert rt.stats[0] == len(levels)


# ------------------------------------------------------------------ GPU
def _kv(n, seed, epoch=1):
    keys = workload.keys_int63(n, seed)
    vals = workload.obj_hash_values(n, epoch=epoch)
    return keys, vals


def _device_tree(n, seed, mutate, corrupt_key):
    """Runs in the remote process: a device tree of n keys, every 97th value
    changed and 300 extra keys when `mutate`, optionally one corrupted key."""
    from riak_ensemble_amd import synctree as S
    keys, vals = _kv(n, seed)
    t = S.new(None)
    t.modstate.insert_int64(keys, vals)
    t = S._after_top_change(t)
    if mutate:
        ks = [int(k) for k in keys[::97]]
        vs = [bytes([0]) + (2).to_bytes(8, 'big') + i.to_bytes(8, 'big') for i in range(len(ks))]
        ek, ev = _kv(300, seed ^ 0x77, epoch=3)
        t, st = S.insert_batch(list(zip(ks + [int(k) for k in ek], vs + [bytes(v) for v in ev])), t)
        assert all(x is None for x in st)
    if corrupt_key is not None:
        t = S.corrupt(corrupt_key, t)
    return t


def _oracle_pair(n, seed):
    import oracle_c as C
    keys, vals = _kv(n, seed)
    a = C.OTree().bulk_load_int64(keys, vals)
    b = C.OTree().bulk_load_int64(keys, vals)
    ks = [int(k) for k in keys[::97]]
    vs = np.array([list(bytes([0]) + (2).to_bytes(8, 'big') + i.to_bytes(8, 'big')) for i in range(len(ks))], np.uint8)
    b.insert_int64_seq(np.array(ks, np.int64), vs)
    ek, ev = _kv(300, seed ^ 0x77, epoch=3)
    b.insert_int64_seq(ek, ev)
    return a, b


@pytest.mark.gpu
def test_streaming_exchange_device_trees_across_processes():
    from riak_ensemble_amd import synctree as S
    n, seed = 100_000, workload.SEED ^ 0x3131
    keys, vals = _kv(n, seed)
    a = S.new(None)
    a.modstate.insert_int64(keys, vals)
    a = S._after_top_change(a)
    oa, ob = _oracle_pair(n, seed)
    with remote.RemoteTree(_device_tree, (n, seed, True, None)) as rt:
        for opts in ((), ('local_only',), ('remote_only',)):
            rt.levels.clear()
            before = rt.requests
            got = S.compare(S.height(a), S.direct_exchange(a), rt.fun, None, list(opts))
            assert got == oa.compare(ob, opts), opts
            assert rt.requests - before == len(rt.levels) <= S.height(a) + 2   # one message per level
        # a bucket that was not announced: one single-bucket request (the reference's fallback)
        before = rt.requests
        img = rt.fun('exchange_get', (S.height(a) + 1, 5))
        assert rt.requests == before + 1
        assert img == ob.node(S.height(a) + 1, 5)
    # exact order of test/synctree_remote.erl:37-39 with device trees on both sides
    with remote.RemoteTree(_pure_build, (6,)) as rt:
        a10 = _pure_build(10)
        assert S.compare(S.height(a10), S.direct_exchange(a10), rt.fun) == R.expected_diff(10, 4)


def _pure_build(n):
    """test/synctree_pure.erl:70-80 on the device path."""
    from riak_ensemble_amd import synctree as S
    t = S.new(None)
    for k in range(n, 0, -1):
        t = S.insert(k, (k * 10).to_bytes(8, 'big'), t)
    return t


@pytest.mark.gpu
def test_streaming_exchange_corrupted_remote_crashes():
    """A corrupted remote segment: its exchange_get is {corrupted, L, B} and
    orddict_delta has no clause for it (riak_ensemble_exchange.erl:27-29
    reports exchange_failed); the reference crashes, so does this."""
    from riak_ensemble_amd import synctree as S
    n, seed = 20_000, workload.SEED ^ 0x3232
    keys, vals = _kv(n, seed)
    a = S.new(None)
    a.modstate.insert_int64(keys, vals)
    a = S._after_top_change(a)
    with remote.RemoteTree(_device_tree, (n, seed, True, int(keys[97]))) as rt:
        with pytest.raises(S.SynctreeCrash):
            S.compare(S.height(a), S.direct_exchange(a), rt.fun)
