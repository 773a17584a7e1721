"""Exchange diff application: riak_ensemble_exchange.erl
:71-97 + valid_obj_hash (riak_ensemble_peer.erl:1726-1729), device batch
(st_exchange_apply) vs the CPU restatement oracle/exchange_ref.py."""
import numpy as np
import pytest

import exchange_ref as X
import oracle_c as C
from riak_ensemble_amd import workload


def obj(epoch, seq, prefix=0):
    return bytes([prefix]) + epoch.to_bytes(8, 'big') + seq.to_bytes(8, 'big')


def _pair(n=2000, crash_at=None):
    """local: keys[0 : 0.9n]; remote: keys[0.1n : n]; remote newer on
    [0.1n, 0.2n), local newer on [0.2n, 0.3n); equal elsewhere."""
    keys = [int(k) for k in workload.keys_int63(n)]
    loc, rem = {}, {}
    for i, k in enumerate(keys):
        if i < 0.9 * n:
            loc[k] = obj(2 if 0.2 * n <= i < 0.3 * n else 1, i)
        if i >= 0.1 * n:
            rem[k] = obj(1, i + 5 if i < 0.2 * n else i)
    if crash_at is not None:
        rem[keys[crash_at]] = obj(1, crash_at + 7, prefix=1)   # not <<?H_OBJ_NONE,_>>
    return keys, loc, rem


def _otree(d):
    t = C.OTree()
    for k, v in d.items():
        t.insert(k, v)
    return t


def test_oracle_semantics():
    n = 2000
    keys, loc, rem = _pair(n)
    a, b = _otree(loc), _otree(rem)
    st, nd, na = X.exchange_apply(a, b)
    # 0.1n local-only + 0.1n remote-newer + 0.1n local-newer + 0.1n remote-only
    assert st == 'ok' and nd == 4 * n // 10 and na == 2 * n // 10
    exp = dict(loc)
    for i, k in enumerate(keys):
        if 0.1 * n <= i < 0.2 * n or i >= 0.9 * n:
            exp[k] = rem[k]
    assert a.top_hash() == _otree(exp).top_hash()
    # equal hashes are "newer or equal": an identical tree applies nothing
    assert X.exchange_apply(_otree(rem), _otree(rem))[2] == 0


def test_oracle_crash_is_partial():
    keys, loc, rem = _pair(2000, crash_at=500)
    a, b = _otree(loc), _otree(rem)
    diffs = a.compare(b)
    idx = [k for k, _ in diffs].index(keys[500])
    st, nd, na = X.exchange_apply(a, b)
    assert st == 'exchange_failed'
    before = diffs[:idx]
    assert na == sum(1 for _, (x, y) in before if x == '$none' or (y != '$none' and y >= x))


def _dev(d):
    from riak_ensemble_amd import synctree_hip
    t = synctree_hip.DeviceTree()
    ks = list(d)
    t.insert_batch(ks, [d[k] for k in ks])
    return t


@pytest.mark.gpu
@pytest.mark.parametrize('crash_at', [None, 1500, 50])
def test_device_exchange_apply(crash_at):
    n = 20000
    keys, loc, rem = _pair(n, crash_at)
    oa, ob = _otree(loc), _otree(rem)
    da, db = _dev(loc), _dev(rem)
    assert da.top_hash() == oa.top_hash() and db.top_hash() == ob.top_hash()
    st, nd, na = X.exchange_apply(oa, ob)
    r = da.exchange_apply(db)
    assert r[0] == st and r[1]['diffs'] == nd and r[1]['applied'] == na
    assert da.top_hash() == oa.top_hash()
    assert da.verify()
    # applying again converges: only local-only and local-newer diffs remain
    if crash_at is None:
        r2 = da.exchange_apply(db)
        assert r2[0] == 'ok' and r2[1]['applied'] == 0 and r2[1]['diffs'] == 2 * n // 10
