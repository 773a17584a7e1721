"""CPU restatement of the exchange's diff application — TEST INFRASTRUCTURE
ONLY (the checker for st_exchange_apply; never imported by the product).

riak_ensemble_exchange.erl:71-97: compare(Height, Local, Remote) with default
options, then for each diff in list order
    {Key, {'$none', B}} -> riak_ensemble_peer_tree:insert(Key, B, Tree)
    {_Key, {_, '$none'}} -> ok
    {Key, {A, B}}       -> insert(Key, B) iff valid_obj_hash(B, A)
valid_obj_hash (riak_ensemble_peer.erl:1726-1729) has one clause, for two
<<?H_OBJ_NONE, _/binary>> hashes (?H_OBJ_NONE = 0), returning B >= A (Erlang
binary order: bytewise, then length); any other pair raises function_clause,
which ends the list comprehension (the diffs before it are applied).
"""

NONE = '$none'


def _valid_obj_hash(actual, known):
    if not (actual[:1] == b'\x00' and known[:1] == b'\x00'):
        raise ValueError('function_clause')
    return actual >= known   # Python bytes order == Erlang binary order


def exchange_apply(local, remote):
    """local/remote: oracle trees with .compare(other) and .insert(key, value)
    (oracle_c.OTree or synctree_ref via an adapter).  Returns
    (status, n_diffs, n_applied) with status 'ok' | 'exchange_failed' |
    ('crash', side, corrupted_tuple) when the compare crashes."""
    diffs = local.compare(remote)
    if isinstance(diffs, tuple):
        return (diffs, 0, 0)
    applied = 0

    def ins(key, value):
        r = local.insert(key, value)   # a corrupted path: insert refused, ignored
        return 0 if isinstance(r, tuple) else 1

    for key, (a, b) in diffs:
        if a == NONE:
            applied += ins(key, b)
        elif b == NONE:
            continue
        else:
            try:
                take = _valid_obj_hash(b, a)
            except ValueError:
                return ('exchange_failed', len(diffs), applied)
            if take:
                applied += ins(key, b)
    return ('ok', len(diffs), applied)
