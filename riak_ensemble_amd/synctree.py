"""riak_ensemble_amd.synctree — the reference ``synctree`` module API
(src/synctree.erl:77-86) on the MI355X device path.

Same function names, argument meaning and results as the Erlang module:

    T  = new(Id, Width, Segments, Mod, Opts)        # Mod: synctree_hip
    T2 = insert(Key, Value, T)     -> tree | ('corrupted', Level, Bucket)
    get(Key, T)                    -> Value | 'notfound' | ('corrupted', L, B)
    exchange_get(Level, Bucket, T) -> orddict | ('corrupted', L, B)
    compare(Height, Local, Remote[, AccFun[, Opts]]), local_compare(T1, T2)
    rehash(T), rehash_upper(T), verify(T), verify_upper(T), top_hash(T),
    height(T), corrupt(Key, T), m_batch(Update, T), m_flush(T)

Trees live in device memory (HBM).  Like the ETS backend (the reference's
default, synctree.erl:144-145), every record of one tree shares the stored
nodes, while each record value carries its own ``top_hash`` field — the
device is told which top hash the record in hand holds before every
verified operation, so stale records behave exactly as in Erlang.
Where the reference crashes, :class:`SynctreeCrash` (or ``TypeError`` /
``ValueError`` for bad arguments) is raised.

Bulk extensions (device-native, same semantics as repeated calls):
``insert_batch``, ``get_batch``, ``exchange_get_batch``.
"""
from . import _lib
from . import synctree_hip
from . import terms

WIDTH = 16                # synctree.erl:88
SEGMENTS = 1024 * 1024    # synctree.erl:89
NOTFOUND, UNDEFINED, NONE, CORRUPTED = terms.NOTFOUND, terms.UNDEFINED, terms.NONE, terms.CORRUPTED


class SynctreeCrash(Exception):
    """Where src/synctree.erl raises (function_clause, case_clause, badmatch)."""


class Tree:
    """The #tree{} record (synctree.erl:103-114); functional updates."""
    __slots__ = ('id', 'width', 'segments', 'height', 'shift', 'shift_max', 'top_hash', 'buffer', 'buffered',
                 'mod', 'modstate')

    def replace(self, **kw):
        t = Tree()
        for s in Tree.__slots__:
            setattr(t, s, kw[s] if s in kw else getattr(self, s))
        return t

    def __repr__(self):
        th = self.top_hash if isinstance(self.top_hash, str) else self.top_hash.hex()
        return '#tree{id=%r, width=%d, segments=%d, top_hash=%s}' % (self.id, self.width, self.segments, th)


def _device_state(t):
    if t.mod is not synctree_hip:
        raise ValueError('riak_ensemble_amd.synctree runs on the device backend (synctree_hip) only')
    return t.modstate


def _sync_record(t):
    """Make the device's #tree.top_hash slot hold this record's value."""
    st = _device_state(t)
    if getattr(st, '_rec_top', None) != t.top_hash:
        st.set_record_top(t.top_hash)
        st._rec_top = t.top_hash


def _after_top_change(t):
    st = t.modstate
    top = st.top_hash()
    st._rec_top = top
    return t.replace(top_hash=top)


# ---------------------------------------------------------------- construction
def newdb(id_, opts=()):
    """synctree.erl:127-133 — the persistent-backend constructor.  The device
    tree stands in for synctree_leveldb; with opts ``leveldb`` (the DB's
    records: a dict or (key, value) pairs) and ``tree_id`` (binary) it opens
    the tree those records hold, as synctree_leveldb:new/1 + reload_top_hash
    would (synctree_leveldb.erl:59-64, synctree.erl:172-175)."""
    return new(id_, 'default', 'default', synctree_hip, opts)


def checkpoint(t, tree_id=b''):
    """The synctree_leveldb records of tree t (src/synctree_leveldb.erl:104-152),
    encoded on the device: [(DbKey, term_to_binary(Node))] to write into the
    peer's LevelDB."""
    return _device_state(t).snapshot_leveldb(tree_id)


def checkpoint_into(t, db, tree_id=b''):
    """Checkpoint tree t into an existing DB (a dict standing in for the peer's
    LevelDB): one write batch that deletes this tree's records the new
    snapshot no longer holds -- nodes emptied and deleted by rehash since the
    last checkpoint (synctree.erl:529-531) -- and puts every record of the
    snapshot.  Returns the number of deletes."""
    recs = checkpoint(t, tree_id)
    new_keys = {k for k, _ in recs}
    prefix = bytes([0]) + bytes(tree_id)
    height = _device_state(t).height
    stale = [k for k in db if k.startswith(prefix) and k not in new_keys and _is_tree_key(k, prefix, height)]
    for k in stale:
        del db[k]
    db.update(recs)
    return len(stale)


def _is_tree_key(k, prefix, height):
    """Could db_key(Id, Level, Bucket) of this tree have produced k?
    (<<0, Id, Level:8, encode_unsigned(Bucket)>>, synctree_leveldb.erl:104-109)"""
    rest = k[len(prefix):]
    return len(rest) >= 2 and rest[0] <= height + 1 and (len(rest) == 2 or rest[1] != 0)


def new(id_=None, width='default', segments='default', mod=synctree_hip, opts=()):
    """synctree.erl:135-170 (+ reload_top_hash, 172-175)."""
    if width == 'default':
        width = WIDTH
    if segments == 'default':
        segments = SEGMENTS
    if mod is not synctree_hip:
        raise ValueError('backend %r is not a device backend' % (mod,))
    o = dict(opts) if opts else {}
    records = o.pop('leveldb', None)
    tree_id = o.pop('tree_id', b'')
    o.update(width=width, segments=segments)
    try:
        state = mod.new(o)
    except ValueError as e:
        raise SynctreeCrash('case_clause in compute_height/compute_shift: %s' % e)
    if records is not None:
        if isinstance(records, dict):
            records = list(records.items())
        state.restore_leveldb(records, tree_id)
    t = Tree()
    t.id = id_
    t.width = state.width
    t.segments = state.segments
    t.height = state.height
    t.shift = state.shift
    t.shift_max = state.shift * state.height
    t.buffer = []
    t.buffered = 0
    t.mod = mod
    t.modstate = state
    top = state.fetch_batch(0, [0])[0]
    t.top_hash = top
    state._rec_top = None
    return t


def height(t):
    return t.height


def top_hash(t):
    return t.top_hash


# ---------------------------------------------------------------- insert / get
def insert(key, value, t):
    """synctree.erl:189-199."""
    if not isinstance(value, (bytes, bytearray)):
        raise SynctreeCrash('function_clause: synctree:insert/3 needs a binary value')
    _sync_record(t)
    st = t.modstate.insert_batch([key], [bytes(value)])[0]
    if st is not None:
        return st
    return _after_top_change(t)


def insert_batch(kvs, t):
    """N inserts in order (last writer wins).  Returns (Tree, [None |
    ('corrupted', L, B) per key])."""
    kvs = list(kvs)
    for _, v in kvs:
        if not isinstance(v, (bytes, bytearray)):
            raise SynctreeCrash('function_clause: synctree:insert/3 needs a binary value')
    if not kvs:
        return t, []
    _sync_record(t)
    status = t.modstate.insert_batch([k for k, _ in kvs], [bytes(v) for _, v in kvs])
    if all(s is not None for s in status):
        return t, status
    return _after_top_change(t), status


def get(key, t):
    """synctree.erl:213-227."""
    if t.top_hash == UNDEFINED:
        return NOTFOUND
    _sync_record(t)
    return t.modstate.get_batch([key])[0]


def get_batch(keys, t):
    if t.top_hash == UNDEFINED:
        return [NOTFOUND for _ in keys]
    _sync_record(t)
    return t.modstate.get_batch(list(keys))


def exchange_get(level, bucket, t):
    """synctree.erl:231-237."""
    if level == 0 and bucket == 0:
        return [(0, t.top_hash)]
    if level < 1 or level > t.height + 1:
        raise SynctreeCrash('badarg: no level %r' % (level,))
    _sync_record(t)
    return t.modstate.exchange_get_batch(level, [bucket])[0]


def exchange_get_batch(level, buckets, t):
    """Batched exchange_get for one level (the streaming start_exchange_level
    protocol of test/synctree_remote.erl:25-35)."""
    if level == 0:
        return [[(0, t.top_hash)] for _ in buckets]
    _sync_record(t)
    return t.modstate.exchange_get_batch(level, list(buckets))


def corrupt(key, t):
    """synctree.erl:241-247."""
    _device_state(t).corrupt(key)
    return t


# ---------------------------------------------------------------- buffer (synctree.erl:453-485)
def m_batch(update, t):
    t2 = t.replace(buffer=[update] + t.buffer, buffered=t.buffered + 1)
    if t2.buffered > 200:
        return m_flush(t2)
    return t2


def m_flush(t):
    updates = list(reversed(t.buffer))
    synctree_hip.store_batch(updates, _device_state(t))
    return t.replace(buffer=[], buffered=0)


# ---------------------------------------------------------------- rehash / verify
def rehash_upper(t):
    """synctree.erl:489-491."""
    if t.height == 0:
        raise SynctreeCrash('rehash_upper/1 at Height 0 does not terminate in the reference')
    t = m_flush(t)
    _device_state(t).rehash(upper=True)
    return _after_top_change(t)


def rehash(t):
    """synctree.erl:493-509."""
    t = m_flush(t)
    _device_state(t).rehash(upper=False)
    return _after_top_change(t)


def verify_upper(t):
    """synctree.erl:549-551."""
    if t.height == 0:
        raise SynctreeCrash('verify_upper/1 at Height 0 crashes in the reference')
    _sync_record(t)
    return t.modstate.verify(upper=True)


def verify(t):
    """synctree.erl:553-555."""
    _sync_record(t)
    return t.modstate.verify(upper=False)


# ---------------------------------------------------------------- exchange (synctree.erl:354-449)
def direct_exchange(t):
    """synctree.erl:354-359."""
    def f(op, arg):
        if op == 'exchange_get':
            return exchange_get(arg[0], arg[1], t)
        return 'ok'
    f._st_tree = t
    return f


def local_compare(t1, t2):
    """synctree.erl:361-368."""
    return compare(height(t1), direct_exchange(t1), direct_exchange(t2))


def filter_type(opts):
    """synctree.erl:421-432."""
    lo = 'local_only' in opts
    ro = 'remote_only' in opts
    if lo and ro:
        raise SynctreeCrash('case_clause: both local_only and remote_only')
    return 'local_only' if lo else ('remote_only' if ro else 'all')


_FILTER_CODE = {'all': _lib.ST_FILTER_ALL, 'local_only': _lib.ST_FILTER_LOCAL_ONLY,
                'remote_only': _lib.ST_FILTER_REMOTE_ONLY}


def compare(height_, local, remote, accfun=None, opts=()):
    """synctree.erl:372-382.  accfun=None is the default ``Keys ++ Acc``.

    Two direct_exchange funs over device trees of the same shape run the whole
    level-synchronous diff on the GPU (kernel K3).  Any other pair of funs
    (e.g. a remote peer behind message passing) runs the same algorithm with
    each level's buckets fetched through the funs."""
    filt = filter_type(opts)
    ta, tb = getattr(local, '_st_tree', None), getattr(remote, '_st_tree', None)
    if (accfun is None and ta is not None and tb is not None and ta.mod is synctree_hip and tb.mod is synctree_hip
            and ta.width == tb.width and ta.segments == tb.segments and height_ == ta.height
            and ta.modstate.device == tb.modstate.device):
        _sync_record(ta)
        _sync_record(tb)
        r = ta.modstate.compare(tb.modstate, _FILTER_CODE[filt])
        if r[0] == 'corrupted':
            raise SynctreeCrash('function_clause in riak_ensemble_util:orddict_delta/3: %s exchange_get returned %r'
                                % (r[1], r[2]))
        return [(k, vv) for _, k, vv in r[1]]
    return _compare_generic(height_, local, remote, accfun, filt)


def _fetch_level(fn, level, buckets):
    t = getattr(fn, '_st_tree', None)
    if t is not None and level > 0:
        return exchange_get_batch(level, buckets, t)
    return [fn('exchange_get', (level, b)) for b in buckets]


def _delta(a, b):
    if not isinstance(a, list) or not isinstance(b, list):
        raise SynctreeCrash('function_clause in riak_ensemble_util:orddict_delta/3: %r / %r' % (a, b))
    return orddict_delta(a, b)


def _apply_filter(kind, delta):
    if kind == 'all':
        return delta
    if kind == 'local_only':
        return [d for d in delta if d[1][1] != NONE]
    return [d for d in delta if d[1][0] != NONE]


def _compare_generic(height_, local, remote, accfun, filt):
    final = height_ + 1
    acc = []
    level, diff = 0, [0]
    while diff:
        remote('start_exchange_level', (level, diff))
        a = _fetch_level(local, level, diff)
        b = _fetch_level(remote, level, diff)
        if level == final:
            for x, y in zip(a, b):
                d = _apply_filter(filt, _delta(x, y))
                acc = (d + acc) if accfun is None else accfun(d, acc)
            return acc
        nxt = []
        for x, y in zip(a, b):
            nxt.extend(k for k, _ in _apply_filter(filt, _delta(x, y)))
        diff = nxt
        level += 1
    return acc


def orddict_delta(d1, d2):
    """riak_ensemble_util.erl:115-141 (merge-join in Erlang term order)."""
    out = []
    i = j = 0
    while i < len(d1) and j < len(d2):
        k1, v1 = d1[i]
        k2, v2 = d2[j]
        a, b = _okey(k1), _okey(k2)
        if a < b:
            out.append((k1, (v1, NONE)))
            i += 1
        elif a > b:
            out.append((k2, (NONE, v2)))
            j += 1
        else:
            if v1 != v2:
                out.append((k1, (v1, v2)))
            i += 1
            j += 1
    out.extend((k, (v, NONE)) for k, v in d1[i:])
    out.extend((k, (NONE, v)) for k, v in d2[j:])
    return out


def _okey(k):
    return terms.order_sk(k)   # Erlang-equal keys (1, 1.0) compare equal
