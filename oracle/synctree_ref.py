"""CPU restatement of riak_ensemble's synctree — TEST INFRASTRUCTURE ONLY.

This module is the Python half of the parity oracle (see oracle/README.md and
DESIGN.md §Oracle).  It is a literal, slow, single-threaded restatement of the
Erlang reference so that the HIP product path can be checked against it.  It
must only be imported by ``tests/``, ``__graft_entry__.smoke()`` and the
``cpu_baseline`` leg of ``bench.py``; the product package never imports it.

Every function cites the reference line it restates
(paths relative to the reference checkout, jrwest/riak_ensemble):

* tree geometry / record .......... src/synctree.erl:88-89, 103-114, 151-175, 270-284
* insert / update_path ............ src/synctree.erl:189-209
* get ............................. src/synctree.erl:213-227
* exchange_get / verified_hashes .. src/synctree.erl:231-237, 288-298
* corrupt ......................... src/synctree.erl:241-247
* get_segment / hash / ensure_bin . src/synctree.erl:251-268
* get_path / verify_hash .......... src/synctree.erl:302-348
* exchange / compare .............. src/synctree.erl:354-449
* m_* buffer ...................... src/synctree.erl:453-485
* rehash / rehash_upper ........... src/synctree.erl:489-543
* verify / verify_upper ........... src/synctree.erl:549-571
* orddict_delta ................... src/riak_ensemble_util.erl:115-141
* ETS backend ..................... src/synctree_ets.erl:32-66
* orddict backend ................. src/synctree_orddict.erl:32-66

Erlang terms are modelled as: integers -> ``int``, floats -> ``float``,
binaries -> ``bytes``, atoms -> ``str``, tuples -> ``tuple``, proper lists ->
``list``, maps -> any ``collections.abc.Mapping`` (its ``items()``).  Erlang
term order (ERTS): number < atom < tuple < map < nil < list < bitstring;
numbers by value (an integer and a float compare as numbers), atoms by their
text, tuples by size then elements, maps by size, then their keys in map-key
order, then their values in that order (map keys compare exactly: every
integer before every float, 1 =/= 1.0 -- the ERTS "Term Comparisons" rules),
lists element-wise with a prefix first, binaries bytewise with a prefix
first.  Keys outside
integer/atom/binary are hashed through term_to_binary (synctree.erl:267-268),
restated below from the ERTS external term format (ETF_ATOMS selects the OTP
era of atom encoding: 'latin1' = before OTP 26, 'utf8' = OTP 26+).

Parity of the hash bytes is pinned by RFC 1321 (MD5 via ``hashlib``) and the
reference's own tests (test/synctree_pure.erl, test/synctree_remote.erl);
see tests/test_oracle_ref.py.
"""

import hashlib
import math
from collections.abc import Mapping

WIDTH = 16                     # synctree.erl:88
SEGMENTS = 1024 * 1024         # synctree.erl:89
H_MD5 = 0                      # synctree.erl:121
NONE = '$none'                 # riak_ensemble_util.erl:110-113
UNDEFINED = 'undefined'
NOTFOUND = 'notfound'
CORRUPTED = 'corrupted'

_TYPE_RANK_NUMBER = 0
_TYPE_RANK_ATOM = 1
_TYPE_RANK_TUPLE = 6
_TYPE_RANK_MAP = 7
_TYPE_RANK_NIL = 8
_TYPE_RANK_LIST = 9
_TYPE_RANK_BITSTRING = 10

ETF_ATOMS = 'latin1'


class ErlangCrash(Exception):
    """Raised where the reference would crash (function_clause, case_clause...)."""


# --------------------------------------------------------------------------
# Term helpers

def term_key(t):
    """Sort key realising Erlang term order (ERTS) on the modelled terms."""
    if isinstance(t, bool):
        raise ErlangCrash('booleans are atoms in Erlang; pass "true"/"false"')
    if isinstance(t, (int, float)):
        return (_TYPE_RANK_NUMBER, t)
    if isinstance(t, str):
        return (_TYPE_RANK_ATOM, t.encode('utf-8'))
    if isinstance(t, tuple):
        return (_TYPE_RANK_TUPLE, len(t), tuple(term_key(e) for e in t))
    if isinstance(t, list):
        if not t:
            return (_TYPE_RANK_NIL,)
        return (_TYPE_RANK_LIST, [term_key(e) for e in t])
    if isinstance(t, (bytes, bytearray)):
        return (_TYPE_RANK_BITSTRING, bytes(t))
    if isinstance(t, Mapping):
        items = _map_items(t)
        return (_TYPE_RANK_MAP, len(items), tuple(exact_term_key(k) for k, _ in items),
                tuple(term_key(v) for _, v in items))
    raise ErlangCrash('term outside the restated domain: %r' % (t,))


def exact_term_key(t):
    """Sort key of the exact order map keys compare in (=:=): numbers split
    by type, integers first; everything under the key compares exactly."""
    if isinstance(t, bool):
        raise ErlangCrash('booleans are atoms in Erlang; pass "true"/"false"')
    if isinstance(t, int):
        return (_TYPE_RANK_NUMBER, 0, t)
    if isinstance(t, float):
        return (_TYPE_RANK_NUMBER, 1, t)
    if isinstance(t, tuple):
        return (_TYPE_RANK_TUPLE, len(t), tuple(exact_term_key(e) for e in t))
    if isinstance(t, list) and t:
        return (_TYPE_RANK_LIST, [exact_term_key(e) for e in t])
    if isinstance(t, Mapping):
        items = _map_items(t)
        return (_TYPE_RANK_MAP, len(items), tuple(exact_term_key(k) for k, _ in items),
                tuple(exact_term_key(v) for _, v in items))
    return term_key(t)


class ErlMap(Mapping):
    """An Erlang map as the restatement models it: pairs with exactly
    distinct keys (1 and 1.0 are two keys)."""

    def __init__(self, pairs=()):
        d = {}
        for k, v in (pairs.items() if isinstance(pairs, Mapping) else pairs):
            d[repr(exact_term_key(k))] = (k, v)
        self._pairs = list(d.values())

    def __getitem__(self, key):
        ek = exact_term_key(key)
        for k, v in self._pairs:
            if exact_term_key(k) == ek:
                return v
        raise KeyError(key)

    def __iter__(self):
        return (k for k, _ in self._pairs)

    def __len__(self):
        return len(self._pairs)

    def items(self):
        return list(self._pairs)

    def __eq__(self, other):
        return isinstance(other, Mapping) and term_key(self) == term_key(other)

    def __hash__(self):
        return hash(repr(term_key(self)))


def _map_items(m):
    """A map's pairs in map-key order (the order of an ERTS flatmap)."""
    return sorted(m.items(), key=lambda kv: exact_term_key(kv[0]))


def _atom_ext(a):
    if ETF_ATOMS == 'latin1' and max((ord(c) for c in a), default=0) < 256:
        raw = a.encode('latin-1')
        return b'd' + len(raw).to_bytes(2, 'big') + raw                   # ATOM_EXT
    raw = a.encode('utf-8')
    if len(raw) < 256:
        return b'w' + bytes([len(raw)]) + raw                             # SMALL_ATOM_UTF8_EXT
    return b'v' + len(raw).to_bytes(2, 'big') + raw                       # ATOM_UTF8_EXT


def _ext(t):
    """One term in the external term format (erts external.c, default options)."""
    if isinstance(t, bool):
        raise ErlangCrash('booleans unsupported')
    if isinstance(t, int):
        if 0 <= t < 256:
            return b'a' + bytes([t])                                      # SMALL_INTEGER_EXT
        if -2 ** 31 <= t < 2 ** 31:
            return b'b' + (t & 0xFFFFFFFF).to_bytes(4, 'big')             # INTEGER_EXT
        mag = abs(t)
        digits = []
        while mag:
            digits.append(mag & 0xFF)
            mag >>= 8
        if len(digits) < 256:
            return b'n' + bytes([len(digits), 1 if t < 0 else 0] + digits)  # SMALL_BIG_EXT
        return b'o' + len(digits).to_bytes(4, 'big') + bytes([1 if t < 0 else 0] + digits)
    if isinstance(t, float):
        import struct
        return b'F' + struct.pack('>d', t)                                # NEW_FLOAT_EXT
    if isinstance(t, str):
        return _atom_ext(t)
    if isinstance(t, (bytes, bytearray)):
        return b'm' + len(t).to_bytes(4, 'big') + bytes(t)                # BINARY_EXT
    if isinstance(t, tuple):
        head = b'h' + bytes([len(t)]) if len(t) < 256 else b'i' + len(t).to_bytes(4, 'big')
        return head + b''.join(_ext(e) for e in t)
    if isinstance(t, list):
        if not t:
            return b'j'                                                   # NIL_EXT
        if len(t) < 65536 and all(type(e) is int and 0 <= e < 256 for e in t):
            return b'k' + len(t).to_bytes(2, 'big') + bytes(t)            # STRING_EXT
        return b'l' + len(t).to_bytes(4, 'big') + b''.join(_ext(e) for e in t) + b'j'
    if isinstance(t, Mapping):   # MAP_EXT; a flatmap (<= 32 keys) writes its pairs in map-key order
        # a hashmap (> 32 keys) is written in ERTS hash order and OTP 26+
        # orders a flatmap's atom keys by atom index: not restated
        if len(t) > 32:
            raise ErlangCrash('map of more than 32 pairs: ETF order not restated (ERTS hash order)')
        if ETF_ATOMS == 'utf8' and sum(1 for k in t if isinstance(k, str)) > 1:
            raise ErlangCrash('OTP 26+ map with several atom keys: ETF order not restated (atom index)')
        items = _map_items(t)
        return b't' + len(items).to_bytes(4, 'big') + b''.join(_ext(k) + _ext(v) for k, v in items)
    raise ErlangCrash('term outside the restated domain: %r' % (t,))


def term_to_binary(t):
    return b'\x83' + _ext(t)


def ensure_binary(key):
    """synctree.erl:261-268."""
    if isinstance(key, bool):
        raise ErlangCrash('booleans unsupported')
    if isinstance(key, int):
        return (key & 0xFFFFFFFFFFFFFFFF).to_bytes(8, 'big')   # <<Key:64/integer>>
    if isinstance(key, str):
        return key.encode('utf-8')                             # atom_to_binary(K, utf8)
    if isinstance(key, (bytes, bytearray)):
        return bytes(key)
    return term_to_binary(key)                                 # term_to_binary(Key)


def md5(data):
    return hashlib.md5(data).digest()


def get_segment(key, segments):
    """synctree.erl:251-253: <<HashKey:128/integer>> = md5(Key), HashKey rem Segments."""
    return int.from_bytes(md5(ensure_binary(key)), 'big') % segments


def hash_node(orddict):
    """synctree.erl:255-259: <<?H_MD5, md5([V || {_,V} <- Orddict])>>."""
    return bytes([H_MD5]) + md5(b''.join(v for _, v in orddict))


def orddict_store(key, value, d):
    """orddict:store/3 (stdlib): replace-or-insert keeping term order."""
    tk = term_key(key)
    out = []
    placed = False
    for k, v in d:
        if not placed:
            ck = term_key(k)
            if tk < ck:
                out.append((key, value))
                placed = True
            elif tk == ck:
                out.append((key, value))
                placed = True
                continue
        out.append((k, v))
    if not placed:
        out.append((key, value))
    return out


def orddict_erase(key, d):
    """orddict:erase/2 (stdlib): drops the entry whose key == Key (so 1 and
    1.0 are one key, like orddict:store above)."""
    tk = term_key(key)
    return [(k, v) for k, v in d if term_key(k) != tk]


def orddict_find(key, default, d):
    """synctree.erl:342-348: lists:keyfind(Key, 1, L) -- the first tuple
    whose key compares EQUAL (==, the keyfind BIF's CMP_EQ: an integer Key
    also finds an equal float key, and vice versa)."""
    tk = term_key(key)
    for k, v in d:
        if term_key(k) == tk:
            return v
    return default


def orddict_delta(d1, d2):
    """riak_ensemble_util.erl:115-141 merge-join."""
    out = []
    i = j = 0
    while i < len(d1) and j < len(d2):
        k1, v1 = d1[i]
        k2, v2 = d2[j]
        a, b = term_key(k1), term_key(k2)
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
    while j < len(d2):
        k2, v2 = d2[j]
        out.append((k2, (NONE, v2)))
        j += 1
    while i < len(d1):
        k1, v1 = d1[i]
        out.append((k1, (v1, NONE)))
        i += 1
    return out


# --------------------------------------------------------------------------
# Backends (the synctree backend behaviour: new/fetch/exists/store/store)

class EtsBackend:
    """synctree_ets.erl:32-66 — a mutable set shared by every tree record."""
    name = 'synctree_ets'

    def __init__(self, opts=None):
        self.t = {}

    def fetch(self, key, default):
        return self.t.get(key, default)

    def exists(self, key):
        return key in self.t

    def store(self, key, val):
        self.t[key] = val
        return self

    def store_batch(self, updates):
        # puts (with deletes turned into a 'deleted' marker) then delete_object
        for u in updates:
            if u[0] == 'put':
                self.t[u[1]] = u[2]
            else:
                self.t[u[1]] = 'deleted'
        for u in updates:
            if u[0] == 'delete' and self.t.get(u[1]) == 'deleted':
                del self.t[u[1]]
        return self


class OrddictBackend:
    """synctree_orddict.erl:32-66 — an immutable sorted list."""
    name = 'synctree_orddict'

    def __init__(self, opts=None, data=None):
        self.data = dict(data) if data else {}

    def fetch(self, key, default):
        return self.data.get(key, default)

    def exists(self, key):
        return key in self.data

    def store(self, key, val):
        d = dict(self.data)
        d[key] = val
        return OrddictBackend(data=d)

    def store_batch(self, updates):
        # lists:ukeymerge(1, lists:sort(Inserts), L): the first of equal keys
        # in the sorted inserts wins, then 'deleted' entries are dropped.
        inserts = {}
        for u in updates:
            k = u[1]
            v = u[2] if u[0] == 'put' else 'deleted'
            cur = inserts.get(k)
            # lists:sort sorts {K,V} tuples fully, ukeymerge keeps the first
            # of each key => the smallest {K,V}; restated with Erlang order
            # on values (binaries/lists > atoms 'deleted').
            if cur is None or _val_order(v) < _val_order(cur):
                inserts[k] = v
        d = dict(self.data)
        d.update(inserts)
        d = {k: v for k, v in d.items() if v != 'deleted'}
        return OrddictBackend(data=d)


def _val_order(v):
    if isinstance(v, str):
        return (1, v.encode())
    if isinstance(v, (bytes, bytearray)):
        return (9, bytes(v))
    if isinstance(v, list):
        return (8, len(v), [(term_key(k), _val_order(x)) for k, x in v])
    return (5, repr(v))


BACKENDS = {'synctree_ets': EtsBackend, 'synctree_orddict': OrddictBackend}


# --------------------------------------------------------------------------
# Tree record and geometry

def compute_height(segments, width):
    """synctree.erl:270-276 (crashes with case_clause when not a power)."""
    height = int(math.log(segments) / math.log(width))
    if int(math.pow(width, height)) == segments:
        return height
    raise ErlangCrash('case_clause: segments not a power of width')


def compute_shift(width):
    """synctree.erl:278-284."""
    shift = int(math.log(width) / math.log(2))
    if int(math.pow(2, shift)) == width:
        return shift
    raise ErlangCrash('case_clause: width not a power of 2')


class Tree:
    """The #tree{} record (synctree.erl:103-114).  Copy-on-update like Erlang."""
    __slots__ = ('id', 'width', 'segments', 'height', 'shift', 'shift_max',
                 'top_hash', 'buffer', 'buffered', 'mod', 'modstate')

    def replace(self, **kw):
        t = Tree()
        for s in Tree.__slots__:
            setattr(t, s, kw.get(s, getattr(self, s)))
        return t


def new(id_=None, width='default', segments='default', mod='synctree_ets', opts=None):
    """synctree.erl:135-170 + reload_top_hash 172-175."""
    if width == 'default':
        width = WIDTH
    if segments == 'default':
        segments = SEGMENTS
    height = compute_height(segments, width)
    shift = compute_shift(width)
    t = Tree()
    t.id = id_
    t.width = width
    t.segments = segments
    t.height = height
    t.shift = shift
    t.shift_max = shift * height
    t.buffer = []
    t.buffered = 0
    t.mod = mod
    t.modstate = BACKENDS[mod](opts)
    t.top_hash = m_fetch((0, 0), UNDEFINED, t)
    return t


def height(t):
    return t.height


def top_hash(t):
    return t.top_hash


# --------------------------------------------------------------------------
# insert / get

def insert(key, value, t):
    """synctree.erl:189-199."""
    if not isinstance(value, (bytes, bytearray)):
        raise ErlangCrash('function_clause: value must be a binary')
    segment = get_segment(key, t.segments)
    path = get_path(segment, t)
    if isinstance(path, tuple):
        return path
    top, updates = update_path(path, key, bytes(value))
    t2 = m_store_batch(updates, t)
    return t2.replace(top_hash=top)


def update_path(path, child, child_hash):
    """synctree.erl:201-209."""
    acc = []
    for (level, bucket), hashes in path:
        hashes2 = orddict_store(child, child_hash, hashes)
        new_hash = hash_node(hashes2)
        acc.insert(0, ('put', (level, bucket), hashes2))
        child, child_hash = bucket, new_hash
    acc.insert(0, ('put', (0, 0), child_hash))
    return child_hash, acc


def get(key, t):
    """synctree.erl:213-227."""
    if t.top_hash == UNDEFINED:
        return NOTFOUND
    segment = get_segment(key, t.segments)
    path = get_path(segment, t)
    if isinstance(path, tuple):
        return path
    return orddict_find(key, NOTFOUND, path[0][1])


def exchange_get(level, bucket, t):
    """synctree.erl:231-237."""
    if level == 0 and bucket == 0:
        return [(0, t.top_hash)]
    return verified_hashes(level, bucket, t)


def corrupt(key, t):
    """synctree.erl:241-247 (test aid: erase without updating the path)."""
    segment = get_segment(key, t.segments)
    bk = (t.height + 1, segment)
    hashes = m_fetch(bk, [], t)
    return m_store(bk, orddict_erase(key, hashes), t)


def verified_hashes(level, bucket, t):
    """synctree.erl:288-298."""
    n = (level - 1) * t.shift
    r = _get_path(n, 1, t.shift, bucket, [(0, t.top_hash)], t)
    if isinstance(r, tuple):
        return r
    return r[0][1]


def get_path(segment, t):
    """synctree.erl:302-304."""
    return _get_path(t.shift_max, 1, t.shift, segment, [(0, t.top_hash)], t)


def _get_path(n, level, shift, segment, up_hashes, t):
    """synctree.erl:306-320 (returns the path deepest-first, or a corruption tuple)."""
    acc = []
    while True:
        bucket = segment >> n
        expected = orddict_find(bucket, UNDEFINED, up_hashes)
        hashes = m_fetch((level, bucket), [], t)
        acc.insert(0, ((level, bucket), hashes))
        if not verify_hash(expected, hashes):
            return (CORRUPTED, level, bucket)
        if n == 0:
            return acc
        n -= shift
        level += 1
        up_hashes = hashes


def verify_hash(expected, hashes):
    """synctree.erl:322-340."""
    if expected == UNDEFINED:
        return hashes == []
    return hash_node(hashes) == expected


# --------------------------------------------------------------------------
# exchange

def direct_exchange(t):
    """synctree.erl:354-359."""
    def f(op, arg):
        if op == 'exchange_get':
            return exchange_get(arg[0], arg[1], t)
        return 'ok'
    return f


def local_compare(t1, t2):
    """synctree.erl:361-368."""
    return compare(height(t1), direct_exchange(t1), direct_exchange(t2))


def _default_accfun(keys, acc):
    return keys + acc          # synctree.erl:373-375 (Keys ++ KeyAcc)


def compare(height_, local, remote, accfun=_default_accfun, opts=()):
    """synctree.erl:372-395."""
    final = height_ + 1
    level, diff, acc = 0, [0], []
    filt = filter_type(opts)
    while diff:
        if level == final:
            return exchange_final(level, diff, local, remote, accfun, acc, filt)
        diff = exchange_level(level, diff, local, remote, filt)
        level += 1
    return acc


def _delta(a, b):
    if not isinstance(a, list) or not isinstance(b, list):
        # orddict_delta/3 has no clause for a {corrupted,L,B} tuple
        raise ErlangCrash('function_clause in orddict_delta: %r / %r' % (a, b))
    return orddict_delta(a, b)


def exchange_level(level, buckets, local, remote, filt):
    """synctree.erl:397-406."""
    remote('start_exchange_level', (level, buckets))
    out = []
    for b in buckets:
        a = local('exchange_get', (level, b))
        bb = remote('exchange_get', (level, b))
        out.extend(bk for bk, _ in apply_filter(filt, _delta(a, bb)))
    return out


def exchange_final(level, buckets, local, remote, accfun, acc, filt):
    """synctree.erl:408-417."""
    remote('start_exchange_level', (level, buckets))
    for b in buckets:
        a = local('exchange_get', (level, b))
        bb = remote('exchange_get', (level, b))
        acc = accfun(apply_filter(filt, _delta(a, bb)), acc)
    return acc


def filter_type(opts):
    """synctree.erl:421-432."""
    lo = 'local_only' in opts
    ro = 'remote_only' in opts
    if lo and not ro:
        return 'local_only'
    if ro and not lo:
        return 'remote_only'
    if not lo and not ro:
        return 'all'
    raise ErlangCrash('case_clause: both local_only and remote_only')


def apply_filter(kind, delta):
    """synctree.erl:434-449."""
    if kind == 'all':
        return delta
    if kind == 'local_only':
        return [d for d in delta if d[1][1] != NONE]
    return [d for d in delta if d[1][0] != NONE]


# --------------------------------------------------------------------------
# backend indirection + write buffer (synctree.erl:453-485)

def m_fetch(key, default, t):
    return t.modstate.fetch(key, default)


def m_store(key, val, t):
    return t.replace(modstate=t.modstate.store(key, val))


def m_store_batch(updates, t):
    return t.replace(modstate=t.modstate.store_batch(updates))


def m_exists(key, t):
    return t.modstate.exists(key)


def m_batch(update, t):
    t2 = t.replace(buffer=[update] + t.buffer, buffered=t.buffered + 1)
    if t2.buffered > 200:
        return m_flush(t2)
    return t2


def m_flush(t):
    updates = list(reversed(t.buffer))
    t2 = m_store_batch(updates, t)
    return t2.replace(buffer=[], buffered=0)


# --------------------------------------------------------------------------
# rehash (synctree.erl:489-543)

def rehash_upper(t):
    return _rehash(t.height, t)


def rehash(t):
    return _rehash(t.height + 1, t)


def _rehash(max_depth, t):
    t2, hashes = _rehash4(1, max_depth, 0, t)
    if not hashes:
        t3 = delete_existing_batch((0, 0), t2)
        top = UNDEFINED
    else:
        top = hash_node(hashes)
        t3 = m_batch(('put', (0, 0), top), t2)
    t4 = m_flush(t3)
    return t4.replace(top_hash=top)


def _rehash4(level, max_depth, bucket, t):
    if level == max_depth:
        return t, m_fetch((level, bucket), [], t)
    x0 = bucket * t.width
    ch = []
    for x in range(x0, x0 + t.width):
        t, hashes = _rehash4(level + 1, max_depth, x, t)
        if hashes:
            ch.append((x, hash_node(hashes)))
    if not ch:
        t = delete_existing_batch((level, bucket), t)
    else:
        t = m_batch(('put', (level, bucket), ch), t)
    return t, ch


def delete_existing_batch(key, t):
    if m_exists(key, t):
        return m_batch(('delete', key), t)
    return t


# --------------------------------------------------------------------------
# verify (synctree.erl:549-571)

def verify_upper(t):
    return _verify(1, t.height, 0, t.top_hash, t)


def verify(t):
    return _verify(1, t.height + 1, 0, t.top_hash, t)


def _verify(level, max_depth, bucket, up_hash, t):
    hashes = m_fetch((level, bucket), [], t)
    if not verify_hash(up_hash, hashes):
        return False
    if level == max_depth:
        return True
    return all(_verify(level + 1, max_depth, c, h, t) for c, h in hashes)


# --------------------------------------------------------------------------
# test-suite helpers (restating test/synctree_pure.erl:70-84)

def build(n, mod='synctree_ets', width='default', segments='default'):
    t = new(None, width, segments, mod)
    for k in range(n, 0, -1):
        t = insert(k, (k * 10).to_bytes(8, 'big'), t)
    return t


def expected_diff(num, diff):
    return [(k, ((k * 10).to_bytes(8, 'big'), NONE)) for k in range(num - diff + 1, num + 1)]


def level_image(t, level):
    """All stored nodes of one level as {bucket: content} (for fixtures)."""
    out = {}
    for b in range(t.width ** (level - 1)):
        v = m_fetch((level, b), [], t)
        if v:
            out[b] = v
    return out
