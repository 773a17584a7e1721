"""CPU restatement of synctree_leveldb's on-disk format — TEST INFRASTRUCTURE ONLY.

Imported only by ``tests/`` (never by the product package).  Restates:

* db_key/2,3 ................ src/synctree_leveldb.erl:104-109
  <<?K_BUCKET=0:8, Id/binary, Level:8, (binary:encode_unsigned(Bucket))/binary>>
* fetch/3 ................... src/synctree_leveldb.erl:111-123
  (binary_to_term; any decode failure or absent key => {ok, Default})
* exists/2 .................. src/synctree_leveldb.erl:125-132
* store/3, store/2 .......... src/synctree_leveldb.erl:134-152
  (term_to_binary of the node; write batch of puts/deletes in order)
* shared DB per path ........ src/synctree_leveldb.erl:59-83 (one dict per path)

``term_to_binary`` / ``binary_to_term`` are ERTS (third-party to the
reference, OTP version unpinned).  They are restated from
the published external term format (version byte 131) for the node domain:
integers (SMALL_INTEGER_EXT 97, INTEGER_EXT 98, SMALL_BIG_EXT 110), atoms
(ATOM_EXT 100 for Latin-1 atoms as term_to_binary writes them before OTP 26
-- the reference's era, the default -- or SMALL_ATOM_UTF8_EXT 119 /
ATOM_UTF8_EXT 118 as from OTP 26: synctree_ref.ETF_ATOMS), binaries
(BINARY_EXT 109), tuples (SMALL_TUPLE_EXT 104), floats (NEW_FLOAT_EXT 70) and
lists (STRING_EXT 107, LIST_EXT 108 ... NIL_EXT 106; [] = 106); the encoder
is synctree_ref's ETF restatement.  The byte
layouts are pinned by known-answer vectors in tests/test_leveldb_format.py
(classic published examples such as term_to_binary(256) =
<<131,98,0,0,1,0>>); the reference's own tests hold no ETF bytes, so the
value encoding is otherwise "parity unpinned" by reference fixtures.

Terms are modelled as in synctree_ref: int, str (atom), bytes (binary),
list, tuple.
"""
import struct

import synctree_ref as ST

K_BUCKET = 0   # synctree_leveldb.erl:44


class BadTerm(Exception):
    """binary_to_term raised (badarg)."""


# ------------------------------------------------------------------ ETF
def _enc(t, out):
    out += ST._ext(t)   # the ETF restatement (atoms in the era ST.ETF_ATOMS selects)


def term_to_binary(t):
    out = bytearray([131])
    _enc(t, out)
    return bytes(out)


def _dec(b, i):
    if i >= len(b):
        raise BadTerm('truncated')
    tg = b[i]
    i += 1

    def need(n):
        if i + n > len(b):
            raise BadTerm('truncated')

    if tg == 97:
        need(1)
        return b[i], i + 1
    if tg == 98:
        need(4)
        return struct.unpack('>i', b[i:i + 4])[0], i + 4
    if tg == 110:
        need(2)
        n, sign = b[i], b[i + 1]
        i += 2
        need(n)
        m = int.from_bytes(b[i:i + n], 'little')
        return (-m if sign else m), i + n
    if tg in (100, 118):
        need(2)
        n = struct.unpack('>H', b[i:i + 2])[0]
        i += 2
        need(n)
        raw = b[i:i + n]
        return (raw.decode('latin-1') if tg == 100 else raw.decode('utf-8')), i + n
    if tg in (115, 119):
        need(1)
        n = b[i]
        i += 1
        need(n)
        raw = b[i:i + n]
        return (raw.decode('latin-1') if tg == 115 else raw.decode('utf-8')), i + n
    if tg == 109:
        need(4)
        n = struct.unpack('>I', b[i:i + 4])[0]
        i += 4
        need(n)
        return bytes(b[i:i + n]), i + n
    if tg == 104:
        need(1)
        n = b[i]
        i += 1
        xs = []
        for _ in range(n):
            x, i = _dec(b, i)
            xs.append(x)
        return tuple(xs), i
    if tg == 106:
        return [], i
    if tg == 107:
        need(2)
        n = struct.unpack('>H', b[i:i + 2])[0]
        need(2 + n)
        return list(b[i + 2:i + 2 + n]), i + 2 + n
    if tg == 70:
        need(8)
        return struct.unpack('>d', b[i:i + 8])[0], i + 8
    if tg == 108:
        need(4)
        n = struct.unpack('>I', b[i:i + 4])[0]
        i += 4
        xs = []
        for _ in range(n):
            x, i = _dec(b, i)
            xs.append(x)
        tail, i = _dec(b, i)
        if tail != []:
            raise BadTerm('improper list outside the restated domain')
        return xs, i
    if tg == 99:   # FLOAT_EXT: "%.20e" in 31 bytes
        need(31)
        return float(b[i:i + 31].split(b'\0')[0].decode('ascii')), i + 31
    if tg == 116:  # MAP_EXT
        need(4)
        n = struct.unpack('>I', b[i:i + 4])[0]
        i += 4
        pairs = []
        for _ in range(n):
            k, i = _dec(b, i)
            v, i = _dec(b, i)
            pairs.append((k, v))
        return ST.ErlMap(pairs), i
    raise BadTerm('tag %d outside the restated domain' % tg)


def binary_to_term(b):
    b = bytes(b)
    if not b or b[0] != 131:
        raise BadTerm('bad version')
    t, i = _dec(b, 1)
    if i != len(b):
        raise BadTerm('trailing bytes')
    return t


def _node_term(node):
    """The Erlang term of a node as synctree_ref holds it: orddicts are lists
    of (K, V) pairs; the top hash is a binary."""
    if isinstance(node, list):
        return [(k, v) for k, v in node]
    return node


# ------------------------------------------------------------------ backend
def encode_unsigned(b):
    """binary:encode_unsigned/1."""
    return b.to_bytes(max(1, (b.bit_length() + 7) // 8), 'big')


def db_key(id_, level, bucket):
    """synctree_leveldb.erl:104-109."""
    if not isinstance(level, int) or not isinstance(bucket, int):
        raise ST.ErlangCrash('function_clause: db_key/3')
    return bytes([K_BUCKET]) + id_ + bytes([level]) + encode_unsigned(bucket)


_DBS = {}


class LeveldbBackend:
    """synctree_leveldb.erl:59-152 over an in-memory {key bytes: value bytes}
    DB shared by path (the ETS registry of :52-83)."""
    name = 'synctree_leveldb'

    def __init__(self, opts=None):
        opts = dict(opts or {})
        path = opts.get('path', '/tmp/ST/oracle')
        self.db = _DBS.setdefault(path, {})
        self.id = opts.get('tree_id', b'')
        if not isinstance(self.id, (bytes, bytearray)):
            raise ST.ErlangCrash('case_clause: tree_id must be a binary')
        self.id = bytes(self.id)

    def fetch(self, key, default):
        v = self.db.get(db_key(self.id, *key))
        if v is None:
            return default
        try:
            t = binary_to_term(v)
        except BadTerm:
            return default
        return [tuple(x) for x in t] if isinstance(t, list) else t

    def exists(self, key):
        return db_key(self.id, *key) in self.db

    def store(self, key, val):
        self.db[db_key(self.id, *key)] = term_to_binary(_node_term(val))
        return self

    def store_batch(self, updates):
        for u in updates:
            if u[0] == 'put':
                self.db[db_key(self.id, *u[1])] = term_to_binary(_node_term(u[2]))
            else:
                self.db.pop(db_key(self.id, *u[1]), None)
        return self


ST.BACKENDS['synctree_leveldb'] = LeveldbBackend


def reset_dbs():
    _DBS.clear()


def tree_records(db, id_):
    """The records of one tree id in a DB, as {key: value}."""
    p = bytes([K_BUCKET]) + id_
    return {k: v for k, v in db.items() if k.startswith(p)}
