"""Erlang-term view of synctree keys and values for the host mirror.

Keys on the device path are (type, bytes) (src/synctree.erl:261-268):
integers in int64 -> <<K:64/big>>, atoms -> atom_to_binary(K, utf8),
binaries -> themselves, and every other key (tuples, lists, maps, floats,
integers outside int64) -> term_to_binary(K) (ST_KEY_TERM; the device derives
the order-preserving record, riak_ensemble_amd/csrc/term_key.h).  In Python:
``int`` is an Erlang integer, ``float`` a float, ``str`` an atom, ``bytes`` a
binary, ``tuple`` a tuple, ``list`` a proper list and :class:`Map` (or a
``dict``) a map.  Pids, ports, refs and funs stay outside the key domain.

term_to_binary here writes what ERTS writes with default options: atoms in
the form of the configured OTP era (:data:`ETF_ATOMS`: ``'latin1'`` = before
OTP 26, ATOM_EXT for Latin-1 atoms -- the reference's era; ``'utf8'`` = OTP
26+), floats as NEW_FLOAT_EXT (OTP 17+), lists of bytes as STRING_EXT.

Atoms returned by the API are plain strings: ``'notfound'``,
``'undefined'``, ``'$none'``; corruption is the tuple
``('corrupted', Level, Bucket)``.
"""
import ctypes
import struct
from collections.abc import Mapping

import numpy as np

from . import _lib

NOTFOUND = 'notfound'
UNDEFINED = 'undefined'
NONE = '$none'
CORRUPTED = 'corrupted'

_I64_MIN, _I64_MAX = -(1 << 63), (1 << 63) - 1

ETF_ATOMS = 'latin1'


def exact_order(t):
    """Sort key of Erlang's exact (map-key) term order: like term order, but
    every integer sorts before every float and 1 =/= 1.0 (map keys compare
    with =:=).  Under a map key everything compares exactly."""
    if isinstance(t, bool):
        raise TypeError('Python bools are not Erlang terms (use the atoms "true"/"false")')
    if isinstance(t, int):
        return (0, 0, t)
    if isinstance(t, float):
        return (0, 1, t)
    if isinstance(t, str):
        return (1, t.encode('utf-8'))
    if isinstance(t, tuple):
        return (6, len(t), tuple(exact_order(e) for e in t))
    if isinstance(t, Mapping):
        m = t if isinstance(t, Map) else Map(t)
        return (7, len(m), tuple(exact_order(k) for k in m), tuple(exact_order(v) for v in m.values()))
    if isinstance(t, list):
        return (9, [exact_order(e) for e in t]) if t else (8,)
    if isinstance(t, (bytes, bytearray, memoryview)):
        return (10, bytes(t))
    raise TypeError('%r is not a term of the key domain' % (t,))


class Map(Mapping):
    """An Erlang map: keys compare exactly (1 and 1.0 are two keys), and the
    entries are kept in map-key order -- the order term_to_binary writes a
    map of up to 32 keys in (ERTS flatmaps)."""
    __slots__ = ('_items',)

    def __init__(self, items=()):
        if isinstance(items, Mapping):
            items = items.items()
        byk = {}
        for k, v in items:
            byk[repr(exact_order(k))] = (k, v)   # a later pair replaces an exactly equal key
        self._items = tuple(sorted(byk.values(), key=lambda kv: exact_order(kv[0])))

    def __getitem__(self, key):
        ek = exact_order(key)
        for k, v in self._items:
            if exact_order(k) == ek:
                return v
        raise KeyError(key)

    def __iter__(self):
        return (k for k, _ in self._items)

    def __len__(self):
        return len(self._items)

    def items(self):
        return list(self._items)

    def __eq__(self, other):
        if not isinstance(other, Mapping):
            return NotImplemented
        o = other if isinstance(other, Map) else Map(other)
        return len(o) == len(self) and all(exact_order(a) == exact_order(c) and b == d
                                           for (a, b), (c, d) in zip(self._items, o._items))

    def __hash__(self):
        return hash(repr([exact_order(k) for k in self]))

    def __repr__(self):
        return 'Map(%r)' % (list(self._items),)


def _map_etf_domain(m, atoms):
    """term_to_binary writes a map's pairs in map-key order only for a
    flatmap (at most 32 keys) whose order ERTS derives from the keys' term
    order: a larger map is a hashmap, written in the runtime's hash order, and
    OTP 26+ orders the atom keys of a flatmap by atom index.  Those byte
    strings cannot be restated here (a key's segment is md5 of them,
    synctree.erl:251-268): pass such keys as ERTS-produced ETF bytes
    (ST_KEY_TERM, what the NIF does) instead."""
    if len(m) > 32:
        raise TypeError('a map key of more than 32 pairs is written in ERTS hash order: pass its '
                        'term_to_binary bytes (ST_KEY_TERM) instead')
    if atoms == 'utf8' and sum(1 for k in m if isinstance(k, str)) > 1:
        raise TypeError('OTP 26+ writes the atom keys of a map in atom-index order: pass the map key\'s '
                        'term_to_binary bytes (ST_KEY_TERM) instead')


def _etf(t, out, atoms):
    if isinstance(t, bool):
        raise TypeError('Python bools are not Erlang terms (use the atoms "true"/"false")')
    if isinstance(t, int):
        if 0 <= t <= 255:
            out += bytes([97, t])
        elif -(1 << 31) <= t < (1 << 31):
            out += b'b' + struct.pack('>i', t)
        else:
            m = abs(t)
            mag = m.to_bytes((m.bit_length() + 7) // 8, 'little')
            sign = 1 if t < 0 else 0
            if len(mag) <= 255:
                out += bytes([110, len(mag), sign]) + mag
            else:
                out += bytes([111]) + struct.pack('>I', len(mag)) + bytes([sign]) + mag
    elif isinstance(t, float):
        out += b'F' + struct.pack('>d', t)
    elif isinstance(t, str):
        if len(t) > 255:
            raise TypeError('atom longer than 255 characters (system_limit)')
        if atoms == 'latin1' and all(ord(c) < 256 for c in t):
            b = t.encode('latin-1')
            out += bytes([100]) + struct.pack('>H', len(b)) + b
        else:
            b = t.encode('utf-8')
            out += (bytes([119, len(b)]) if len(b) < 256 else bytes([118]) + struct.pack('>H', len(b))) + b
    elif isinstance(t, (bytes, bytearray, memoryview)):
        b = bytes(t)
        out += bytes([109]) + struct.pack('>I', len(b)) + b
    elif isinstance(t, tuple):
        out += bytes([104, len(t)]) if len(t) <= 255 else bytes([105]) + struct.pack('>I', len(t))
        for e in t:
            _etf(e, out, atoms)
    elif isinstance(t, list):
        if not t:
            out += bytes([106])
        elif len(t) <= 65535 and all(isinstance(e, int) and not isinstance(e, bool) and 0 <= e <= 255 for e in t):
            out += bytes([107]) + struct.pack('>H', len(t)) + bytes(t)
        else:
            out += bytes([108]) + struct.pack('>I', len(t))
            for e in t:
                _etf(e, out, atoms)
            out += bytes([106])
    elif isinstance(t, Mapping):
        m = t if isinstance(t, Map) else Map(t)
        _map_etf_domain(m, atoms)
        out += bytes([116]) + struct.pack('>I', len(m))
        for k, v in m.items():
            _etf(k, out, atoms)
            _etf(v, out, atoms)
    else:
        raise TypeError('%r is not a term of the key domain (pids, ports, refs, funs are not)' % (t,))


def term_to_binary(t, atoms=None):
    """ERTS term_to_binary/1 on the key domain (see the module doc)."""
    out = bytearray([131])
    _etf(t, out, atoms or ETF_ATOMS)
    return bytes(out)


def _dec(b, i):
    tag = b[i]
    i += 1
    if tag == 97:
        return b[i], i + 1
    if tag == 98:
        return struct.unpack_from('>i', b, i)[0], i + 4
    if tag in (110, 111):
        if tag == 110:
            n, i = b[i], i + 1
        else:
            n, i = struct.unpack_from('>I', b, i)[0], i + 4
        sign, i = b[i], i + 1
        v = int.from_bytes(b[i:i + n], 'little')
        return (-v if sign else v), i + n
    if tag == 70:
        return struct.unpack_from('>d', b, i)[0], i + 8
    if tag == 99:
        return float(b[i:i + 31].split(b'\0')[0].decode('ascii')), i + 31
    if tag in (100, 115, 118, 119):
        if tag in (100, 118):
            n, i = struct.unpack_from('>H', b, i)[0], i + 2
        else:
            n, i = b[i], i + 1
        raw = b[i:i + n]
        return (raw.decode('latin-1') if tag in (100, 115) else raw.decode('utf-8')), i + n
    if tag in (104, 105):
        if tag == 104:
            n, i = b[i], i + 1
        else:
            n, i = struct.unpack_from('>I', b, i)[0], i + 4
        el = []
        for _ in range(n):
            e, i = _dec(b, i)
            el.append(e)
        return tuple(el), i
    if tag == 106:
        return [], i
    if tag == 107:
        n = struct.unpack_from('>H', b, i)[0]
        return list(b[i + 2:i + 2 + n]), i + 2 + n
    if tag == 108:
        n, i = struct.unpack_from('>I', b, i)[0], i + 4
        el = []
        for _ in range(n):
            e, i = _dec(b, i)
            el.append(e)
        tail, i = _dec(b, i)
        if tail != []:
            if isinstance(tail, list):
                return el + tail, i
            raise ValueError('improper lists have no Python form')
        return el, i
    if tag == 109:
        n = struct.unpack_from('>I', b, i)[0]
        return bytes(b[i + 4:i + 4 + n]), i + 4 + n
    if tag == 116:
        n, i = struct.unpack_from('>I', b, i)[0], i + 4
        pairs = []
        for _ in range(n):
            k, i = _dec(b, i)
            v, i = _dec(b, i)
            pairs.append((k, v))
        return Map(pairs), i
    raise ValueError('ETF tag %d outside the key domain' % tag)


def binary_to_term(b):
    b = bytes(b)
    if not b or b[0] != 131:
        raise ValueError('not a term_to_binary encoding')
    t, i = _dec(b, 1)
    if i != len(b):
        raise ValueError('trailing bytes')
    return t


def key_parts(key):
    """(ST_KEY_*, bytes): ensure_binary bytes, or term_to_binary for ST_KEY_TERM."""
    if isinstance(key, bool):
        raise TypeError('Python bools are not Erlang keys (use the atoms "true"/"false")')
    if isinstance(key, int) and _I64_MIN <= key <= _I64_MAX:
        return _lib.ST_KEY_INT, (key & 0xFFFFFFFFFFFFFFFF).to_bytes(8, 'big')
    if isinstance(key, str):
        return _lib.ST_KEY_ATOM, key.encode('utf-8')
    if isinstance(key, (bytes, bytearray, memoryview)):
        return _lib.ST_KEY_BINARY, bytes(key)
    return _lib.ST_KEY_TERM, term_to_binary(key)


def key_from_parts(kt, kb):
    if kt == _lib.ST_KEY_INT:
        return int.from_bytes(kb, 'big', signed=True)
    if kt == _lib.ST_KEY_ATOM:
        return kb.decode('utf-8')
    if kt == _lib.ST_KEY_TERM:
        return binary_to_term(kb)
    return bytes(kb)


def order_sk(key):
    """The part of `key`'s device record that decides its order (krec_order_len
    in csrc/st_kernels.h): Erlang-equal keys (1 and 1.0) have equal parts."""
    r = order_key(key)
    kt, _ = key_parts(key)
    if kt != _lib.ST_KEY_TERM:
        return r
    el = r[-4] | (r[-3] << 8)
    sl = r[-2] | (r[-1] << 8)
    return r[:len(r) - 4 - el - (0 if sl == 0xFFFF else sl)]


def order_key(key):
    """The device key record of `key` (bytes): their lexicographic order is
    Erlang term order (riak_ensemble_amd/csrc/term_key.h)."""
    kt, kb = key_parts(key)
    if kt == _lib.ST_KEY_INT:
        return bytes([0x10, kb[0] ^ 0x80]) + kb[1:]
    if kt == _lib.ST_KEY_ATOM:
        return b'\x20' + kb
    if kt == _lib.ST_KEY_BINARY:
        return b'\x50' + kb
    L = _lib.load()
    n = ctypes.c_uint64()
    _lib.check(L.st_key_record(kt, kb, len(kb), None, 0, ctypes.byref(n)), 'st_key_record')
    buf = ctypes.create_string_buffer(int(n.value))
    _lib.check(L.st_key_record(kt, kb, len(kb), buf, n.value, ctypes.byref(n)), 'st_key_record')
    return buf.raw


def pack_keys(keys):
    """-> (ktype u8[n], kheap u8[], koff u64[n+1]) numpy arrays."""
    n = len(keys)
    kt = np.zeros(n + 1, np.uint8)
    parts = []
    koff = np.zeros(n + 1, np.uint64)
    o = 0
    for i, k in enumerate(keys):
        t, b = key_parts(k)
        kt[i] = t
        parts.append(b)
        o += len(b)
        koff[i + 1] = o
    kh = np.frombuffer(b''.join(parts) + b'\0' * 8, np.uint8).copy()
    return kt, kh, koff


def pack_blobs(blobs):
    """Byte strings -> (heap u8[], off u64[n+1])."""
    off = np.zeros(len(blobs) + 1, np.uint64)
    if blobs:
        off[1:] = np.cumsum([len(b) for b in blobs])
    return np.frombuffer(b''.join(bytes(b) for b in blobs) + b'\0' * 8, np.uint8).copy(), off


def pack_values(values):
    n = len(values)
    voff = np.zeros(n + 1, np.uint64)
    o = 0
    parts = []
    for i, v in enumerate(values):
        if not isinstance(v, (bytes, bytearray, memoryview)):
            raise TypeError('function_clause: synctree values are binaries (synctree.erl:190)')
        parts.append(bytes(v))
        o += len(v)
        voff[i + 1] = o
    vh = np.frombuffer(b''.join(parts) + b'\0' * 8, np.uint8).copy()
    return vh, voff
