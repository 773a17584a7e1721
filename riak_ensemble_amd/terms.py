"""Erlang-term view of synctree keys and values for the host mirror.

Keys on the device path are (type, ensure_binary bytes)
(src/synctree.erl:261-268): integers -> <<K:64/big>>, atoms ->
atom_to_binary(K, utf8), binaries -> themselves.  In Python: ``int`` is an
Erlang integer (int64 range), ``str`` an atom, ``bytes`` a binary.  Keys the
reference would pass through term_to_binary (tuples, lists, ...) are outside
the device domain and raise ``TypeError``.

Atoms returned by the API are plain strings: ``'notfound'``,
``'undefined'``, ``'$none'``; corruption is the tuple
``('corrupted', Level, Bucket)``.
"""
import numpy as np

from . import _lib

NOTFOUND = 'notfound'
UNDEFINED = 'undefined'
NONE = '$none'
CORRUPTED = 'corrupted'

_I64_MIN, _I64_MAX = -(1 << 63), (1 << 63) - 1


def key_parts(key):
    """(ST_KEY_*, ensure_binary bytes)."""
    if isinstance(key, bool):
        raise TypeError('Python bools are not Erlang keys (use the atoms "true"/"false")')
    if isinstance(key, int):
        if not _I64_MIN <= key <= _I64_MAX:
            raise TypeError('integer key outside int64: the device path covers int64 keys')
        return _lib.ST_KEY_INT, (key & 0xFFFFFFFFFFFFFFFF).to_bytes(8, 'big')
    if isinstance(key, str):
        return _lib.ST_KEY_ATOM, key.encode('utf-8')
    if isinstance(key, (bytes, bytearray, memoryview)):
        return _lib.ST_KEY_BINARY, bytes(key)
    raise TypeError('key %r needs term_to_binary (outside the device key domain)' % (key,))


def key_from_parts(kt, kb):
    if kt == _lib.ST_KEY_INT:
        return int.from_bytes(kb, 'big', signed=True)
    if kt == _lib.ST_KEY_ATOM:
        return kb.decode('utf-8')
    return bytes(kb)


def order_key(key):
    """A bytes key whose lexicographic order is Erlang term order on the domain
    (the same record encoding the device sorts by)."""
    kt, kb = key_parts(key)
    if kt == _lib.ST_KEY_INT:
        return bytes([kt, kb[0] ^ 0x80]) + kb[1:]
    return bytes([kt]) + kb


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
