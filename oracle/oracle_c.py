"""ctypes binding of the C restatement (oracle/synctree_oracle.c).

TEST INFRASTRUCTURE ONLY — imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg, never by the product package.  The API mirrors
oracle/synctree_ref.py (same names, same Erlang-shaped return values) so the
two restatements can be cross-checked on identical inputs.
"""
import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, 'build', 'libsynctree_oracle.so')
_lib = None

NONE = '$none'
NOTFOUND = 'notfound'
UNDEFINED = 'undefined'
CORRUPTED = 'corrupted'

c_u8p = ctypes.POINTER(ctypes.c_uint8)


def build():
    subprocess.check_call(['make', '-s', '-C', _HERE])


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        vp, u64, u32, u8, i64 = ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint8, ctypes.c_int64
        P = ctypes.POINTER
        L.ot_new.restype = vp
        L.ot_new.argtypes = [u64, u64, P(ctypes.c_int)]
        L.ot_free.argtypes = [vp]
        L.ot_height.restype = u64
        L.ot_height.argtypes = [vp]
        L.ot_segment_of.restype = u64
        L.ot_segment_of.argtypes = [vp, ctypes.c_char_p, u32]
        L.ot_insert.restype = ctypes.c_int
        L.ot_insert.argtypes = [vp, u8, ctypes.c_char_p, u32, ctypes.c_char_p, u32, P(u32), P(u64)]
        L.ot_get.restype = ctypes.c_int
        L.ot_get.argtypes = [vp, u8, ctypes.c_char_p, u32, P(c_u8p), P(u32), P(u32), P(u64)]
        L.ot_corrupt.argtypes = [vp, u8, ctypes.c_char_p, u32]
        L.ot_rehash.argtypes = [vp, ctypes.c_int]
        L.ot_rehash_par.argtypes = [vp, ctypes.c_int]
        L.ot_verify.restype = ctypes.c_int
        L.ot_verify.argtypes = [vp, ctypes.c_int]
        L.ot_top_hash.restype = ctypes.c_int
        L.ot_top_hash.argtypes = [vp, ctypes.c_char_p]
        L.ot_node_count.restype = i64
        L.ot_node_count.argtypes = [vp, u32, u64]
        L.ot_node_stored.restype = ctypes.c_int
        L.ot_node_stored.argtypes = [vp, u32, u64]
        L.ot_node_child.argtypes = [vp, u32, u64, u32, P(u64), ctypes.c_char_p]
        L.ot_node_entry.argtypes = [vp, u32, u64, u32, P(u8), P(c_u8p), P(u32), P(c_u8p), P(u32)]
        L.ot_level_entries.argtypes = [vp, u32, vp, vp]
        L.ot_store_inner.argtypes = [vp, u32, u64, u32, vp, vp]
        L.ot_store_segment.argtypes = [vp, u64, u32, vp, vp, vp, vp, vp]
        L.ot_delete_node.argtypes = [vp, u32, u64]
        L.ot_store_top.argtypes = [vp, ctypes.c_char_p, ctypes.c_int]
        L.ot_compare.restype = vp
        L.ot_compare.argtypes = [vp, vp, ctypes.c_int, P(ctypes.c_int), P(u32), P(u64), P(ctypes.c_int)]
        L.ot_diff_count.restype = u64
        L.ot_diff_count.argtypes = [vp]
        L.ot_diff_get.argtypes = [vp, u64, P(u8), P(c_u8p), P(u32), P(c_u8p), P(u32), P(c_u8p), P(u32), P(u64)]
        L.ot_diff_free.argtypes = [vp]
        L.ot_bulk_load.restype = ctypes.c_int
        L.ot_bulk_load.argtypes = [vp, u64, vp, vp, vp, vp, vp]
        L.ot_bulk_load_int64.restype = ctypes.c_int
        L.ot_bulk_load_int64.argtypes = [vp, u64, vp, vp, u32]
        L.ot_md5.argtypes = [ctypes.c_char_p, u64, ctypes.c_char_p]
        L.ot_num_entries.restype = u64
        L.ot_num_entries.argtypes = [vp]
        L.ot_insert_int64_seq.restype = u64
        L.ot_insert_int64_seq.argtypes = [vp, u64, vp, vp, u32]
        L.ot_bulk_load_int64_par.restype = ctypes.c_int
        L.ot_bulk_load_int64_par.argtypes = [vp, u64, vp, vp, u32, ctypes.c_int]
        L.ot_apply_int64_batch.restype = ctypes.c_int
        L.ot_apply_int64_batch.argtypes = [vp, u64, vp, vp, u32, ctypes.c_int]
        _lib = L
    return _lib


def md5(data):
    out = ctypes.create_string_buffer(16)
    lib().ot_md5(bytes(data), len(data), out)
    return out.raw


def key_parts(key):
    """(type, ensure_binary bytes) — synctree.erl:261-268 on the int/atom/binary domain."""
    if isinstance(key, bool):
        raise TypeError('booleans are not keys')
    if isinstance(key, int):
        if not -(1 << 63) <= key < (1 << 63):
            raise ValueError('integer key outside int64')
        return 0, (key & 0xFFFFFFFFFFFFFFFF).to_bytes(8, 'big')
    if isinstance(key, str):
        return 1, key.encode('utf-8')
    if isinstance(key, (bytes, bytearray)):
        return 2, bytes(key)
    raise TypeError('unsupported key %r' % (key,))


def key_from_parts(kt, kb):
    if kt == 0:
        return int.from_bytes(kb, 'big', signed=True)
    if kt == 1:
        return kb.decode('utf-8')
    return kb


def _bytes(p, n):
    return ctypes.string_at(p, n) if n else b''


def pack_keys_values(keys, values):
    kt = np.zeros(len(keys) + 1, np.uint8)
    kparts, vparts = [], []
    koff = np.zeros(len(keys) + 1, np.uint64)
    voff = np.zeros(len(keys) + 1, np.uint64)
    ko = vo = 0
    for i, (k, v) in enumerate(zip(keys, values)):
        t, b = key_parts(k)
        kt[i] = t
        kparts.append(b)
        vparts.append(bytes(v))
        ko += len(b)
        vo += len(v)
        koff[i + 1] = ko
        voff[i + 1] = vo
    kh = np.frombuffer(b''.join(kparts) + b'\0', np.uint8).copy()
    vh = np.frombuffer(b''.join(vparts) + b'\0', np.uint8).copy()
    return kt, kh, koff, vh, voff


class OTree:
    def __init__(self, width=16, segments=1 << 20):
        err = ctypes.c_int(0)
        self.h = lib().ot_new(width, segments, ctypes.byref(err))
        if not self.h:
            raise ValueError('bad geometry (reference: case_clause)')
        self.width, self.segments = width, segments
        self.height = int(lib().ot_height(self.h))

    def __del__(self):
        if getattr(self, 'h', None):
            lib().ot_free(self.h)
            self.h = None

    def segment_of(self, key):
        _, kb = key_parts(key)
        return int(lib().ot_segment_of(self.h, kb, len(kb)))

    def insert(self, key, value):
        kt, kb = key_parts(key)
        cl, cb = ctypes.c_uint32(), ctypes.c_uint64()
        r = lib().ot_insert(self.h, kt, kb, len(kb), bytes(value), len(value), ctypes.byref(cl), ctypes.byref(cb))
        if r == 2:
            return (CORRUPTED, cl.value, cb.value)
        return self

    def get(self, key):
        kt, kb = key_parts(key)
        vp, vl = c_u8p(), ctypes.c_uint32()
        cl, cb = ctypes.c_uint32(), ctypes.c_uint64()
        r = lib().ot_get(self.h, kt, kb, len(kb), ctypes.byref(vp), ctypes.byref(vl), ctypes.byref(cl),
                         ctypes.byref(cb))
        if r == 1:
            return NOTFOUND
        if r == 2:
            return (CORRUPTED, cl.value, cb.value)
        return _bytes(vp, vl.value)

    def corrupt(self, key):
        kt, kb = key_parts(key)
        lib().ot_corrupt(self.h, kt, kb, len(kb))
        return self

    def rehash(self):
        lib().ot_rehash(self.h, 0)
        return self

    def rehash_par(self, threads=0):
        lib().ot_rehash_par(self.h, threads)
        return self

    def rehash_upper(self):
        lib().ot_rehash(self.h, 1)
        return self

    def verify(self):
        return bool(lib().ot_verify(self.h, 0))

    def verify_upper(self):
        return bool(lib().ot_verify(self.h, 1))

    def top_hash(self):
        buf = ctypes.create_string_buffer(17)
        if lib().ot_top_hash(self.h, buf):
            return buf.raw
        return UNDEFINED

    def node(self, level, bucket):
        """Mod:fetch({Level,Bucket}, [], _) image."""
        n = int(lib().ot_node_count(self.h, level, bucket))
        out = []
        if level == self.height + 1:
            for i in range(n):
                kt, kp, kl, vp, vl = ctypes.c_uint8(), c_u8p(), ctypes.c_uint32(), c_u8p(), ctypes.c_uint32()
                lib().ot_node_entry(self.h, level, bucket, i, ctypes.byref(kt), ctypes.byref(kp), ctypes.byref(kl),
                                    ctypes.byref(vp), ctypes.byref(vl))
                out.append((key_from_parts(kt.value, _bytes(kp, kl.value)), _bytes(vp, vl.value)))
        else:
            for i in range(n):
                c = ctypes.c_uint64()
                h = ctypes.create_string_buffer(17)
                lib().ot_node_child(self.h, level, bucket, i, ctypes.byref(c), h)
                out.append((c.value, h.raw))
        return out

    def level_entries(self, level):
        """(present[u8], hashes[n,17]) recorded for each bucket of `level` in its parent."""
        n = self.width ** (level - 1)
        present = np.zeros(n, np.uint8)
        hashes = np.zeros((n, 17), np.uint8)
        lib().ot_level_entries(self.h, level, present.ctypes.data, hashes.ctypes.data)
        return present, hashes

    def store_inner(self, level, bucket, children):
        ch = np.array([c for c, _ in children], np.uint64)
        hs = np.frombuffer(b''.join(h for _, h in children) + b'\0', np.uint8).copy()
        lib().ot_store_inner(self.h, level, bucket, len(children), ch.ctypes.data, hs.ctypes.data)

    def store_segment(self, seg, entries):
        kt, kh, koff, vh, voff = pack_keys_values([k for k, _ in entries], [v for _, v in entries])
        lib().ot_store_segment(self.h, seg, len(entries), kt.ctypes.data, kh.ctypes.data, koff.ctypes.data,
                               vh.ctypes.data, voff.ctypes.data)

    def delete_node(self, level, bucket):
        lib().ot_delete_node(self.h, level, bucket)

    def bulk_load(self, keys, values):
        kt, kh, koff, vh, voff = pack_keys_values(keys, values)
        r = lib().ot_bulk_load(self.h, len(keys), kt.ctypes.data, kh.ctypes.data, koff.ctypes.data,
                               vh.ctypes.data, voff.ctypes.data)
        if r != 0:
            raise ValueError('bulk_load needs a fresh tree')
        return self

    def num_entries(self):
        return int(lib().ot_num_entries(self.h))

    def insert_int64_seq(self, keys, values):
        """len(keys) sequential insert/3 calls in C; returns #rejected."""
        keys = np.ascontiguousarray(keys, np.int64)
        values = np.ascontiguousarray(values, np.uint8)
        return int(lib().ot_insert_int64_seq(self.h, len(keys), keys.ctypes.data, values.ctypes.data, values.shape[1]))

    def bulk_load_int64_par(self, keys, values, threads=0):
        """bulk_load_int64 with OpenMP threads (0 = all): same result."""
        keys = np.ascontiguousarray(keys, np.int64)
        values = np.ascontiguousarray(values, np.uint8)
        r = lib().ot_bulk_load_int64_par(self.h, len(keys), keys.ctypes.data, values.ctypes.data, values.shape[1],
                                         threads)
        if r != 0:
            raise ValueError('bulk_load needs a fresh tree')
        return self

    def apply_int64_batch(self, keys, values, threads=0):
        """len(keys) sequential insert/3 calls on a CONSISTENT tree (no
        corruption: every path verifies), computed as merged segments + the
        full rehash (OpenMP threads, 0 = all); same result as insert_int64_seq
        on such a tree (pinned in tests/test_oracle.py)."""
        keys = np.ascontiguousarray(keys, np.int64)
        values = np.ascontiguousarray(values, np.uint8)
        lib().ot_apply_int64_batch(self.h, len(keys), keys.ctypes.data, values.ctypes.data, values.shape[1], threads)
        return self

    def bulk_load_int64(self, keys, values):
        """keys: int64 ndarray [n]; values: uint8 ndarray [n, vlen]."""
        keys = np.ascontiguousarray(keys, np.int64)
        values = np.ascontiguousarray(values, np.uint8)
        r = lib().ot_bulk_load_int64(self.h, len(keys), keys.ctypes.data, values.ctypes.data, values.shape[1])
        if r != 0:
            raise ValueError('bulk_load needs a fresh tree')
        return self

    def compare(self, other, opts=()):
        """local_compare(self, other) with the reference's filters and fold order."""
        lo, ro = 'local_only' in opts, 'remote_only' in opts
        if lo and ro:
            raise ValueError('case_clause: both filters')
        filt = 1 if lo else (2 if ro else 0)
        st, cl, cb, cs = ctypes.c_int(), ctypes.c_uint32(), ctypes.c_uint64(), ctypes.c_int()
        d = lib().ot_compare(self.h, other.h, filt, ctypes.byref(st), ctypes.byref(cl), ctypes.byref(cb),
                             ctypes.byref(cs))
        try:
            if st.value == 2:
                return ('crash', 'local' if cs.value == 0 else 'remote', (CORRUPTED, cl.value, cb.value))
            out = []
            for i in range(int(lib().ot_diff_count(d))):
                kt, kp, kl = ctypes.c_uint8(), c_u8p(), ctypes.c_uint32()
                ap, al, bp, bl, sg = c_u8p(), ctypes.c_uint32(), c_u8p(), ctypes.c_uint32(), ctypes.c_uint64()
                lib().ot_diff_get(d, i, ctypes.byref(kt), ctypes.byref(kp), ctypes.byref(kl), ctypes.byref(ap),
                                  ctypes.byref(al), ctypes.byref(bp), ctypes.byref(bl), ctypes.byref(sg))
                va = NONE if al.value == 0xFFFFFFFF else _bytes(ap, al.value)
                vb = NONE if bl.value == 0xFFFFFFFF else _bytes(bp, bl.value)
                out.append((key_from_parts(kt.value, _bytes(kp, kl.value)), (va, vb)))
            return out
        finally:
            lib().ot_diff_free(d)


def build(n, width=16, segments=1 << 20):
    """test/synctree_pure.erl:70-80 restated on the C oracle."""
    t = OTree(width, segments)
    for k in range(n, 0, -1):
        t.insert(k, (k * 10).to_bytes(8, 'big'))
    return t
