"""synctree_hip — the device-resident synctree backend.

Mirrors the synctree backend behaviour (``new/1, fetch/3, exists/2,
store/3, store/2``: src/synctree_ets.erl:22-66, src/synctree_orddict.erl:22-66)
over libsynctree_hip.so, and adds the bulk callbacks the synctree module uses
when they exist (insert_batch, rehash, verify, exchange_get, compare): the
plug point SURVEY.md §8b recommends.  State is a :class:`DeviceTree`.
"""
import ctypes

import numpy as np

from . import _lib
from . import terms

name = 'synctree_hip'


def _ptr(a):
    return None if a is None else ctypes.c_void_p(a.ctypes.data)


def _bytes(p, o0, o1):
    n = int(o1 - o0)
    if n <= 0:
        return b''
    return ctypes.string_at(ctypes.addressof(p.contents) + int(o0), n)


class _Closed:
    """Handle of a closed DeviceTree: passing it to the library raises."""

    @property
    def _as_parameter_(self):
        raise ValueError('DeviceTree is closed')

    value = None

    def __bool__(self):
        return False


class DeviceTree:
    """One device-resident tree (a C-ABI st_tree handle)."""

    def __init__(self, width=16, segments=1 << 20, device=0):
        L = _lib.load()
        h = ctypes.c_void_p()
        _lib.check(L.st_create(width, segments, device, ctypes.byref(h)), 'st_create')
        self.h = h
        self.L = L
        self.device = device
        self.width = int(L.st_width(h))
        self.segments = int(L.st_segments(h))
        self.height = int(L.st_height(h))
        self.shift = self.width.bit_length() - 1
        self._g1 = self._i1 = None   # cached ctypes buffers of get1 / insert1

    def close(self):
        """Free the device tree; any later call raises (the handle is gone)."""
        if getattr(self, 'h', None):
            self.L.st_destroy(self.h)
            self.h = _Closed()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ------------------------------------------------------------ writes
    def insert_batch(self, keys, values):
        """Sequential-insert semantics; returns per-key status: None (ok) or
        ('corrupted', Level, Bucket)."""
        n = len(keys)
        if n == 0:
            return []
        kt, kh, ko = terms.pack_keys(keys)
        vh, vo = terms.pack_values(values)
        st = np.zeros(n, np.int32)
        cl = np.zeros(n, np.uint32)
        cb = np.zeros(n, np.uint64)
        _lib.check(self.L.st_insert_batch(self.h, n, _ptr(kt), _ptr(kh), _ptr(ko), _ptr(vh), _ptr(vo), _ptr(st),
                                          _ptr(cl), _ptr(cb)), 'st_insert_batch')
        return [None if st[i] == _lib.ST_OK else (terms.CORRUPTED, int(cl[i]), int(cb[i])) for i in range(n)]

    def insert_int64(self, keys, values):
        """keys: int64 ndarray [n]; values: uint8 ndarray [n, vlen] (host).
        Returns the number of keys rejected by path verification."""
        nc = ctypes.c_uint64(0)
        keys = np.ascontiguousarray(keys, np.int64)
        values = np.ascontiguousarray(values, np.uint8)
        _lib.check(self.L.st_insert_int64(self.h, len(keys), _ptr(keys), _ptr(values), values.shape[1], 0,
                                          ctypes.byref(nc)), 'st_insert_int64')
        return int(nc.value)

    def insert_int64_device(self, keys_ptr, vals_ptr, n, vlen, stream=None):
        """Same with device-resident inputs (int64 keys, n*vlen value bytes)
        written by work on `stream` (a hipStream_t handle, e.g. torch's
        ``current_stream().cuda_stream``; None / 0 = the null stream, torch's
        default): the library orders its reads after that stream's work
        (st_insert_int64_dev, an event, no host wait) and returns after its
        last read of them."""
        nc = ctypes.c_uint64(0)
        _lib.check(self.L.st_insert_int64_dev(self.h, n, ctypes.c_void_p(keys_ptr), ctypes.c_void_p(vals_ptr), vlen,
                                              ctypes.c_void_p(stream or None), ctypes.byref(nc)),
                   'st_insert_int64_dev')
        return int(nc.value)

    def corrupt(self, key):
        kt, kb = terms.key_parts(key)
        _lib.check(self.L.st_corrupt(self.h, kt, kb, len(kb)), 'st_corrupt')

    def store_node(self, level, bucket, node):
        """Raw Mod:store({Level,Bucket}, Node): no verification, no rehash."""
        if level == 0:
            if node in (terms.UNDEFINED, None):
                _lib.check(self.L.st_store_top(self.h, None, 0), 'st_store_top')
            else:
                _lib.check(self.L.st_store_top(self.h, bytes(node), 0), 'st_store_top')
        elif level == self.height + 1:
            keys = [k for k, _ in node]
            vals = [v for _, v in node]
            kt, kh, ko = terms.pack_keys(keys)
            vh, vo = terms.pack_values(vals)
            _lib.check(self.L.st_store_segment(self.h, bucket, len(node), _ptr(kt), _ptr(kh), _ptr(ko), _ptr(vh),
                                               _ptr(vo)), 'st_store_segment')
        else:
            ch = np.array([c for c, _ in node], np.uint64)
            hs = np.frombuffer(b''.join(bytes(h) for _, h in node) + b'\0', np.uint8).copy()
            for _, h in node:
                if len(h) != 17:
                    raise ValueError('inner entries are 17-byte hashes on the device path')
            _lib.check(self.L.st_store_inner(self.h, level, bucket, len(node), _ptr(ch), _ptr(hs)), 'st_store_inner')

    def delete_node(self, level, bucket):
        _lib.check(self.L.st_delete_node(self.h, level, bucket), 'st_delete_node')

    def set_record_top(self, top):
        _lib.check(self.L.st_set_record_top(self.h, None if top == terms.UNDEFINED else bytes(top)),
                   'st_set_record_top')

    # ------------------------------------------------------------ rehash / verify
    def rehash(self, upper=False):
        _lib.check(self.L.st_rehash(self.h, 1 if upper else 0), 'st_rehash')

    def verify(self, upper=False):
        ok = ctypes.c_int(0)
        _lib.check(self.L.st_verify(self.h, 1 if upper else 0, ctypes.byref(ok)), 'st_verify')
        return bool(ok.value)

    def top_hash(self):
        buf = ctypes.create_string_buffer(17)
        p = ctypes.c_int(0)
        _lib.check(self.L.st_top_hash(self.h, buf, ctypes.byref(p)), 'st_top_hash')
        return buf.raw if p.value else terms.UNDEFINED

    def level_entries(self, level):
        n = self.width ** (level - 1)
        present = np.zeros(n, np.uint8)
        hashes = np.zeros((n, 17), np.uint8)
        _lib.check(self.L.st_level_entries(self.h, level, _ptr(present), _ptr(hashes)), 'st_level_entries')
        return present, hashes

    # ------------------------------------------------------------ partition
    def set_etf_atoms(self, utf8):
        """ETF atom forms of leveldb snapshots: False = before OTP 26 (ATOM_EXT
        for Latin-1 atoms, the default), True = OTP 26+ (st_set_etf_atoms)."""
        _lib.check(self.L.st_set_etf_atoms(self.h, 1 if utf8 else 0), 'st_set_etf_atoms')

    def set_partition(self, seg_lo, seg_hi):
        """Own segments [seg_lo, seg_hi) only (st_set_partition)."""
        _lib.check(self.L.st_set_partition(self.h, int(seg_lo), int(seg_hi)), 'st_set_partition')

    def combine_upper(self, present16, hashes17):
        """Store the 16 level-2 entries and recompute level 1 + top (st_combine_upper)."""
        present16 = np.ascontiguousarray(present16, np.uint8)
        hashes17 = np.ascontiguousarray(hashes17, np.uint8).reshape(16, 17)
        _lib.check(self.L.st_combine_upper(self.h, _ptr(present16), _ptr(hashes17)), 'st_combine_upper')

    def num_entries(self):
        return int(self.L.st_num_entries(self.h))

    def mem_stats(self):
        """Device bytes of this tree by part (st_mem_stats)."""
        v = (ctypes.c_uint64 * 6)()
        _lib.check(self.L.st_mem_stats(self.h, v), 'st_mem_stats')
        return dict(zip(('slots', 'csr', 'tiles', 'spare_csr', 'overlay', 'freed_block_cache'), [int(x) for x in v]))

    def sync(self):
        _lib.check(self.L.st_sync(self.h), 'st_sync')

    # ------------------------------------------------------------ reads
    def _take(self, rp):
        try:
            return rp.contents
        except ValueError:
            raise _lib.DeviceError('null result')

    def get1(self, key):
        """get/2 of one key through st_get1 (no result block): the value,
        'notfound' or ('corrupted', L, B)."""
        kt, kb = terms.key_parts(key)
        if self._g1 is None:
            self._g1 = (ctypes.create_string_buffer(4096), ctypes.c_uint32(), ctypes.c_uint32(), ctypes.c_uint64())
        buf, vl, cl, cb = self._g1
        rc = self.L.st_get1(self.h, kt, kb, len(kb), buf, 4096, ctypes.byref(vl), ctypes.byref(cl), ctypes.byref(cb))
        if rc == _lib.ST_OK:
            return buf.raw[:vl.value]
        if rc == _lib.ST_NOTFOUND:
            return terms.NOTFOUND
        if rc == _lib.ST_CORRUPTED:
            return (terms.CORRUPTED, int(cl.value), int(cb.value))
        if rc == _lib.ST_EINVAL and vl.value > 4096:   # a long value: the batch call
            return self.get_batch([key])[0]
        _lib.check(rc, 'st_get1')

    def insert1(self, key, value):
        """insert/3 of one key through st_insert1: None or ('corrupted', L, B)."""
        if not isinstance(value, (bytes, bytearray)):
            raise TypeError('function_clause: synctree values are binaries (synctree.erl:190)')
        kt, kb = terms.key_parts(key)
        if self._i1 is None:
            self._i1 = (ctypes.c_uint32(), ctypes.c_uint64())
        cl, cb = self._i1
        rc = self.L.st_insert1(self.h, kt, kb, len(kb), bytes(value), len(value), ctypes.byref(cl), ctypes.byref(cb))
        if rc == _lib.ST_OK:
            return None
        if rc == _lib.ST_CORRUPTED:
            return (terms.CORRUPTED, int(cl.value), int(cb.value))
        _lib.check(rc, 'st_insert1')

    def get_batch(self, keys):
        n = len(keys)
        if n == 0:
            return []
        kt, kh, ko = terms.pack_keys(keys)
        rp = ctypes.POINTER(_lib.StResult)()
        _lib.check(self.L.st_get_batch(self.h, n, _ptr(kt), _ptr(kh), _ptr(ko), ctypes.byref(rp)), 'st_get_batch')
        try:
            r = self._take(rp)
            out = []
            for i in range(n):
                s = r.status[i]
                if s == _lib.ST_OK:
                    out.append(_bytes(r.aheap, r.aoff[i], r.aoff[i + 1]))
                elif s == _lib.ST_NOTFOUND:
                    out.append(terms.NOTFOUND)
                else:
                    out.append((terms.CORRUPTED, int(r.clevel[i]), int(r.cbucket[i])))
            return out
        finally:
            self.L.st_free_result(rp)

    def _images(self, fn, level, buckets):
        n = len(buckets)
        bk = np.array(buckets, np.uint64)
        rp = ctypes.POINTER(_lib.StResult)()
        _lib.check(fn(self.h, level, n, _ptr(bk), ctypes.byref(rp)), 'node images')
        try:
            r = self._take(rp)
            out = []
            for i in range(n):
                if r.status[i] == _lib.ST_CORRUPTED:
                    out.append((terms.CORRUPTED, int(r.clevel[i]), int(r.cbucket[i])))
                    continue
                e0, e1 = r.eoff[i], r.eoff[i + 1]
                if level == 0:
                    out.append(_bytes(r.hash17, 17 * e0, 17 * e1) if e1 > e0 else terms.UNDEFINED)
                elif level <= self.height:
                    out.append([(int(r.child[e]), _bytes(r.hash17, 17 * e, 17 * e + 17)) for e in range(e0, e1)])
                else:
                    out.append([(terms.key_from_parts(r.ktype[e], _bytes(r.kheap, r.koff[e], r.koff[e + 1])),
                                 _bytes(r.aheap, r.aoff[e], r.aoff[e + 1])) for e in range(e0, e1)])
            return out
        finally:
            self.L.st_free_result(rp)

    def exchange_get_batch(self, level, buckets):
        """Verified node images (exchange_get/3 for level >= 1)."""
        return self._images(self.L.st_exchange_get_batch, level, buckets)

    def fetch_batch(self, level, buckets):
        """Raw node images (Mod:fetch/3, no verification)."""
        return self._images(self.L.st_fetch_batch, level, buckets)

    def segments_of(self, keys):
        kt, kh, ko = terms.pack_keys(keys)
        out = np.zeros(len(keys), np.uint64)
        _lib.check(self.L.st_segment_of_batch(self.h, len(keys), _ptr(kt), _ptr(kh), _ptr(ko), _ptr(out)),
                   'st_segment_of_batch')
        return [int(x) for x in out]

    def compare(self, remote, filt=_lib.ST_FILTER_ALL):
        """Device compare (K3).  Returns ('ok', [(seg, key, (va, vb))...]) in
        reference order, or ('corrupted', side, (corrupted, L, B))."""
        rp = ctypes.POINTER(_lib.StResult)()
        cl, cb, cs = ctypes.c_uint32(), ctypes.c_uint64(), ctypes.c_int()
        rc = _lib.check(self.L.st_compare(self.h, remote.h, filt, ctypes.byref(rp), ctypes.byref(cl), ctypes.byref(cb),
                                          ctypes.byref(cs)), 'st_compare')
        if rc == _lib.ST_CORRUPTED:
            return ('corrupted', 'local' if cs.value == 0 else 'remote', (terms.CORRUPTED, int(cl.value), int(cb.value)))
        try:
            r = self._take(rp)
            out = []
            for i in range(int(r.n_entries)):
                kind = r.kind[i]
                k = terms.key_from_parts(r.ktype[i], _bytes(r.kheap, r.koff[i], r.koff[i + 1]))
                va = terms.NONE if kind == _lib.ST_DIFF_REMOTE_ONLY else _bytes(r.aheap, r.aoff[i], r.aoff[i + 1])
                vb = terms.NONE if kind == _lib.ST_DIFF_LOCAL_ONLY else _bytes(r.bheap, r.boff[i], r.boff[i + 1])
                out.append((int(r.seg[i]), k, (va, vb)))
            return ('ok', out)
        finally:
            self.L.st_free_result(rp)

    def compare_device(self, remote, filt=_lib.ST_FILTER_ALL):
        """Device compare with results left on the device: number of diffs or
        ('corrupted', ...)."""
        nd, cl, cb, cs = ctypes.c_uint64(), ctypes.c_uint32(), ctypes.c_uint64(), ctypes.c_int()
        rc = _lib.check(self.L.st_compare_device(self.h, remote.h, filt, ctypes.byref(nd), ctypes.byref(cl),
                                                 ctypes.byref(cb), ctypes.byref(cs)), 'st_compare_device')
        if rc == _lib.ST_CORRUPTED:
            return ('corrupted', 'local' if cs.value == 0 else 'remote', (terms.CORRUPTED, int(cl.value), int(cb.value)))
        return int(nd.value)

    def compare_stats(self):
        """(visited nodes per level [0..H+1], final-level segment bytes) of the
        last compare on this tree (st_compare_stats)."""
        v = np.zeros(40, np.uint64)
        b = ctypes.c_uint64()
        _lib.check(self.L.st_compare_stats(self.h, v.ctypes.data_as(_lib.u64p), 40, ctypes.byref(b)),
                   'st_compare_stats')
        return [int(x) for x in v[:self.height + 2]], int(b.value)

    def exchange_apply(self, remote):
        """riak_ensemble_exchange.erl:71-97 against one remote tree, as one
        device batch (st_exchange_apply).  Returns ('ok', info),
        ('exchange_failed', info) for the valid_obj_hash function_clause
        crash (diffs before it applied), or ('corrupted', side, tuple) when
        the compare meets a corrupted node (nothing applied)."""
        nd, na, nr, cr = ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_int()
        cl, cb, cs = ctypes.c_uint32(), ctypes.c_uint64(), ctypes.c_int()
        rc = _lib.check(self.L.st_exchange_apply(self.h, remote.h, ctypes.byref(nd), ctypes.byref(na), ctypes.byref(nr),
                                                 ctypes.byref(cr), ctypes.byref(cl), ctypes.byref(cb), ctypes.byref(cs)),
                        'st_exchange_apply')
        if rc == _lib.ST_CORRUPTED:
            return ('corrupted', 'local' if cs.value == 0 else 'remote', (terms.CORRUPTED, int(cl.value), int(cb.value)))
        info = {'diffs': int(nd.value), 'applied': int(na.value), 'rejected': int(nr.value)}
        return ('exchange_failed' if cr.value else 'ok', info)

    def exchange_plan(self, remote):
        """Dry run of exchange_apply (st_exchange_plan): ('ok' | 'exchange_failed',
        {'diffs', 'take'}) or ('corrupted', side, tuple); nothing applied."""
        nd, nt, cr = ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_int()
        cl, cb, cs = ctypes.c_uint32(), ctypes.c_uint64(), ctypes.c_int()
        rc = _lib.check(self.L.st_exchange_plan(self.h, remote.h, ctypes.byref(nd), ctypes.byref(nt), ctypes.byref(cr),
                                                ctypes.byref(cl), ctypes.byref(cb), ctypes.byref(cs)), 'st_exchange_plan')
        if rc == _lib.ST_CORRUPTED:
            return ('corrupted', 'local' if cs.value == 0 else 'remote', (terms.CORRUPTED, int(cl.value), int(cb.value)))
        return ('exchange_failed' if cr.value else 'ok', {'diffs': int(nd.value), 'take': int(nt.value)})

    # ------------------------------------------------------------ LevelDB format
    def snapshot_leveldb(self, tree_id=b''):
        """The synctree_leveldb records of this tree (src/synctree_leveldb.erl:
        104-109, 134-152), encoded on the device: list of (key, value) bytes
        in (Level, Bucket) order."""
        rp = ctypes.POINTER(_lib.StKv)()
        tid = bytes(tree_id)
        _lib.check(self.L.st_snapshot_leveldb(self.h, tid, len(tid), ctypes.byref(rp)), 'st_snapshot_leveldb')
        try:
            kv = rp.contents
            n = int(kv.n)
            ko = np.ctypeslib.as_array(kv.koff, (n + 1,)).copy()
            vo = np.ctypeslib.as_array(kv.voff, (n + 1,)).copy()
            kh = _bytes(kv.kheap, 0, ko[n])
            vh = _bytes(kv.vheap, 0, vo[n])
        finally:
            self.L.st_free_kv(rp)
        return [(kh[ko[i]:ko[i + 1]], vh[vo[i]:vo[i + 1]]) for i in range(n)]

    def snapshot_leveldb_device(self, tree_id=b''):
        """Device-only encode (bench): (records, key bytes, value bytes)."""
        n, kb, vb = ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_uint64()
        tid = bytes(tree_id)
        _lib.check(self.L.st_snapshot_leveldb_device(self.h, tid, len(tid), ctypes.byref(n), ctypes.byref(kb),
                                                     ctypes.byref(vb)), 'st_snapshot_leveldb_device')
        return int(n.value), int(kb.value), int(vb.value)

    def restore_leveldb(self, records, tree_id=b''):
        """Replace the tree with the nodes in LevelDB records [(key, value)]
        and reload #tree.top_hash from {0,0} (synctree.erl:151-175).
        Returns (nodes loaded, undecodable nodes skipped)."""
        kh, ko = terms.pack_blobs([k for k, _ in records])
        vh, vo = terms.pack_blobs([v for _, v in records])
        nl, ns = ctypes.c_uint64(), ctypes.c_uint64()
        tid = bytes(tree_id)
        _lib.check(self.L.st_restore_leveldb(self.h, tid, len(tid), len(records), _ptr(kh), _ptr(ko), _ptr(vh),
                                             _ptr(vo), ctypes.byref(nl), ctypes.byref(ns)), 'st_restore_leveldb')
        return int(nl.value), int(ns.value)

    # ------------------------------------------------------------ timing
    def set_timing(self, on=True):
        _lib.check(self.L.st_set_timing(self.h, 1 if on else 0), 'st_set_timing')

    def kernel_stats(self, kernel):
        n, ms = ctypes.c_uint64(), ctypes.c_double()
        _lib.check(self.L.st_kernel_stats(self.h, kernel.encode(), ctypes.byref(n), ctypes.byref(ms)), 'stats')
        return int(n.value), float(ms.value)

    def set_stream(self, stream_handle):
        _lib.check(self.L.st_set_stream(self.h, ctypes.c_void_p(stream_handle)), 'st_set_stream')

    def page_stats(self):
        """(pages in use, batches through the pages, page builds, folds,
        entry slots of segments moved to new pages, value bytes of the
        segments the batches touched) -- st_page_stats."""
        v = (ctypes.c_uint64 * 6)()
        _lib.check(self.L.st_page_stats(self.h, v), 'st_page_stats')
        return tuple(int(x) for x in v)

    def debug_knob(self, knob, value):
        """Fault injection for tests (st_debug_knob)."""
        _lib.check(self.L.st_debug_knob(self.h, knob, int(value)), 'st_debug_knob')


# ---------------------------------------------------------------------------
# The backend behaviour (synctree_ets.erl:22-66) over a DeviceTree state.

def new(opts=()):
    opts = dict(opts) if opts else {}
    return DeviceTree(opts.get('width', 16), opts.get('segments', 1 << 20), opts.get('device', 0))


def fetch(key, default, state):
    level, bucket = key
    img = state.fetch_batch(level, [bucket])[0]
    if level == 0:
        return default if img == terms.UNDEFINED else img
    return img if img else default


def exists(key, state):
    level, bucket = key
    img = state.fetch_batch(level, [bucket])[0]
    return img != terms.UNDEFINED and img != []


def store(key, val, state):
    state.store_node(key[0], key[1], val)
    return state


def store_batch(updates, state):
    """Mod:store/2: puts (deletes as 'deleted' markers) then deletes."""
    for u in updates:
        if u[0] == 'put':
            state.store_node(u[1][0], u[1][1], u[2])
    for u in updates:
        if u[0] == 'delete':
            state.delete_node(u[1][0], u[1][1])
    return state


def rehash_group(trees):
    """rehash/1 of every tree in `trees` (one geometry, one device) as one
    device batch (st_rehash_group): ensembles sharded onto one GPU."""
    if not trees:
        return
    L = trees[0].L
    arr = (ctypes.c_void_p * len(trees))(*[t.h.value for t in trees])
    _lib.check(L.st_rehash_group(arr, len(trees)), 'st_rehash_group')


def insert1_multi(trees, keys, values):
    """insert/3 of keys[i] -> values[i] into trees[i] for every i, as ONE device
    launch over all the trees (st_insert1_multi).  Returns per request None or
    ('corrupted', Level, Bucket)."""
    n = len(trees)
    if n == 0:
        return []
    for v in values:
        if not isinstance(v, (bytes, bytearray)):
            raise TypeError('function_clause: synctree values are binaries (synctree.erl:190)')
    L = trees[0].L
    arr = (ctypes.c_void_p * n)(*[t.h.value for t in trees])
    kt, kh, ko = terms.pack_keys(keys)
    vh, vo = terms.pack_values(values)
    st = np.zeros(n, np.int32)
    cl = np.zeros(n, np.uint32)
    cb = np.zeros(n, np.uint64)
    _lib.check(L.st_insert1_multi(arr, n, _ptr(kt), _ptr(kh), _ptr(ko), _ptr(vh), _ptr(vo), _ptr(st), _ptr(cl),
                                  _ptr(cb)), 'st_insert1_multi')
    return [None if st[i] == _lib.ST_OK else (terms.CORRUPTED, int(cl[i]), int(cb[i])) for i in range(n)]


def get1_multi(trees, keys, vcap=1 << 20):
    """get/2 of keys[i] in trees[i] for every i, as ONE device launch
    (st_get1_multi): the value, 'notfound' or ('corrupted', L, B) per request."""
    n = len(trees)
    if n == 0:
        return []
    L = trees[0].L
    arr = (ctypes.c_void_p * n)(*[t.h.value for t in trees])
    kt, kh, ko = terms.pack_keys(keys)
    vout = np.zeros(vcap, np.uint8)
    vo = np.zeros(n + 1, np.uint64)
    st = np.zeros(n, np.int32)
    cl = np.zeros(n, np.uint32)
    cb = np.zeros(n, np.uint64)
    rc = L.st_get1_multi(arr, n, _ptr(kt), _ptr(kh), _ptr(ko), _ptr(vout), vcap, _ptr(vo), _ptr(st), _ptr(cl), _ptr(cb))
    if rc == _lib.ST_ERANGE:   # too small: the call reported the bytes needed in vo[n]
        vcap = int(vo[n])
        vout = np.zeros(max(vcap, 1), np.uint8)
        rc = L.st_get1_multi(arr, n, _ptr(kt), _ptr(kh), _ptr(ko), _ptr(vout), vcap, _ptr(vo), _ptr(st), _ptr(cl),
                             _ptr(cb))
    _lib.check(rc, 'st_get1_multi')
    out = []
    for i in range(n):
        if st[i] == _lib.ST_OK:
            out.append(bytes(vout[int(vo[i]):int(vo[i + 1])]))
        elif st[i] == _lib.ST_NOTFOUND:
            out.append(terms.NOTFOUND)
        else:
            out.append((terms.CORRUPTED, int(cl[i]), int(cb[i])))
    return out


def tops_to_device(trees, dev_ptr, stream=None):
    """Top-hash records (18 B each: present, hash17) of `trees` into device
    memory at dev_ptr (st_tops_to_device_on), e.g. a torch uint8 tensor to
    all-gather across ranks; the write waits for the work enqueued on
    `stream` (None = the null stream, torch's default) before the call."""
    if not trees:
        return
    L = trees[0].L
    arr = (ctypes.c_void_p * len(trees))(*[t.h.value for t in trees])
    _lib.check(L.st_tops_to_device_on(arr, len(trees), ctypes.c_void_p(dev_ptr), ctypes.c_void_p(stream or None)),
               'st_tops_to_device_on')
