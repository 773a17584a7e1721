"""ctypes binding of libsynctree_hip.so (include/synctree_hip.h).

The HIP library is the product: there is no CPU fallback.  Loading fails
loudly when the shared object is missing (build it with ``make`` or
``__graft_entry__.build()``), and every call raises on a device error.
"""
import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# ST_LIB: another build of the library (A/B runs of tools/); the default is the in-tree build
LIB_PATH = os.environ.get('ST_LIB') or os.path.join(_HERE, 'libsynctree_hip.so')

ST_OK, ST_NOTFOUND, ST_CORRUPTED = 0, 1, 2
ST_EINVAL, ST_EDEVICE, ST_ENOMEM, ST_ERANGE = -1, -2, -3, -4
ST_KEY_INT, ST_KEY_ATOM, ST_KEY_BINARY, ST_KEY_TERM = 0, 1, 2, 3
ST_FILTER_ALL, ST_FILTER_LOCAL_ONLY, ST_FILTER_REMOTE_ONLY = 0, 1, 2
ST_DIFF_BOTH, ST_DIFF_LOCAL_ONLY, ST_DIFF_REMOTE_ONLY = 0, 1, 2

u8p = ctypes.POINTER(ctypes.c_uint8)
u32p = ctypes.POINTER(ctypes.c_uint32)
u64p = ctypes.POINTER(ctypes.c_uint64)
i32p = ctypes.POINTER(ctypes.c_int32)


class StResult(ctypes.Structure):
    _fields_ = [('n', ctypes.c_uint64), ('status', i32p), ('clevel', u32p), ('cbucket', u64p), ('eoff', u64p),
                ('n_entries', ctypes.c_uint64), ('child', u64p), ('hash17', u8p), ('ktype', u8p), ('koff', u64p),
                ('kheap', u8p), ('aoff', u64p), ('aheap', u8p), ('boff', u64p), ('bheap', u8p), ('kind', u8p),
                ('seg', u64p)]


class StKv(ctypes.Structure):
    _fields_ = [('n', ctypes.c_uint64), ('koff', u64p), ('kheap', u8p), ('voff', u64p), ('vheap', u8p)]


class DeviceError(RuntimeError):
    pass


# name -> (restype, argtypes)
_SIGS = {
    'st_create': (ctypes.c_int, [ctypes.c_uint64, ctypes.c_uint64, ctypes.c_int, ctypes.POINTER(ctypes.c_void_p)]),
    'st_destroy': (None, [ctypes.c_void_p]),
    'st_set_stream': (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p]),
    'st_sync': (ctypes.c_int, [ctypes.c_void_p]),
    'st_height': (ctypes.c_uint32, [ctypes.c_void_p]),
    'st_width': (ctypes.c_uint64, [ctypes.c_void_p]),
    'st_segments': (ctypes.c_uint64, [ctypes.c_void_p]),
    'st_num_entries': (ctypes.c_uint64, [ctypes.c_void_p]),
    'st_mem_stats': (ctypes.c_int, [ctypes.c_void_p, u64p]),
    'st_last_error': (ctypes.c_char_p, []),
    'st_insert_batch': (ctypes.c_int, [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p,
                                       ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                       ctypes.c_void_p, ctypes.c_void_p]),
    'st_insert_int64': (ctypes.c_int, [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p,
                                       ctypes.c_uint32, ctypes.c_int, u64p]),
    'st_insert_int64_dev': (ctypes.c_int, [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p,
                                           ctypes.c_uint32, ctypes.c_void_p, u64p]),
    'st_corrupt': (ctypes.c_int, [ctypes.c_void_p, ctypes.c_uint8, ctypes.c_char_p, ctypes.c_uint32]),
    'st_store_inner': (ctypes.c_int, [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_uint32,
                                      ctypes.c_void_p, ctypes.c_void_p]),
    'st_store_segment': (ctypes.c_int, [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_void_p,
                                        ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]),
    'st_delete_node': (ctypes.c_int, [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint64]),
    'st_store_top': (ctypes.c_int, [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_int]),
    'st_set_record_top': (ctypes.c_int, [ctypes.c_void_p, ctypes.c_char_p]),
    'st_rehash': (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int]),
    'st_verify': (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.POINTER(ctypes.c_int)]),
    'st_top_hash': (ctypes.c_int, [ctypes.c_void_p, ctypes.c_char_p, ctypes.POINTER(ctypes.c_int)]),
    'st_level_entries': (ctypes.c_int, [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p]),
    'st_exchange_apply': (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                         ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                         ctypes.c_void_p]),
    'st_exchange_plan': (ctypes.c_int, [ctypes.c_void_p] * 8),
    'st_rehash_group': (ctypes.c_int, [ctypes.c_void_p, ctypes.c_uint32]),
    'st_set_partition': (ctypes.c_int, [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64]),
    'st_combine_upper': (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]),
    'st_free_result': (None, [ctypes.POINTER(StResult)]),
    'st_get_batch': (ctypes.c_int, [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p,
                                    ctypes.c_void_p, ctypes.POINTER(ctypes.POINTER(StResult))]),
    'st_exchange_get_batch': (ctypes.c_int, [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_void_p,
                                             ctypes.POINTER(ctypes.POINTER(StResult))]),
    'st_fetch_batch': (ctypes.c_int, [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_void_p,
                                      ctypes.POINTER(ctypes.POINTER(StResult))]),
    'st_compare': (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int,
                                  ctypes.POINTER(ctypes.POINTER(StResult)), u32p, u64p, ctypes.POINTER(ctypes.c_int)]),
    'st_compare_device': (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, u64p, u32p, u64p,
                                         ctypes.POINTER(ctypes.c_int)]),
    'st_segment_of_batch': (ctypes.c_int, [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p,
                                           ctypes.c_void_p, ctypes.c_void_p]),
    'st_free_kv': (None, [ctypes.POINTER(StKv)]),
    'st_snapshot_leveldb': (ctypes.c_int, [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_uint32,
                                           ctypes.POINTER(ctypes.POINTER(StKv))]),
    'st_snapshot_leveldb_device': (ctypes.c_int, [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_uint32, u64p, u64p,
                                                  u64p]),
    'st_restore_leveldb': (ctypes.c_int, [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_uint32, ctypes.c_uint64,
                                          ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, u64p,
                                          u64p]),
    'st_compare_stats': (ctypes.c_int, [ctypes.c_void_p, u64p, ctypes.c_uint32, u64p]),
    'st_tops_to_device': (ctypes.c_int, [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p]),
    'st_tops_to_device_on': (ctypes.c_int, [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p]),
    'st_set_etf_atoms': (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int]),
    'st_get1': (ctypes.c_int, [ctypes.c_void_p, ctypes.c_uint8, ctypes.c_char_p, ctypes.c_uint32, ctypes.c_void_p,
                               ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]),
    'st_insert1': (ctypes.c_int, [ctypes.c_void_p, ctypes.c_uint8, ctypes.c_char_p, ctypes.c_uint32, ctypes.c_char_p,
                                  ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p]),
    'st_key_record': (ctypes.c_int, [ctypes.c_uint8, ctypes.c_char_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_uint64,
                                     u64p]),
    'st_set_timing': (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int]),
    'st_kernel_stats': (ctypes.c_int, [ctypes.c_void_p, ctypes.c_char_p, u64p, ctypes.POINTER(ctypes.c_double)]),
    'st_debug_knob': (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_int64]),
    'st_page_stats': (ctypes.c_int, [ctypes.c_void_p, u64p]),
    'st_insert1_multi': (ctypes.c_int, [ctypes.c_void_p, ctypes.c_uint32] + [ctypes.c_void_p] * 8),
    'st_get1_multi': (ctypes.c_int, [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p,
                                     ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64] + [ctypes.c_void_p] * 4),
}
ST_DBG_SKIP_MAIL, ST_DBG_PAGES, ST_DBG_PAGE_CHECK, ST_DBG_PAGE_POISON, ST_DBG_PAGE_DOWN = 1, 2, 3, 4, 5

EXPORTED = sorted(_SIGS)
_lib = None


def load():
    """Load the HIP library (no fallback: raises if it was not built)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RuntimeError('libsynctree_hip.so not found at %s — build it (make / __graft_entry__.build()); '
                           'there is no CPU fallback' % LIB_PATH)
    L = ctypes.CDLL(LIB_PATH)
    for name, (res, args) in _SIGS.items():
        if os.environ.get('ST_LIB') and not hasattr(L, name):
            continue   # an older build under A/B: symbols it lacks stay unbound
        f = getattr(L, name)
        f.restype = res
        f.argtypes = args
    _lib = L
    return L


def last_error():
    return load().st_last_error().decode(errors='replace')


def check(rc, what=''):
    """Raise on library errors; pass ST_OK / ST_NOTFOUND / ST_CORRUPTED through."""
    if rc in (ST_OK, ST_NOTFOUND, ST_CORRUPTED):
        return rc
    msg = '%s failed (%d): %s' % (what, rc, last_error())
    if rc in (ST_EINVAL, ST_ERANGE):
        raise ValueError(msg)
    raise DeviceError(msg)
