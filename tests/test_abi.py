"""CPU checks of the drop-in boundary: the C-ABI library loads without a GPU
and exports every symbol include/synctree_hip.h declares (no compute calls)."""
import ctypes
import os
import re

import pytest

from riak_ensemble_amd import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, 'include', 'synctree_hip.h')


def declared_functions():
    src = open(HEADER).read()
    src = re.sub(r'/\*.*?\*/', '', src, flags=re.S)
    names = re.findall(r'\b(st_[a-z0-9_]+)\s*\(', src)
    return sorted(set(names))


def test_library_built():
    assert os.path.exists(_lib.LIB_PATH), 'run make / __graft_entry__.build()'


def test_exports_every_declared_symbol():
    L = ctypes.CDLL(_lib.LIB_PATH)
    declared = declared_functions()
    assert len(declared) >= 25
    missing = [n for n in declared if not hasattr(L, n)]
    assert not missing, missing


def test_binding_covers_header():
    assert sorted(_lib.EXPORTED) == declared_functions()


def test_load_is_loud_when_missing(monkeypatch, tmp_path):
    monkeypatch.setattr(_lib, 'LIB_PATH', str(tmp_path / 'nope.so'))
    monkeypatch.setattr(_lib, '_lib', None)
    with pytest.raises(RuntimeError):
        _lib.load()


def test_error_codes_map_to_exceptions():
    _lib.load()
    with pytest.raises(ValueError):
        _lib.check(_lib.ST_EINVAL, 'x')
    with pytest.raises(_lib.DeviceError):
        _lib.check(_lib.ST_EDEVICE, 'x')
    assert _lib.check(_lib.ST_CORRUPTED) == _lib.ST_CORRUPTED


def test_library_is_built_from_current_sources():
    """The in-tree .so is newer than every source it is built from (a stale
    build would test old kernels)."""
    import glob
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    lib = os.path.join(root, 'riak_ensemble_amd', 'libsynctree_hip.so')
    srcs = glob.glob(os.path.join(root, 'riak_ensemble_amd', 'csrc', '*'))
    stale = [s for s in srcs if os.path.getmtime(s) > os.path.getmtime(lib) + 1]
    assert not stale, 'rebuild (make): %s' % stale
