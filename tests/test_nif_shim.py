"""The Erlang NIF over the C-ABI (c_src/synctree_hip_nif.c):
compile-checked against the erl_nif API declarations (tests/nif_stub/, no
Erlang/OTP in this image), every NIF the backend module of INTEGRATION.md
calls is registered, and every library symbol the NIF calls is exported."""
import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
NIF = os.path.join(ROOT, 'c_src', 'synctree_hip_nif.c')


def _src():
    with open(NIF) as f:
        return f.read()


@pytest.mark.skipif(shutil.which('gcc') is None, reason='gcc missing')
def test_nif_compiles():
    r = subprocess.run(['gcc', '-fsyntax-only', '-Wall', '-Wextra', '-Werror', '-std=c99',
                        '-I', os.path.join(ROOT, 'tests', 'nif_stub'), '-I', os.path.join(ROOT, 'include'), NIF],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr


def _registered():
    tab = _src().split('static ErlNifFunc funcs[] = {')[1].split('};')[0]
    return {(m.group(1), int(m.group(2))) for m in re.finditer(r'\{"(\w+)", (\d+), nif_\w+', tab)}


def test_backend_calls_only_registered_nifs():
    """Every synctree_hip_nif:F(...) the Erlang side of INTEGRATION.md calls
    exists with that arity (store/2, get/2, corrupt/2, insert/3 included)."""
    with open(os.path.join(ROOT, 'INTEGRATION.md')) as f:
        doc = f.read()
    reg = _registered()
    calls = set()
    for m in re.finditer(r'synctree_hip_nif:(\w+)\(', doc):
        # arity: top-level commas up to the matching parenthesis
        i, depth, args, seen = m.end(), 1, 0, False
        while depth:
            c = doc[i]
            if c in '([{':
                depth += 1
            elif c in ')]}':
                depth -= 1
            elif c == ',' and depth == 1:
                args += 1
            elif not c.isspace() and depth >= 1:
                seen = True
            i += 1
        calls.add((m.group(1), args + 1 if seen else 0))
    assert calls, 'no NIF calls found in INTEGRATION.md'
    missing = sorted(calls - reg)
    assert not missing, missing
    for name in ('store', 'get', 'corrupt', 'insert', 'restore', 'snapshot', 'fetch', 'exchange_get', 'compare'):
        assert any(n == name for n, _ in reg), name


def test_nif_calls_exported_symbols():
    from riak_ensemble_amd import _lib
    used = set(re.findall(r'\b(st_[a-z0-9_]+)\(', _src()))
    assert used <= set(_lib.EXPORTED) | {'st_last_error', 'st_height', 'st_free_result', 'st_free_kv', 'st_destroy'}, \
        sorted(used - set(_lib.EXPORTED))
    import ctypes
    L = ctypes.CDLL(_lib.LIB_PATH)
    for s in used:
        assert hasattr(L, s), s
