"""Seeded synthetic synctree workloads (BASELINE.md "Inputs for every row").

Keys: the first N distinct splitmix64 outputs (seed 0x5EED0001) masked to
[0, 2^63), used as Erlang integer keys (ensure_binary => <<K:64/big>>,
src/synctree.erl:261-262).  Values: the object hash <<0, Epoch:64, Seq:64>>
(src/riak_ensemble_peer.erl:1717-1724), 17 bytes, Epoch = 1, Seq = index.
"""
import numpy as np

SEED = 0x5EED0001
_M64 = (1 << 64) - 1


def splitmix64(seed, n, start=0):
    """n consecutive splitmix64 outputs (uint64 ndarray)."""
    with np.errstate(over='ignore'):
        i = np.arange(start + 1, start + n + 1, dtype=np.uint64)
        z = np.uint64(seed) + i * np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    return z


def keys_int63(n, seed=SEED):
    """First n distinct splitmix64 outputs masked to [0, 2^63), in generation order."""
    out = np.empty(0, np.int64)
    start = 0
    while len(out) < n:
        want = n - len(out) + 16
        z = (splitmix64(seed, want, start) & np.uint64(0x7FFFFFFFFFFFFFFF)).astype(np.int64)
        start += want
        cat = np.concatenate([out, z])
        _, first = np.unique(cat, return_index=True)
        out = cat[np.sort(first)]
    return out[:n]


def obj_hash_values(n, epoch=1, seq0=0):
    """[n, 17] uint8: <<0, Epoch:64/big, Seq:64/big>> with Seq = seq0 + index."""
    v = np.zeros((n, 17), np.uint8)
    e = np.array([epoch], '>u8').view(np.uint8)
    v[:, 1:9] = e
    seq = (np.arange(n, dtype=np.uint64) + np.uint64(seq0)).astype('>u8')
    v[:, 9:17] = seq.view(np.uint8).reshape(n, 8)
    return v


def test_values(keys):
    """[n, 8] uint8: <<(K*10):64>> like test/synctree_pure.erl:79."""
    k = (np.asarray(keys, np.int64).astype(np.uint64) * np.uint64(10)).astype('>u8')
    return k.view(np.uint8).reshape(len(keys), 8)
