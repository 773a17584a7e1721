"""Multi-GPU sharding: segment-range partition of one tree and
ensemble sharding with a top-hash all-gather.

CPU tests run the distributed orchestration of riak_ensemble_amd/parallel.py
over world-size 2 and 4 `gloo` process groups, with a CPU stand-in for the
per-rank device tree (the C restatement in oracle/, here only the checker's
building block), and check the combined top hash against the unpartitioned
restatement.  The GPU tests run real partitioned DeviceTrees on one MI355X,
exchanging the level-2 entries in-process, against the oracle.
"""
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from riak_ensemble_amd import parallel, workload


class OraclePartition:
    """CPU stand-in for a partitioned DeviceTree: the C restatement of one
    tree holding only the owned segments' keys; combine_upper hashes the root
    node from the 16 gathered level-2 entries (synctree.erl:255-259)."""

    def __init__(self, segments=1 << 20):
        import oracle_c
        self.C = oracle_c
        self.width, self.segments = 16, segments
        self.lo, self.hi = 0, segments
        self.keys = np.zeros(0, np.int64)
        self.vals = np.zeros((0, 17), np.uint8)
        self.t = None
        self.top = 'undefined'

    def set_partition(self, lo, hi):
        self.lo, self.hi = lo, hi

    def insert_int64(self, keys, vals):
        probe = self.C.OTree(16, self.segments)
        seg = np.array([probe.segment_of(int(k)) for k in keys])
        own = (seg >= self.lo) & (seg < self.hi)
        # last writer wins per key (sequential insert semantics)
        cat_k = np.concatenate([self.keys, keys[own]])
        cat_v = np.concatenate([self.vals, vals[own]])
        _, last = np.unique(cat_k[::-1], return_index=True)
        idx = len(cat_k) - 1 - last
        self.keys, self.vals = cat_k[idx], cat_v[idx]
        self.t = None

    def rehash(self):
        self.t = self.C.OTree(16, self.segments).bulk_load_int64(self.keys, self.vals)

    def level_entries(self, level):
        return self.t.level_entries(level)

    def combine_upper(self, present16, hashes17):
        import synctree_ref as R
        node = [(b, bytes(hashes17[b])) for b in range(16) if present16[b]]
        self.top = R.hash_node(node) if node else 'undefined'

    def top_hash(self):
        return self.top


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, n, segments, out):
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'oracle'))
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        keys = workload.keys_int63(n)
        vals = workload.obj_hash_values(n)
        pt = parallel.PartitionedTree(OraclePartition(segments), dist)
        pt.tree.insert_int64(keys, vals)
        pt.rehash()
        top1 = pt.top_hash()
        # incremental batch: overwrite the first half (Seq + n) and add new keys
        k2 = np.concatenate([keys[: n // 2], workload.keys_int63(n + n // 2)[n:]])
        v2 = workload.obj_hash_values(len(k2), seq0=n)
        pt.tree.insert_int64(k2, v2)
        pt.rehash()
        top2 = pt.top_hash()
        tops = parallel.gather_tops(dist, [top1, 'undefined'] if rank == 0 else [top2, top1])
        np.save(os.path.join(out, 'r%d.npy' % rank),
                np.frombuffer(top1 + top2, np.uint8))
        if rank == 0:
            with open(os.path.join(out, 'tops.bin'), 'wb') as f:
                f.write(b''.join(t if t != 'undefined' else bytes(17) for t in tops))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize('world', [2, 4])
def test_partitioned_tree_gloo(world, tmp_path):
    import oracle_c as C
    n, segments = 3000, 1 << 20
    mp.spawn(_worker, args=(world, _free_port(), n, segments, str(tmp_path)), nprocs=world, join=True)
    keys = workload.keys_int63(n)
    vals = workload.obj_hash_values(n)
    full1 = C.OTree(16, segments).bulk_load_int64(keys, vals).top_hash()
    t2 = C.OTree(16, segments).bulk_load_int64(keys, vals)
    k2 = np.concatenate([keys[: n // 2], workload.keys_int63(n + n // 2)[n:]])
    v2 = workload.obj_hash_values(len(k2), seq0=n)
    for k, v in zip(k2.tolist(), v2):
        t2.insert(int(k), bytes(v))
    full2 = t2.top_hash()
    for r in range(world):
        got = np.load(tmp_path / ('r%d.npy' % r)).tobytes()
        assert got[:17] == full1 and got[17:] == full2, 'rank %d disagrees with the unpartitioned tree' % r
    tops = (tmp_path / 'tops.bin').read_bytes()
    exp = [full1, bytes(17)] + [full2, full1] * (world - 1)
    assert tops == b''.join(exp)


def test_partition_range():
    assert parallel.partition_range(0, 1, 1 << 20) == (0, 1 << 20)
    assert parallel.partition_range(3, 8, 1 << 20) == (3 << 17, 4 << 17)
    with pytest.raises(ValueError):
        parallel.partition_range(0, 3, 1 << 20)


class _LocalGroup:
    """In-process stand-in for a process group: ranks = partitions held by
    this process (GPU tests on a one-GPU box)."""

    def __init__(self, rank, world):
        self.rank, self.world = rank, world

    def get_rank(self, group=None):
        return self.rank

    def get_world_size(self, group=None):
        return self.world


def _device_partitions(world, keys, vals):
    from riak_ensemble_amd import synctree_hip
    parts = []
    for r in range(world):
        t = synctree_hip.DeviceTree()
        parts.append(parallel.PartitionedTree(t, _LocalGroup(r, world)))
    for p in parts:
        assert p.tree.insert_int64(keys, vals) == 0
    return parts


def _combine_all(parts):
    rows = []
    for p in parts:
        pres, hashes = p.tree.level_entries(2)
        a, b = p.b2
        rows.append(np.concatenate([pres[a:b, None], hashes[a:b]], axis=1))
    rows = np.concatenate(rows)
    for p in parts:
        p.tree.combine_upper(rows[:, 0].copy(), rows[:, 1:].copy())


@pytest.mark.gpu
@pytest.mark.parametrize('world', [2, 4, 8])
def test_device_partition_parity(world):
    import oracle_c as C
    n = 200_000
    keys = workload.keys_int63(n)
    vals = workload.obj_hash_values(n)
    parts = _device_partitions(world, keys, vals)
    ot = C.OTree().bulk_load_int64(keys, vals)
    assert sum(p.tree.num_entries() for p in parts) == n
    for p in parts:
        p.tree.rehash()
    _combine_all(parts)
    for p in parts:
        assert p.top_hash() == ot.top_hash()
        # owned level-2 .. segment entries equal the unpartitioned tree's
        for lvl in (2, 3, 6):
            pa, ha = p.tree.level_entries(lvl)
            pb, hb = ot.level_entries(lvl)
            m = len(pa) // world
            sl = slice(p.rank * m, (p.rank + 1) * m)
            assert (pa[sl] == pb[sl]).all() and (ha[sl] == hb[sl]).all()
    # incremental batch through the insert path (dirty-path rehash), then combine
    k2 = np.concatenate([keys[:1000], workload.keys_int63(n + 500)[n:]])
    v2 = workload.obj_hash_values(len(k2), seq0=n)
    for p in parts:
        assert p.tree.insert_int64(k2, v2) == 0
    _combine_all(parts)
    for k, v in zip(k2.tolist(), v2):
        ot.insert(int(k), bytes(v))
    for p in parts:
        assert p.top_hash() == ot.top_hash()
    # and a full rehash of the partitions reproduces it
    for p in parts:
        p.tree.rehash()
    _combine_all(parts)
    assert all(p.top_hash() == ot.top_hash() for p in parts)


@pytest.mark.gpu
def test_partition_rejects_bad_ranges():
    from riak_ensemble_amd import synctree_hip, _lib
    t = synctree_hip.DeviceTree()
    with pytest.raises(Exception):
        t.set_partition(0, 12345)
    s = synctree_hip.DeviceTree(width=16, segments=4096)
    with pytest.raises(Exception):
        s.set_partition(0, 2048)
    t.set_partition(0, 1 << 19)
    with pytest.raises(Exception):
        t.rehash(upper=True)


@pytest.mark.gpu
def test_group_rehash_parity():
    """Ensemble sharding on one GPU: st_rehash_group over trees of different
    sizes (incl. an empty one and a corrupted-then-rehashed one) == per-tree
    rehash == the oracle."""
    import oracle_c as C
    from riak_ensemble_amd import synctree_hip
    sizes = [0, 1, 1000, 50_000, 200_000, 7]
    trees, oracles = [], []
    for e, n in enumerate(sizes):
        keys = workload.keys_int63(n, workload.SEED ^ e) if n else np.zeros(0, np.int64)
        vals = workload.obj_hash_values(n)
        t = synctree_hip.DeviceTree()
        if n:
            t.insert_int64(keys, vals)
        trees.append(t)
        oracles.append(C.OTree().bulk_load_int64(keys, vals) if n else C.OTree())
    # stale inner state in one tree: a raw segment store without rehash
    seg = int(np.nonzero(oracles[3].level_entries(6)[0])[0][5])
    node = oracles[3].node(6, seg)
    bad = [(node[0][0], b'\x00' + bytes(16))] + node[1:]
    trees[3].store_node(6, seg, bad)
    oracles[3].store_segment(seg, bad)
    oracles[3].rehash()
    synctree_hip.rehash_group(trees)
    for t, o in zip(trees, oracles):
        assert t.top_hash() == o.top_hash()
        for lvl in (2, 5, 6):
            pa, ha = t.level_entries(lvl)
            pb, hb = o.level_entries(lvl)
            assert (pa == pb).all() and (ha == hb).all()
        assert t.verify()
    # twice in a row (self-resetting counters) and against the single-tree path
    synctree_hip.rehash_group(trees[::-1])
    tops = [t.top_hash() for t in trees]
    for t in trees:
        t.rehash()
    assert [t.top_hash() for t in trees] == tops
