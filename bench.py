"""bench.py — synctree keys rehashed/s (+ build and exchange tree-diff rates)
on MI355X, per BASELINE.json.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--keys 10000000]

A step is one full ``synctree:rehash/1`` (src/synctree.erl:493-509) of a
device-resident 10M-key tree: K1 segment_hash over all 2^20 segments + K2
level_rehash for levels 5..1 + the top hash (BASELINE config 2).  With N GPUs
(torchrun, one rank per GPU) every rank owns its own ensemble's tree (keys
seeded SEED ^ rank): ensemble sharding, weak scaling, no collective in the
timed region.  An RCCL all-gather of the per-ensemble top hashes
runs once after timing to show the cross-GPU combine.

Also reported (rank 0): build = st_insert_int64 of the 10M keys from HBM into
an empty tree (key->segment, sort, merge, dirty rehash); compare = config 3
(two 10M-key trees, 0.1% of non-empty segments with a bumped first value,
rehashed) through the device K3 compare; the per-kernel roofline of K1 from
HIP events on the library's stream; the CPU baseline (oracle/ C port, one
host thread) rehashing the same 10M-key tree.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

# MI355X peaks (/opt/skills/guides/MI355X_MICROARCH.md): HBM3E 8.0 TB/s spec.
# Integer VALU, measured on gfx950 (tools/microbench/valu_peak.cpp,
# profiles/r01_valu_peak.txt): v_add_u32 / v_bitop3_b32 issue a wave64 in 2
# SIMD cycles, v_add3_u32 / v_alignbit_b32 in 4.  The MD5 block loop of
# k_segment_hash_tiled (ISA count) is 130 add + 64 bitop3
# (2 cyc) and 65 add3 + 64 alignbit (4 cyc) = 916 SIMD cycles per wave =
# 14.3 SIMD-cycles per 64-B block.
HBM_PEAK_GBS = 8000.0
SIMDS = 256 * 4
CLOCK_HZ = 2.4e9
MD5_SIMD_CYCLES_PER_BLOCK = 916.0 / 64
# HBM bytes of one K1 launch (k_segment_hash_tiled_p) from rocprofv3 PMC,
# separate FETCH_SIZE / WRITE_SIZE passes (profiles/r01_session5_pmc_summary.txt):
# FETCH_SIZE x 2 (gfx950 counts half of a wide coalesced 16-B/lane stream,
# MI355X_MICROARCH.md; the doubled 220.1 MB = 211.1 MB tiles + 8.4 MB tile
# metadata) + WRITE_SIZE (37.1 MB: 19 MB of entries stored as scattered
# 16-B + 2-B writes), KiB -> bytes.
K1_PMC_TRAFFIC_BYTES = int((2 * 107486.5 + 36233.6) * 1024)
METRIC = 'synctree keys rehashed/sec + exchange tree-diffs/sec at 10M keys, 1–8 GPUs'


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def md5_blocks(nbytes):
    return (np.asarray(nbytes, np.int64) + 8) // 64 + 1


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=20)
    ap.add_argument('--warmup', type=int, default=5)
    ap.add_argument('--keys', type=int, default=10_000_000)
    ap.add_argument('--no-cpu', action='store_true', help='skip the CPU baseline leg')
    ap.add_argument('--no-extras', action='store_true', help='skip build/compare/ensemble legs')
    ap.add_argument('--ensembles', type=int, default=32, help='config-4 leg: ensembles (trees) per GPU')
    ap.add_argument('--ensemble-keys', type=int, default=1_000_000, help='config-4 leg: keys per ensemble')
    ap.add_argument('--part-keys', type=int, default=100_000_000, help='config-5 leg: keys in the partitioned tree')
    ap.add_argument('--part-batches', type=int, default=5, help='config-5 leg: timed write batches')
    ap.add_argument('--part-batch-keys', type=int, default=1_000_000, help='config-5 leg: keys per write batch')
    args = ap.parse_args()

    import torch
    world = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    local = int(os.environ.get('LOCAL_RANK', '0'))
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group('nccl', device_id=torch.device('cuda', local))
    else:
        dist = None
        torch.cuda.set_device(local)
    dev = torch.device('cuda', local)

    from riak_ensemble_amd import synctree_hip, workload

    n = args.keys
    seed = workload.SEED ^ rank
    keys_h = workload.keys_int63(n, seed)
    vals_h = workload.obj_hash_values(n)
    keys_d = torch.from_numpy(keys_h).to(dev)
    vals_d = torch.from_numpy(vals_h).to(dev)
    torch.cuda.synchronize()

    tree = synctree_hip.DeviceTree(device=local)
    t0 = time.perf_counter()
    nc = tree.insert_int64_device(keys_d.data_ptr(), vals_d.data_ptr(), n, 17)
    torch.cuda.synchronize()
    build_s = time.perf_counter() - t0
    assert nc == 0 and tree.num_entries() == n
    top0 = tree.top_hash()

    # ---------------- timed region: K full rehashes
    for _ in range(args.warmup):
        tree.rehash()
    tree.sync()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        tree.rehash()
    tree.sync()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    el = time.perf_counter() - t0
    if dist:
        t = torch.tensor([el], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    assert tree.top_hash() == top0, 'rehash changed the top hash of a consistent tree'

    # per-kernel HIP-event timing on the library stream (same steps, timing on)
    tree.set_timing(True)
    tree.kernel_stats('*reset*')
    for _ in range(args.steps):
        tree.rehash()
    k1_n, k1_ms = tree.kernel_stats('segment_hash')
    k2_n, k2_ms = tree.kernel_stats('level_rehash')
    tree.set_timing(False)

    # cross-GPU combine of the ensembles' top hashes (RCCL all-gather, untimed)
    tops_ok = True
    if dist:
        from riak_ensemble_amd import parallel
        tops = parallel.gather_tops(dist, [top0], device=dev)
        tops_ok = len(tops) == world and tops[rank] == top0

    ms_per_step = el * 1000.0 / args.steps
    value = world * n * args.steps / el

    out = None
    if rank == 0:
        # algorithmic bytes / ops of K1 per launch
        S = 1 << 20
        counts = None
        pres, _ = tree.level_entries(6)
        nseg = int(pres.sum())
        # segment sizes from the level-5 images are not needed: values are fixed
        # 17 B, so bytes per segment = 17 * keys in segment.  Use the oracle-free
        # count from the device CSR through exchange_get is costly; instead the
        # block count follows from the per-segment key histogram computed on host.
        seg_of = None
        try:
            seg_of = _segment_histogram(tree, keys_h)
        except Exception as e:  # pragma: no cover
            log('histogram failed', e)
        # Algorithmic work of one K1 launch (k_segment_hash_tiled): the hash
        # input of every segment (its values, 17 B per key: MD5 padding is
        # computed, not data), the tile metadata (segment id + block count,
        # 2 x 4 B per segment; 16 B per 64-segment tile) and the 18-B entry
        # (md5 + tag) written per segment.  The tiles K1 actually streams hold
        # each message padded to whole 64-B blocks (64 B x blocks, reported
        # as tile_bytes); the PMC traffic shows what HBM really served.
        if seg_of is not None:
            seg_blocks = int(md5_blocks(seg_of[seg_of > 0] * 17).sum())
        else:
            seg_blocks = int(n * 17 / 64 + nseg)
        blocks = seg_blocks
        k1_bytes = 17 * n + S * 8 + (S // 64) * 16 + S * 18
        k1_avg_ms = max(k1_ms / max(k1_n, 1), 1e-9)
        achieved_gbs = k1_bytes / (k1_avg_ms / 1e3) / 1e9
        t_hbm = k1_bytes / (HBM_PEAK_GBS * 1e9)
        t_valu = blocks * MD5_SIMD_CYCLES_PER_BLOCK / (SIMDS * CLOCK_HZ)
        roof = {'bound': 'hbm' if t_hbm >= t_valu else 'valu', 'achieved': round(achieved_gbs, 1),
                'peak': HBM_PEAK_GBS, 'unit': 'GB/s', 'frac': round(achieved_gbs / HBM_PEAK_GBS, 4),
                'traffic': K1_PMC_TRAFFIC_BYTES,
                'kernel': 'k_segment_hash_tiled_p (K1 segment_hash)', 'kernel_avg_ms': round(k1_avg_ms, 4),
                'bytes_per_launch': k1_bytes, 'tile_bytes_per_launch': 64 * seg_blocks, 'md5_blocks_per_launch': blocks,
                't_min_hbm_us': round(t_hbm * 1e6, 2),
                'valu': {'t_min_us': round(t_valu * 1e6, 2), 'frac': round(t_valu / (k1_avg_ms / 1e3), 4),
                         'simd_cycles_per_block': round(MD5_SIMD_CYCLES_PER_BLOCK, 2),
                         'peak': '1024 SIMDs x 2.4 GHz'},
                'level_rehash_avg_ms_per_step': round(k2_ms / max(args.steps, 1), 4),
                'level_rehash_kernel': 'k_levels_flow16 (levels 5..1 + top, one launch)'}
        out = {'metric': METRIC, 'value': round(value, 1), 'unit': 'keys/s', 'n_gpus': world,
               'steps': args.steps, 'warmup': args.warmup, 'ms_per_step': round(ms_per_step, 4),
               'higher_is_better': True, 'scaling': 'weak', 'vs_baseline': None, 'dtype': 'u32',
               'data': 'synthetic: first N distinct splitmix64 keys (seed 0x5EED0001 ^ rank) masked to 63 bits, '
                       '17-byte obj-hash values <<0,1:64,Seq:64>>',
               'config': {'workload': 'config2: full rehash of a 10M-key synctree per GPU (W=16, 2^20 segments)',
                          'keys_per_gpu': n, 'width': 16, 'segments': S,
                          'parallelism': 'ensemble-sharded: one tree per GPU, no collective in the timed region'},
               'roofline': roof,
               'rehash_top_hash': top0.hex(), 'tops_allgather_ok': tops_ok,
               'build': {'keys_per_s': round(n / build_s, 1), 'seconds': round(build_s, 4),
                         'note': 'first st_insert_int64 from HBM into an empty tree (includes allocator warm-up)'}}
        if not args.no_extras:
            out['build'] = _bench_build(synctree_hip, keys_d, vals_d, n, local, torch)
            out['compare'] = _bench_compare(synctree_hip, tree, keys_h, vals_h, keys_d, vals_d, n, local, torch)
            out['leveldb'] = _bench_leveldb(synctree_hip, tree, local, torch)
    tree.close()
    del keys_d, vals_d
    if not args.no_extras:
        # config 5 runs on every rank (one tree partitioned by segment range)
        part = _bench_partition(synctree_hip, dist, args, local, torch)
        if rank == 0:
            out['partition'] = part
            out['ensembles'] = _bench_ensembles(synctree_hip, workload, args.ensembles, args.ensemble_keys, local, torch)
            out['config1'] = _bench_config1(synctree_hip, workload, local, torch, cpu=not args.no_cpu)
    if rank == 0:
        if not args.no_cpu:
            out['cpu_baseline'] = _cpu_baseline(keys_h, vals_h, top0)
    if dist:
        dist.barrier()
        dist.destroy_process_group()
    if rank == 0:
        print(json.dumps(out), flush=True)


def _bench_leveldb(synctree_hip, tree, local, torch, reps=5):
    """synctree_leveldb format of the 10M-key tree:
    device encode of every node record (k_snap_sizes + 3 scans + k_snap_write),
    the host-inclusive snapshot (D2H of the records), and restore into a fresh
    tree from those host records (host ETF decode + upload)."""
    import ctypes
    from riak_ensemble_amd import _lib
    L = _lib.load()
    tid = b'ens-1'
    tree.snapshot_leveldb_device(tid)   # warm-up
    tree.set_timing(True)
    kn = ('snap_entry_sizes', 'snap_sizes', 'snap_write', 'snap_entries')
    k0 = [tree.kernel_stats(k) for k in kn]
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        n, kb, vb = tree.snapshot_leveldb_device(tid)
    dt = (time.perf_counter() - t0) / reps
    k1 = [tree.kernel_stats(k) for k in kn]
    tree.set_timing(False)
    kms = [(b[1] - a[1]) / max(1, b[0] - a[0]) for a, b in zip(k0, k1)]
    rp = ctypes.POINTER(_lib.StKv)()
    t0 = time.perf_counter()
    _lib.check(L.st_snapshot_leveldb(tree.h, tid, len(tid), ctypes.byref(rp)), 'snapshot')
    host_s = time.perf_counter() - t0
    kv = rp.contents
    fresh = synctree_hip.DeviceTree(device=local)
    nl, ns = ctypes.c_uint64(), ctypes.c_uint64()
    t0 = time.perf_counter()
    _lib.check(L.st_restore_leveldb(fresh.h, tid, len(tid), kv.n, kv.kheap, kv.koff, kv.vheap, kv.voff,
                                    ctypes.byref(nl), ctypes.byref(ns)), 'restore')
    restore_s = time.perf_counter() - t0
    L.st_free_kv(rp)
    same = fresh.top_hash() == tree.top_hash() and int(nl.value) == n and int(ns.value) == 0
    fresh.close()
    return {'records': n, 'key_bytes': kb, 'value_bytes': vb,
            'device_encode_ms': round(dt * 1e3, 3),
            'kernel_ms': {k: round(m, 4) for k, m in zip(kn, kms)},
            # k_snap_entries per entry: koff 8 + key record 9 + voff 8 + value 17
            # + entry offset 8 read, the entry's ETF bytes written (the values
            # heap minus list headers/NILs and inner-node records)
            'entries_roofline': _entries_roof(tree, vb, kms[3]),
            'encode_GB_per_s_written': round((kb + vb) / dt / 1e9, 1),
            'snapshot_to_host_ms': round(host_s * 1e3, 1),
            'restore_from_host_ms': round(restore_s * 1e3, 1),
            'restore_same_top_hash': bool(same),
            'what': 'config2 tree (10M keys): every node as <<0,Id,Level,encode_unsigned(Bucket)>> => '
                    'term_to_binary(Node) (synctree_leveldb.erl:104-152); restore = new/5 + reload_top_hash'}


def _entries_roof(tree, vb, ms):
    ne = tree.num_entries()
    # entry bytes = value bytes - {0,0} record - inner-node records - segment
    # list headers/NILs (7 B per non-empty segment)
    inner = 0
    for L in range(2, tree.height + 2):
        p = tree.level_entries(L)[0]
        ids = np.nonzero(p)[0]
        inner += 7 * int(p.reshape(-1, tree.width).any(1).sum()) + int((24 + np.where(ids < 256, 2, 5)).sum())
    nseg = int(tree.level_entries(tree.height + 1)[0].sum())
    written = vb - 23 - inner - 7 * nseg
    algo = ne * (8 + 9 + 8 + 17 + 8) + written
    gbs = algo / (ms / 1e3) / 1e9 if ms > 0 else 0.0
    return {'bound': 'hbm', 'achieved': round(gbs, 1), 'peak': HBM_PEAK_GBS, 'unit': 'GB/s',
            'frac': round(gbs / HBM_PEAK_GBS, 4), 'bytes_per_launch': int(algo)}


def _segment_histogram(tree, keys_h):
    """Keys per segment via the device key->segment map (st_segment_of_batch)."""
    segs = np.zeros(0, np.uint64)
    step = 1 << 21
    parts = []
    for i in range(0, len(keys_h), step):
        parts.append(np.array(tree.segments_of(keys_h[i:i + step].tolist()), np.int64))
    segs = np.concatenate(parts)
    return np.bincount(segs, minlength=1 << 20)


def _bench_build(synctree_hip, keys_d, vals_d, n, local, torch, reps=3):
    """Full build (insert of N keys from HBM into an empty tree)."""
    times = []
    for _ in range(reps + 1):
        t = synctree_hip.DeviceTree(device=local)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        t.insert_int64_device(keys_d.data_ptr(), vals_d.data_ptr(), n, 17)
        torch.cuda.synchronize()
        times.append(time.perf_counter() - t0)
        t.close()
    best = min(times[1:])
    return {'keys_per_s': round(n / best, 1), 'seconds': round(best, 4),
            'what': 'st_insert_int64: key->segment MD5, radix sort, run sort, merge, gather, dirty rehash (all levels)'}


def _bench_compare(synctree_hip, tree_a, keys_h, vals_h, keys_d, vals_d, n, local, torch, reps=10):
    """Config 3: B = A with the first value of every 1000th non-empty segment
    bumped (test/synctree_intercepts.erl:96-104) and rehashed."""
    pres, _ = tree_a.level_entries(6)
    segs = np.nonzero(pres)[0][::1000].tolist()
    imgs = tree_a.exchange_get_batch(6, segs)
    mut = [(img[0][0], bytes([(img[0][1][0] + 1) % 256]) + img[0][1][1:]) for img in imgs]
    tb = synctree_hip.DeviceTree(device=local)
    tb.insert_int64_device(keys_d.data_ptr(), vals_d.data_ptr(), n, 17)
    tb.insert_batch([k for k, _ in mut], [v for _, v in mut])
    nd = tree_a.compare_device(tb)
    assert nd == len(segs), (nd, len(segs))
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        tree_a.compare_device(tb)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / reps
    t0 = time.perf_counter()
    res = tree_a.compare(tb)
    dt_host = time.perf_counter() - t0
    assert res[0] == 'ok' and len(res[1]) == len(segs)
    # (B's bumped FIRST byte is the ?H_OBJ_NONE prefix: the reference exchange
    # would crash in valid_obj_hash on these diffs, and so does ours)
    assert tree_a.exchange_apply(tb)[0] == 'exchange_failed'
    tb.close()
    # riak_ensemble_exchange.erl:71-97 as one device batch: B2 = A with the
    # same keys' Seq advanced (last byte + 1, so B2 > A: valid_obj_hash holds);
    # compare + apply into a fresh copy of A, which then equals B2
    mut2 = [(k, v[:-1] + bytes([v[-1] + 1])) for k, v in
            ((img[0][0], img[0][1]) for img in imgs) if v[-1] < 255]
    tb2 = synctree_hip.DeviceTree(device=local)
    tb2.insert_int64_device(keys_d.data_ptr(), vals_d.data_ptr(), n, 17)
    tb2.insert_batch([k for k, _ in mut2], [v for _, v in mut2])
    ta = synctree_hip.DeviceTree(device=local)
    ta.insert_int64_device(keys_d.data_ptr(), vals_d.data_ptr(), n, 17)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    res_apply = ta.exchange_apply(tb2)
    torch.cuda.synchronize()
    dt_apply = time.perf_counter() - t0
    assert res_apply[0] == 'ok' and res_apply[1]['applied'] == len(mut2), res_apply
    assert ta.top_hash() == tb2.top_hash(), 'exchange did not converge the trees'
    ta.close()
    tb2.close()
    return {'tree_compares_per_s': round(1.0 / dt, 1), 'ms_per_compare': round(dt * 1e3, 4),
            'diff_keys': nd, 'diff_keys_per_s': round(nd / dt, 1),
            'ms_per_compare_incl_d2h_records': round(dt_host * 1e3, 4),
            'exchange_apply_ms': round(dt_apply * 1e3, 4),
            'exchange_apply': 'st_exchange_apply: compare + valid_obj_hash select + one batched insert/3 of the %d '
                              'newer remote values (dirty-path rehash); trees converge (equal top hashes)' % len(mut2),
            'what': 'config3: 10M vs 10M keys, every 1000th non-empty segment differs; K3 with per-node '
                    'self-verification, diff records materialised on device'}


def _bench_ensembles(synctree_hip, workload, E, nk, local, torch, reps=10):
    """Config 4 shape on one GPU: E independent ensembles x nk keys (keys
    seeded SEED ^ e), all rehashed as ONE batch (st_rehash_group) vs one
    st_rehash per tree."""
    trees = []
    for e in range(E):
        k = torch.from_numpy(workload.keys_int63(nk, workload.SEED ^ (e + 1))).to(torch.device('cuda', local))
        v = torch.from_numpy(workload.obj_hash_values(nk)).to(k.device)
        t = synctree_hip.DeviceTree(device=local)
        t.insert_int64_device(k.data_ptr(), v.data_ptr(), nk, 17)
        trees.append(t)
    torch.cuda.synchronize()
    tops = [t.top_hash() for t in trees]
    synctree_hip.rehash_group(trees)
    assert [t.top_hash() for t in trees] == tops
    t0 = time.perf_counter()
    for _ in range(reps):
        synctree_hip.rehash_group(trees)
    torch.cuda.synchronize()
    dt_g = (time.perf_counter() - t0) / reps
    t0 = time.perf_counter()
    for _ in range(reps):
        for t in trees:
            t.rehash()
    for t in trees:
        t.sync()
    dt_s = (time.perf_counter() - t0) / reps
    assert [t.top_hash() for t in trees] == tops
    for t in trees:
        t.close()
    return {'keys_per_s': round(E * nk / dt_g, 1), 'ms_per_batch': round(dt_g * 1e3, 4),
            'per_tree_rehash_keys_per_s': round(E * nk / dt_s, 1), 'ensembles': E, 'keys_per_ensemble': nk,
            'what': 'config4 shape per GPU: %d ensembles x %d keys rehashed as one st_rehash_group batch '
                    '(K1 over all trees\' tiles + one level-dataflow launch), vs st_rehash per tree' % (E, nk)}


def _dev_keys(seed, start, n, dev, torch):
    """splitmix64(seed + i), i = start+1 .. start+n, masked to 63 bits, on the
    device (a bijection before the mask: distinct keys with overwhelming
    probability; inserts are last-writer-wins anyway)."""
    return _dev_keys_at(seed, torch.arange(start, start + n, dtype=torch.int64, device=dev), dev, torch)


def _dev_values(seq, dev, torch, epoch=1):
    """<<0, Epoch:64, Seq:64>> rows for an int64 seq tensor (device)."""
    v = torch.zeros((seq.numel(), 17), dtype=torch.uint8, device=dev)
    v[:, 8] = epoch
    for b in range(8):
        v[:, 9 + b] = ((seq >> (56 - 8 * b)) & 0xFF).to(torch.uint8)
    return v


def _bench_partition(synctree_hip, dist, args, local, torch):
    """Config 5: one tree of part_keys keys partitioned by segment range over
    the ranks (st_set_partition); timed: part_batches write batches of
    part_batch_keys keys (50 % overwrites with Seq + 1, 50 % new keys), each an
    insert/3 batch with dirty-path rehash on every rank + the all-gather of the
    level-2 entries and level 1 + top (parallel.PartitionedTree.combine)."""
    from riak_ensemble_amd import parallel
    import numpy as np
    dev = torch.device('cuda', local)
    world = dist.get_world_size() if dist else 1
    grp = dist if dist else _SoloGroup()
    pt = parallel.PartitionedTree(synctree_hip.DeviceTree(device=local), grp, device=dev)
    N, B, K = args.part_keys, args.part_batch_keys, args.part_batches
    seed = 0x5EED0005
    chunk = 10_000_000
    t0 = time.perf_counter()
    for a in range(0, N, chunk):
        m = min(chunk, N - a)
        k = _dev_keys(seed, a, m, dev, torch)
        v = _dev_values(torch.arange(a, a + m, dtype=torch.int64, device=dev), dev, torch)
        pt.tree.insert_int64_device(k.data_ptr(), v.data_ptr(), m, 17)
        del k, v
    pt.combine()
    torch.cuda.synchronize()
    load_s = time.perf_counter() - t0
    rng = np.random.default_rng(5)
    batches = []
    for j in range(K + 1):
        old = torch.from_numpy(rng.integers(0, N, B // 2)).to(dev)          # overwrites: Seq + 1 of a loaded key
        k = torch.cat([_dev_keys_at(seed, old, dev, torch), _dev_keys(seed, N + j * B, B - B // 2, dev, torch)])
        seq = torch.cat([old + 1, torch.arange(N + j * B, N + j * B + (B - B // 2), device=dev)])
        batches.append((k.contiguous(), _dev_values(seq, dev, torch).contiguous()))
    # one warm-up batch, then K timed
    k, v = batches[0]
    pt.tree.insert_int64_device(k.data_ptr(), v.data_ptr(), B, 17)
    pt.combine()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for j in range(1, K + 1):
        k, v = batches[j]
        pt.tree.insert_int64_device(k.data_ptr(), v.data_ptr(), B, 17)
        pt.combine()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    el = time.perf_counter() - t0
    top = pt.top_hash()
    same = True
    if dist:
        t = torch.tensor([el], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
        tops = parallel.gather_tops(dist, [top], device=dev)
        same = all(x == top for x in tops)
    entries = pt.tree.num_entries()
    pt.tree.close()
    return {'batch_keys_per_s': round(K * B / el, 1), 'ms_per_batch': round(el * 1e3 / K, 4), 'batches': K,
            'batch_keys': B, 'tree_keys': N, 'ranks': world, 'entries_on_rank0': entries,
            'tops_agree_across_ranks': same, 'load_s': round(load_s, 3),
            'what': 'config5: %d-key tree partitioned by segment range over %d rank(s); per batch: insert/3 of %d keys '
                    '(50%% overwrites Seq+1, 50%% new; verify + dirty-path rehash) on every rank, all-gather of the '
                    'level-2 entries, level 1 + top (keys generated on device: splitmix64 masked to 63 bits)'
                    % (N, world, B)}


def _dev_keys_at(seed, idx, dev, torch):
    """Keys at arbitrary generation indices idx (0-based) of _dev_keys."""
    def c(x):
        return x - (1 << 64) if x >= 1 << 63 else x

    def lsr(z, k):
        return (z >> k) & ((1 << (64 - k)) - 1)
    z = c(seed) + (idx + 1) * c(0x9E3779B97F4A7C15)
    z = (z ^ lsr(z, 30)) * c(0xBF58476D1CE4E5B9)
    z = (z ^ lsr(z, 27)) * c(0x94D049BB133111EB)
    z = z ^ lsr(z, 31)
    return z & 0x7FFFFFFFFFFFFFFF


class _SoloGroup:
    @staticmethod
    def get_rank(group=None):
        return 0

    @staticmethod
    def get_world_size(group=None):
        return 1


def _bench_config1(synctree_hip, workload, local, torch, n=100_000, cpu=True):
    """Config 1: a 100k-key tree, full build (n inserts) + rehash + top hash.
    GPU: one st_insert_int64 batch + st_rehash.  CPU: the C restatement in
    reference-faithful mode (one verified insert per key, DFS rehash over all
    2^20 slots), one thread -- the reference Erlang cannot run here."""
    keys = workload.keys_int63(n, workload.SEED ^ 0x100)
    vals = workload.obj_hash_values(n)
    best = 1e9
    for _ in range(4):
        t = synctree_hip.DeviceTree(device=local)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        t.insert_int64(keys, vals)
        t.rehash()
        top = t.top_hash()
        best = min(best, time.perf_counter() - t0)
    # the per-key verified-path calls (get/2, insert/3,
    # synctree.erl:189-227) one at a time through the C-ABI (ctypes), i.e. the
    # low-batch latency path; the tree is the 100k-key one just built
    kl = [int(k) for k in keys[:200]]
    t0 = time.perf_counter()
    for k in kl:
        t.get_batch([k])
    gpu_get_us = (time.perf_counter() - t0) / len(kl) * 1e6
    t0 = time.perf_counter()
    for k in kl:
        t.insert_batch([k], [b'\x00' * 17])
    gpu_ins_us = (time.perf_counter() - t0) / len(kl) * 1e6
    t.close()
    out = {'gpu_keys_per_s': round(n / best, 1), 'gpu_ms': round(best * 1e3, 3),
           'what': 'config1: 100k keys, build + rehash + top_hash (GPU: host arrays in, one insert batch)',
           'per_key_latency_us': {'gpu_get': round(gpu_get_us, 1), 'gpu_insert': round(gpu_ins_us, 1),
                                  'what': 'one get/2 or insert/3 per C-ABI call (verified path + dirty-path '
                                          'rehash on the device), 200 calls, ctypes overhead included'}}
    if cpu:
        sys.path.insert(0, os.path.join(ROOT, 'oracle'))
        import oracle_c
        ot = oracle_c.OTree()
        t0 = time.perf_counter()
        for k, v in zip(keys.tolist(), vals):
            ot.insert(int(k), bytes(v))
        ot.rehash()
        ctop = ot.top_hash()
        dt = time.perf_counter() - t0
        t0 = time.perf_counter()
        for k in kl:
            ot.get(k)
        out['per_key_latency_us']['cpu_get'] = round((time.perf_counter() - t0) / len(kl) * 1e6, 1)
        t0 = time.perf_counter()
        for k in kl:
            ot.insert(k, b'\x00' * 17)
        out['per_key_latency_us']['cpu_insert'] = round((time.perf_counter() - t0) / len(kl) * 1e6, 1)
        assert ctop == top, 'config1: CPU restatement and GPU disagree'
        out['cpu'] = {'keys_per_s': round(n / dt, 1), 'seconds': round(dt, 3), 'cores': 1, 'kind': 'port',
                      'sample': 'oracle/synctree_oracle.c: 100k verified inserts (ctypes per key) + rehash + top_hash'}
    return out


def _cpu_baseline(keys_h, vals_h, top0, reps=2):
    sys.path.insert(0, os.path.join(ROOT, 'oracle'))
    import oracle_c
    t0 = time.perf_counter()
    ot = oracle_c.OTree().bulk_load_int64(keys_h, vals_h)
    load_s = time.perf_counter() - t0
    assert ot.top_hash() == top0, 'CPU port disagrees with the device top hash'
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        ot.rehash()
        ts.append(time.perf_counter() - t0)
    best = min(ts)
    return {'value': round(len(keys_h) / best, 1), 'unit': 'keys/s', 'cores': 1, 'kind': 'port',
            'sample': 'full synctree:rehash/1 restatement (oracle/synctree_oracle.c, DFS over all 2^20 segment '
                      'slots) of the same 10M-key tree, best of %d; tree load %.1f s untimed' % (reps, load_s),
            'seconds_per_rehash': round(best, 3)}


if __name__ == '__main__':
    main()
