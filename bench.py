"""bench.py — synctree keys rehashed/s (+ build, exchange tree-diffs/s and the
other BASELINE configs) on MI355X, per BASELINE.json.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--keys 10000000]

A step is one full ``synctree:rehash/1`` (src/synctree.erl:493-509) of a
device-resident 10M-key tree: K1 segment_hash over all 2^20 segments + the
inner levels 5..1 + the top hash (BASELINE config 2).  ``--gpus N`` with no
torchrun environment starts N ranks itself (``torch.distributed.run``, one
process per GPU) before any GPU call; every rank owns its own ensemble's tree
(keys seeded SEED ^ rank): ensemble sharding, weak scaling, no collective in
the timed region.  ``value`` = all ranks' keys / the slowest
rank's time.

Also reported (rank 0 unless noted):
  build      st_insert_int64 of the 10M keys from HBM into an empty tree
  compare    config 3: two 10M-key trees, every 1000th non-empty segment's
             first value bumped; K3 with the ordered diff records on the
             device (tree-diffs/s) and copied to the host; + compare roofline
  ensembles  config 4 per GPU (every rank): --ensembles trees x 1M keys, one
             st_rehash_group batch + the RCCL all-gather of every ensemble's
             top hash (st_tops_to_device -> all_gather_into_tensor)
  partition  config 5 (every rank): a 100M-key tree partitioned by segment
             range over the ranks, 1M-key write batches
  config1    100k keys build + rehash + top hash; per-key get/insert latency
  cold_l3    K1 with the 256 MiB Infinity Cache flushed before every launch
  cpu_baseline  the C port (oracle/) rehashing the same 10M-key tree on the
             host: 1 thread and every host core
The K1 roofline's ``traffic`` comes from rocprofv3 PMC passes (FETCH_SIZE,
WRITE_SIZE) run by this script on a K1-only child process (N = 1).
"""
import argparse
import json
import os
import shutil
import socket
import subprocess
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

# MI355X peaks (/opt/skills/guides/MI355X_MICROARCH.md): HBM3E 8.0 TB/s spec.
# Integer VALU, measured on gfx950 (tools/microbench/valu_peak.cpp,
# profiles/r01_valu_peak.txt): v_add_u32 / v_bitop3_b32 issue a wave64 in 2
# SIMD cycles, v_add3_u32 / v_alignbit_b32 in 4.  The MD5 block loop (ISA
# count) is 130 add + 64 bitop3 (2 cyc) and 65 add3 + 64
# alignbit (4 cyc) = 916 SIMD cycles per wave = 14.3 SIMD-cycles per block.
HBM_PEAK_GBS = 8000.0
SIMDS = 256 * 4
CLOCK_HZ = 2.4e9
MD5_SIMD_CYCLES_PER_BLOCK = 916.0 / 64
K1_KERNEL = 'k_rehash_fused'   # K1 segment_hash + the inner levels, one launch
METRIC = 'synctree keys rehashed/sec + exchange tree-diffs/sec at 10M keys, 1–8 GPUs'


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def md5_blocks(nbytes):
    return (np.asarray(nbytes, np.int64) + 8) // 64 + 1


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=200)   # 200 x ~66 us: a timed region of ~13 ms, so host jitter does not dominate
    ap.add_argument('--warmup', type=int, default=10)
    ap.add_argument('--keys', type=int, default=10_000_000)
    ap.add_argument('--no-cpu', action='store_true', help='skip the CPU baseline legs')
    ap.add_argument('--no-extras', action='store_true', help='skip every leg but the headline rehash')
    ap.add_argument('--no-pmc', action='store_true', help='skip the rocprofv3 PMC traffic passes')
    ap.add_argument('--no-cold', action='store_true', help='skip the cold-L3 launches (isolated kernel traces)')
    ap.add_argument('--ensembles', type=int, default=512,
                    help='config-4 leg: ensembles (trees) per GPU (4096 over 8 GPUs = 512)')
    ap.add_argument('--ensemble-keys', type=int, default=1_000_000, help='config-4 leg: keys per ensemble')
    ap.add_argument('--part-keys', type=int, default=100_000_000, help='config-5 leg: keys in the partitioned tree')
    ap.add_argument('--part-batches', type=int, default=30,
                    help='config-5 leg: timed write batches')
    ap.add_argument('--part-batch-keys', type=int, default=1_000_000, help='config-5 leg: keys per write batch')
    ap.add_argument('--pmc-probe', action='store_true', help=argparse.SUPPRESS)
    ap.add_argument('--trace-probe', action='store_true', help=argparse.SUPPRESS)
    ap.add_argument('--no-trace', action='store_true', help='skip the rocprofv3 kernel-trace pass (config-4 launch time)')
    return ap.parse_args()


def main():
    args = parse()
    if args.gpus > 1 and 'WORLD_SIZE' not in os.environ:
        # one process per GPU, started before this process touches the GPU
        cmd = [sys.executable, '-m', 'torch.distributed.run', '--nnodes=1', '--nproc-per-node', str(args.gpus),
               '--master-addr', '127.0.0.1', '--master-port', str(_free_port()), os.path.abspath(__file__)] + sys.argv[1:]
        sys.exit(subprocess.call(cmd))
    if args.pmc_probe:
        return pmc_probe(args)
    if args.trace_probe:
        return trace_probe(args)

    world = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    local = int(os.environ.get('LOCAL_RANK', '0'))
    pmc = None
    trace = None
    if rank == 0 and world == 1 and not args.no_pmc:
        pmc = k1_pmc_traffic(args)          # child processes, before this one touches the GPU
    if rank == 0 and world == 1 and not args.no_trace and not args.no_extras:
        trace = group_kernel_trace(args)    # likewise

    import torch
    ndev = torch.cuda.device_count()
    dev_index = local % max(ndev, 1)
    torch.cuda.set_device(dev_index)
    dev = torch.device('cuda', dev_index)
    dist = None
    coll_dev = dev
    if world > 1:
        import torch.distributed as dist
        if ndev >= world:
            dist.init_process_group('nccl', device_id=dev)
        else:   # more ranks than GPUs (a rehearsal on a small box): host collectives
            dist.init_process_group('gloo')
            coll_dev = torch.device('cpu')

    from riak_ensemble_amd import synctree_hip, workload

    n = args.keys
    seed = workload.SEED ^ rank
    keys_h = workload.keys_int63(n, seed)
    vals_h = workload.obj_hash_values(n)
    keys_d = torch.from_numpy(keys_h).to(dev)
    vals_d = torch.from_numpy(vals_h).to(dev)
    torch.cuda.synchronize()

    tree = synctree_hip.DeviceTree(device=dev_index)
    nc = tree.insert_int64_device(keys_d.data_ptr(), vals_d.data_ptr(), n, 17)
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
        t = torch.tensor([el], dtype=torch.float64, device=coll_dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    assert tree.top_hash() == top0, 'rehash changed the top hash of a consistent tree'

    # the kernel's GPU time without per-launch events: the span of the same
    # steps back to back on the library stream, two events around the loop
    # (the rehash is one launch: the span / steps is the launch's time plus
    # the gaps between launches, never more than the step's wall time)
    k1_span = _span_ms(tree, torch, dev, lambda: tree.rehash(), args.steps)
    # per-launch HIP events (timing on), reported beside it
    tree.set_timing(True)
    tree.kernel_stats('*reset*')
    for _ in range(args.steps):
        tree.rehash()
    k1_n, k1_ms = tree.kernel_stats('rehash_fused')
    tree.set_timing(False)

    # cross-GPU combine of the ensembles' top hashes (all-gather, untimed)
    tops_ok = True
    if dist:
        from riak_ensemble_amd import parallel
        tops = parallel.gather_tops(dist, [top0], device=coll_dev)
        tops_ok = len(tops) == world and tops[rank] == top0

    ms_per_step = el * 1000.0 / args.steps
    value = world * n * args.steps / el

    out = None
    if rank == 0:
        S = 1 << 20
        seg_of = _segment_histogram(tree, keys_h)
        seg_blocks = int(md5_blocks(seg_of[seg_of > 0] * 17).sum())
        # Algorithmic bytes of one rehash launch: every value
        # byte the hash reads (17 B per key; MD5 padding is computed, not
        # data) + one 17-byte entry <<0, MD5>> per PRESENT node written
        # (non-empty segments + present inner nodes, counted on this tree).
        # The kernel's own bookkeeping (tile metadata, presence bits, the
        # 18-B slot writes of absent segments) is traffic, not algorithm: it
        # is reported separately (bytes_incl_metadata).
        present_inner = _present_inner(tree)
        nonempty = int((seg_of > 0).sum())
        k1_bytes = 17 * n + 17 * (nonempty + present_inner)
        inner_nodes = sum(16 ** l for l in range(5))
        meta_bytes = 17 * n + S * 8 + (S // 64) * 16 + S // 8 + S * 18 + inner_nodes * 18 + 17 * 16 * 18
        seg_blocks += 349525   # inner-node MD5 blocks (full nodes: 5 each)
        k1_avg_ms = max(k1_span, 1e-9)
        k1_evt_ms = k1_ms / max(k1_n, 1)
        achieved_gbs = k1_bytes / (k1_avg_ms / 1e3) / 1e9
        t_hbm = k1_bytes / (HBM_PEAK_GBS * 1e9)
        t_valu = seg_blocks * MD5_SIMD_CYCLES_PER_BLOCK / (SIMDS * CLOCK_HZ)
        cold = {'frac': None, 'kernel_avg_ms': None, 'achieved_GBps': None} if args.no_cold else \
            _bench_cold_l3(tree, torch, dev, k1_bytes, k1_avg_ms)
        roof = {'bound': 'hbm', 'achieved': round(achieved_gbs, 1), 'peak': HBM_PEAK_GBS, 'unit': 'GB/s',
                'frac': round(achieved_gbs / HBM_PEAK_GBS, 4),
                'traffic': pmc['traffic_bytes'] if pmc and pmc.get('traffic_bytes') else None,
                'kernel': K1_KERNEL + ' (K1 segment_hash + levels 5..1 + top, one launch)',
                'kernel_avg_ms': round(k1_avg_ms, 4),
                'kernel_time_source': 'GPU span of %d back-to-back rehash launches on the library stream / %d '
                                      '(two events around the loop, none per launch)' % (args.steps, args.steps),
                'kernel_avg_ms_events': round(k1_evt_ms, 4),
                'bytes_per_launch': k1_bytes,
                'bytes_formula': '17 B x %d keys (values) + 17 B x (%d non-empty segments + %d present inner nodes) '
                                 '(SURVEY §8(d))' % (n, nonempty, present_inner),
                'bytes_incl_metadata': meta_bytes,
                'cold_l3': {'frac': cold['frac'], 'kernel_avg_ms': cold['kernel_avg_ms'],
                            'achieved': cold['achieved_GBps'],
                            'what': 'same launch after a 1 GiB read (the 256 MiB Infinity Cache flushed): tiles '
                                    'from HBM'},
                'tile_bytes_per_launch': 64 * seg_blocks,
                'md5_blocks_per_launch': seg_blocks, 't_min_hbm_us': round(t_hbm * 1e6, 2),
                'valu': {'t_min_us': round(t_valu * 1e6, 2), 'frac': round(t_valu / (k1_avg_ms / 1e3), 4),
                         'simd_cycles_per_block': round(MD5_SIMD_CYCLES_PER_BLOCK, 2),
                         'peak': '1024 SIMDs x 2.4 GHz'},
                'pmc': pmc}
        out = {'metric': METRIC, 'value': round(value, 1), 'unit': 'keys/s', 'n_gpus': world,
               'steps': args.steps, 'warmup': args.warmup, 'ms_per_step': round(ms_per_step, 4),
               'higher_is_better': True, 'scaling': 'weak', 'vs_baseline': None, 'dtype': 'u32',
               'data': 'synthetic: first N distinct splitmix64 keys (seed 0x5EED0001 ^ rank) masked to 63 bits, '
                       '17-byte obj-hash values <<0,1:64,Seq:64>>',
               'config': {'workload': 'config2: full rehash of a 10M-key synctree per GPU (W=16, 2^20 segments)',
                          'keys_per_gpu': n, 'width': 16, 'segments': S,
                          'parallelism': 'ensemble-sharded: one tree per GPU, no collective in the timed region'},
               'roofline': roof,
               'rehash_top_hash': top0.hex(), 'tops_allgather_ok': tops_ok}
        if not args.no_extras:
            out['build'] = _bench_build(synctree_hip, keys_d, vals_d, n, dev_index, torch)
            out['compare'] = _bench_compare(synctree_hip, tree, keys_d, vals_d, n, dev_index, torch)
            out['verify'] = _bench_verify(tree, n)
            # one exchange with one remote peer as riak_ensemble_exchange runs it:
            # verify_upper precheck (:58-65) + compare + valid_obj_hash apply (:71-97)
            out['exchange_total_ms'] = round(out['verify']['verify_upper']['ms'] +
                                             out['compare']['exchange_apply_ms'], 4)
            out['exchange_total_what'] = ('verify_upper ms + exchange_apply ms (st_exchange_apply = compare + '
                                          'select + one batched insert of the newer remote values)')
            out['leveldb'] = _bench_leveldb(synctree_hip, tree, dev_index, torch)
            out['rehash_after_mutation'] = _bench_rehash_after_mutation(tree, n, torch)
            out['repair'] = _bench_repair(tree, keys_h, torch)
    tree.close()
    del keys_d, vals_d
    if not args.no_extras:
        # configs 4 and 5 run on every rank
        ens = _bench_ensembles(synctree_hip, dist, coll_dev, args, dev_index, torch, trace)
        part = _bench_partition(synctree_hip, dist, coll_dev, args, dev_index, torch)
        if rank == 0:
            out['ensembles'] = ens
            out['partition'] = part
            out['config1'] = _bench_config1(synctree_hip, workload, dev_index, torch, cpu=not args.no_cpu)
    if rank == 0 and not args.no_cpu:
        out['cpu_baseline'] = _cpu_baseline(keys_h, vals_h, top0)
    if dist:
        dist.barrier()
        dist.destroy_process_group()
    if rank == 0:
        print(json.dumps(out), flush=True)


def _span_ms(tree, torch, dev, fn, k):
    """GPU time per call of k back-to-back calls of fn on the tree's stream:
    the tree is moved onto a torch stream for the loop and two events bracket
    it (no per-launch events: nothing is added between the launches)."""
    s = torch.cuda.Stream(device=dev)
    tree.set_stream(s.cuda_stream)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    e0.record(s)
    for _ in range(k):
        fn()
    e1.record(s)
    e1.synchronize()
    tree.set_stream(0)
    return e0.elapsed_time(e1) / k


# ---------------------------------------------------------------- PMC traffic of K1
def pmc_probe(args):
    """Child of k1_pmc_traffic (run under rocprofv3 --pmc): build the tree and
    rehash it a few times; only K1 launches are counted (kernel regex)."""
    import torch
    from riak_ensemble_amd import synctree_hip, workload
    n = args.keys
    keys = torch.from_numpy(workload.keys_int63(n, workload.SEED)).cuda()
    vals = torch.from_numpy(workload.obj_hash_values(n)).cuda()
    t = synctree_hip.DeviceTree()
    t.insert_int64_device(keys.data_ptr(), vals.data_ptr(), n, 17)
    for _ in range(6):
        t.rehash()
    t.sync()
    t.close()


def k1_pmc_traffic(args):
    """HBM bytes per K1 launch from rocprofv3 PMC, one counter group per pass
    (FETCH_SIZE, then WRITE_SIZE), corrected as MI355X_MICROARCH.md §HBM
    prescribes: FETCH_SIZE counts half the bytes of a wide coalesced 16-B/lane
    stream on gfx950 (x2); WRITE_SIZE is exact for 16-B stores.  Both are KiB.
    Infinity-Cache hits are counted too (the tile array may stay resident
    between back-to-back launches)."""
    prof = shutil.which('rocprofv3')
    if not prof:
        return {'error': 'rocprofv3 not found'}
    res = {}
    env = dict(os.environ, TMPDIR=tempfile.gettempdir())
    for ctr in ('FETCH_SIZE', 'WRITE_SIZE'):
        d = tempfile.mkdtemp(prefix='pmc_')
        cmd = ['timeout', '-s', 'KILL', '150', prof, '--pmc', ctr, '--kernel-include-regex', K1_KERNEL, '-f', 'csv',
               '-d', d, '-o', 'pmc', '--', sys.executable, os.path.abspath(__file__), '--pmc-probe', '--keys',
               str(args.keys)]
        t0 = time.perf_counter()
        r = subprocess.run(cmd, stdout=subprocess.DEVNULL, stderr=subprocess.PIPE, env=env)
        vals = []
        for root, _, files in os.walk(d):
            for f in files:
                if f.endswith('counter_collection.csv'):
                    import csv
                    for row in csv.DictReader(open(os.path.join(root, f))):
                        if row.get('Counter_Name') == ctr and K1_KERNEL in row.get('Kernel_Name', ''):
                            vals.append(float(row['Counter_Value']))
        shutil.rmtree(d, ignore_errors=True)
        if r.returncode != 0 or not vals:
            res[ctr] = {'error': 'rc=%d, %d samples: %s' % (r.returncode, len(vals), r.stderr.decode()[-300:])}
            continue
        # the first launch follows the tile build; report the steady state (launches 2..)
        steady = vals[1:] if len(vals) > 1 else vals
        res[ctr] = {'kib_per_launch_mean': round(sum(steady) / len(steady), 1), 'launches': len(vals),
                    'pass_s': round(time.perf_counter() - t0, 1)}
    try:
        fetch = res['FETCH_SIZE']['kib_per_launch_mean'] * 1024 * 2
        write = res['WRITE_SIZE']['kib_per_launch_mean'] * 1024
        res['traffic_bytes'] = int(fetch + write)
        res['read_bytes'] = int(fetch)
        res['write_bytes'] = int(write)
        res['formula'] = 'FETCH_SIZE[KiB] x 1024 x 2 (gfx950 half-count of 16-B/lane streams) + WRITE_SIZE[KiB] x 1024'
    except (KeyError, TypeError):
        pass
    return res


def trace_probe(args):
    """Child of group_kernel_trace (run under rocprofv3 --kernel-trace): the
    config-4 group (args.ensembles trees x args.ensemble_keys keys) rehashed
    as one st_rehash_group launch, 2 warm-up + 8 traced launches."""
    import torch
    from riak_ensemble_amd import synctree_hip, workload
    dev = torch.device('cuda', 0)
    E, nk = args.ensembles, args.ensemble_keys
    vals = _dev_values(torch.arange(nk, dtype=torch.int64, device=dev), dev, torch)
    trees = []
    for e in range(E):
        k = _dev_keys(workload.SEED ^ (e + 1), 0, nk, dev, torch)
        t = synctree_hip.DeviceTree(device=0)
        t.insert_int64_device(k.data_ptr(), vals.data_ptr(), nk, 17)
        trees.append(t)
    for _ in range(10):
        synctree_hip.rehash_group(trees)
    for t in trees:
        t.close()


def group_kernel_trace(args):
    """The config-4 group launch's duration as rocprofv3 --kernel-trace --stats
    reports it (a child process under the profiler, before this process
    touches the GPU): mean / min / max over the launches after the first two
    (tile builds and warm-up).  The bench's roofline for config 4 is priced on
    this mean, so a committed rocprof CSV reproduces it."""
    prof = shutil.which('rocprofv3')
    if not prof:
        return {'error': 'rocprofv3 not found'}
    env = dict(os.environ, TMPDIR=tempfile.gettempdir())
    d = tempfile.mkdtemp(prefix='trace_')
    cmd = ['timeout', '-s', 'KILL', '240', prof, '--kernel-trace', '--kernel-include-regex', 'k_rehash_fused|k_level16_group',
           '-f', 'csv', '-d', d, '-o', 'tr', '--', sys.executable, os.path.abspath(__file__), '--trace-probe', '--ensembles',
           str(args.ensembles), '--ensemble-keys', str(args.ensemble_keys)]
    t0 = time.perf_counter()
    r = subprocess.run(cmd, stdout=subprocess.DEVNULL, stderr=subprocess.PIPE, env=env)
    rows = []
    import csv
    for root, _, files in os.walk(d):
        for f in files:
            if f.endswith('kernel_trace.csv'):
                for row in csv.DictReader(open(os.path.join(root, f))):
                    nm = row.get('Kernel_Name', '')
                    if 'k_rehash_fused' in nm or 'k_level16_group' in nm:
                        rows.append((int(row['Start_Timestamp']), int(row['End_Timestamp']), 'k_rehash_fused' in nm))
    shutil.rmtree(d, ignore_errors=True)
    # one st_rehash_group = the fused launch (K1 + level H of every window)
    # and one k_level16_group launch per level above: its kernels' summed
    # durations, and its GPU span (first start to last end)
    rows.sort()
    calls = []
    for st, en, fused in rows:
        if fused or not calls:
            calls.append([st, en, 0.0, 0])
        c = calls[-1]
        c[1] = max(c[1], en)
        c[2] += (en - st) / 1e6
        c[3] += 1
    if r.returncode != 0 or len(calls) < 3:
        return {'error': 'rc=%d, %d calls: %s' % (r.returncode, len(calls), r.stderr.decode()[-300:])}
    ms = [c[2] for c in calls[2:]]
    span = [(c[1] - c[0]) / 1e6 for c in calls[2:]]
    return {'kernel_ms_mean': round(sum(ms) / len(ms), 4), 'kernel_ms_min': round(min(ms), 4),
            'kernel_ms_max': round(max(ms), 4), 'span_ms_mean': round(sum(span) / len(span), 4),
            'launches_per_call': calls[2][3], 'calls': len(ms), 'pass_s': round(time.perf_counter() - t0, 1),
            'what': 'rocprofv3 --kernel-trace of a child process: each group rehash over the same %d x %d-key ensembles '
                    '(the fused launch k_rehash_fused<GROUP> + one k_level16_group launch per level above level H), '
                    'its kernels\' summed durations; calls 3..10' % (args.ensembles, args.ensemble_keys)}


# ---------------------------------------------------------------- legs
def _bench_cold_l3(tree, torch, dev, k1_bytes, hot_ms, reps=5):
    """The rehash kernel with a cold Infinity Cache: a 1 GiB read (4x the
    256 MiB L3) before every rehash, so the tiles come from HBM (as they
    always do for trees whose tiles exceed the L3, e.g. config 5's 1.8 GB).
    Kernel time from HIP events on the library stream."""
    flush = torch.ones(1 << 30, dtype=torch.uint8, device=dev)
    torch.cuda.synchronize()
    tree.set_timing(True)
    tree.kernel_stats('*reset*')
    for i in range(reps):
        int(flush.sum())          # 1 GiB read: the L3 now holds clean lines of `flush`
        torch.cuda.synchronize()
        tree.rehash()
        tree.sync()
    n, ms = tree.kernel_stats('rehash_fused')
    tree.set_timing(False)
    del flush
    avg = ms / max(n, 1)
    gbs = k1_bytes / (avg / 1e3) / 1e9
    return {'kernel_avg_ms': round(avg, 4), 'achieved_GBps': round(gbs, 1), 'frac': round(gbs / HBM_PEAK_GBS, 4),
            'hot_kernel_avg_ms': round(hot_ms, 4), 'launches': n,
            'what': 'rehash kernel after a 1 GiB read per launch (Infinity Cache flushed): tiles read from HBM'}


def _bench_rehash_after_mutation(tree, n0, torch, reps=10, batch=1000):
    """rehash/1 right after an insert/3 batch: the rehash a
    tree pays when its content changed since the last one (the repair path,
    riak_ensemble_peer_tree.erl:264-277; any rehash after writes).  Each rep
    inserts `batch` new keys (host path, a streaming batch into the pages),
    then times rehash/1.  The first full rehash after a mutation hashes every
    segment straight from the tree's segments (no tile build, rehash_all);
    roofline over its kernels (HIP events): the same SURVEY §8(d) bytes as the
    headline, 17 B per value + 17 B per present node written."""
    rng = np.random.default_rng(11)
    ts, tins = [], []
    for r in range(reps + 1):
        ks = [int(x) for x in rng.integers(1 << 62, (1 << 63) - 1, batch)]
        vs = [bytes([0]) + (2).to_bytes(8, 'big') + (r * batch + i).to_bytes(8, 'big') for i in range(batch)]
        tree.sync()
        t0 = time.perf_counter()
        tree.insert_batch(ks, vs)
        tree.sync()
        t1 = time.perf_counter()
        if r == reps:   # the kernels of one more rep, on HIP events
            tree.set_timing(True)
            tree.kernel_stats('*reset*')
        tree.rehash()
        tree.sync()
        t2 = time.perf_counter()
        if r == reps:
            ks_ms = {}
            for nm in ('segment_hash', 'level_rehash', 'seg_perm', 'tile_build', 'rehash_fused', 'page_fold'):
                c, ms = tree.kernel_stats(nm)
                if c:
                    ks_ms[nm] = round(ms, 4)
            tree.set_timing(False)
        elif r > 0:   # rep 0 builds the pages
            tins.append(t1 - t0)
            ts.append(t2 - t1)
    ts.sort()
    tins.sort()
    n = tree.num_entries()
    nonempty = int((tree.level_entries(tree.height + 1)[0] > 0).sum())
    pres_inner = sum(int((tree.level_entries(l)[0] > 0).sum()) for l in range(1, tree.height + 1))
    alg = 17 * n + 17 * (nonempty + pres_inner)
    kern = ks_ms.get('segment_hash', 0.0) + ks_ms.get('level_rehash', 0.0)
    gbs = alg / (kern / 1e3) / 1e9 if kern else None
    return {'ms_per_rehash': round(ts[len(ts) // 2] * 1e3, 4), 'ms_per_insert_batch': round(tins[len(tins) // 2] * 1e3, 4),
            'batch_keys': batch, 'reps': reps, 'entries': n, 'kernels_ms': ks_ms,
            'roofline': {'bound': 'hbm', 'achieved': round(gbs, 1) if gbs else None, 'peak': HBM_PEAK_GBS,
                         'unit': 'GB/s', 'frac': round(gbs / HBM_PEAK_GBS, 4) if gbs else None, 'traffic': None,
                         'bytes_per_rehash': alg, 'kernel_ms': round(kern, 4),
                         'kernel': 'k_segment_hash_perm (every segment from the pages) + the level kernels'},
            'what': 'insert/3 of %d new keys, then rehash/1 (wall, median of %d; the first full rehash after a '
                    'mutation hashes from the segments, no tile build)' % (batch, reps)}


def _bench_repair(tree, keys_h, torch, reps=10):
    """riak_ensemble_peer_tree do_repair (peer_tree.erl:264-277) after a
    segment-level corruption: delete the segment node, then a full rehash/1.
    The rehash after a mutation rebuilds the hash-ready tiles first
    (k_tile_order_window + scan + k_tile_fill), so this is the rehash a repair
    pays, next to the headline's (tiles valid).  Reps delete different
    non-empty segments of the 10M-key tree (last leg on it)."""
    H1 = tree.height + 1
    segs = tree.segments_of([int(k) for k in keys_h[:reps * 7:7]])
    ts = []
    for s in segs[:reps]:
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        tree.delete_node(H1, s)
        tree.rehash()
        tree.sync()
        ts.append(time.perf_counter() - t0)
    ts.sort()
    tree.set_timing(True)
    tree.kernel_stats('*reset*')
    tree.delete_node(H1, segs[reps] if len(segs) > reps else segs[0])
    tree.rehash()
    tb_n, tb_ms = tree.kernel_stats('tile_build')
    rf_n, rf_ms = tree.kernel_stats('rehash_fused')
    tree.set_timing(False)
    mem = tree.mem_stats()
    return {'ms_per_repair': round(ts[len(ts) // 2] * 1e3, 4), 'reps': reps,
            'kernels_ms': {'tile_build': round(tb_ms, 4), 'rehash_fused': round(rf_ms, 4)},
            'tile_bytes': mem['tiles'], 'csr_bytes': mem['csr'], 'slot_bytes': mem['slots'],
            'what': 'repair path: delete one segment node + full rehash/1 (tile rebuild included), median of %d, '
                    'wall incl. the C-ABI calls; tile_bytes = the device copy of every value the tiled '
                    'layout keeps (the headline rehash reads it)' % reps}


def _present_inner(tree):
    """Present inner nodes (levels 1..H) of a device tree: the entries its
    parents hold for them (st_level_entries of levels 2..H+1 give the
    children's presence; a node is present iff one of its children is)."""
    n = 0
    for lvl in range(2, tree.height + 2):
        n += int(tree.level_entries(lvl)[0].reshape(-1, tree.width).any(1).sum())
    return n


def _segment_histogram(tree, keys_h):
    """Keys per segment via the device key->segment map (st_segment_of_batch)."""
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
            'what': 'st_insert_int64: key->segment MD5, counting sort by segment, run sort, merge, dirty rehash (all levels)'}


def _compare_roofline(tree_a, ms):
    """Algorithmic bytes of one compare: per visited inner node and
    side, its W child entries + the parent's entry (18 B each: md5 + tag),
    read to verify it and diff its children; per visited segment pair the
    offsets, key records, values and entries of both sides (counted on the
    device); plus the 32-B diff records written."""
    vis, seg_bytes = tree_a.compare_stats()
    H = tree_a.height
    inner = sum(vis[1:H + 1])
    W = tree_a.width
    inner_bytes = 2 * inner * (W + 1) * 18
    return vis, inner_bytes + seg_bytes


def _bench_compare(synctree_hip, tree_a, keys_d, vals_d, n, local, torch, reps=20):
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
    # kernel times from HIP events in a second pass (event records add host
    # time to every launch: not inside the wall-clock loop above)
    tree_a.set_timing(True)
    tree_a.kernel_stats('*reset*')
    for _ in range(reps):
        tree_a.compare_device(tb)
    kern = {k: round(tree_a.kernel_stats(k)[1] / reps, 4) for k in ('cmp_walk',)}
    tree_a.set_timing(False)
    vis, algo = _compare_roofline(tree_a, dt * 1e3)
    t0 = time.perf_counter()
    res = tree_a.compare(tb)
    dt_host = time.perf_counter() - t0
    # the records returned to host memory by the C ABI alone (st_compare ->
    # st_result, freed; no Python decoding), as a NIF would take them
    import ctypes
    from riak_ensemble_amd import _lib
    L = _lib.load()
    rp = ctypes.POINTER(_lib.StResult)()
    cl, cb, cs = ctypes.c_uint32(), ctypes.c_uint64(), ctypes.c_int()
    c_times = []
    for _ in range(reps):
        tc = time.perf_counter()
        _lib.check(L.st_compare(tree_a.h, tb.h, _lib.ST_FILTER_ALL, ctypes.byref(rp), ctypes.byref(cl), ctypes.byref(cb),
                                ctypes.byref(cs)), 'st_compare')
        c_times.append(time.perf_counter() - tc)
        assert rp.contents.n_entries == nd
        L.st_free_result(rp)
    c_times.sort()
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
    # a peer exchanges over and over: the local tree's compare state (its
    # first compare allocates it) is warmed by a plan-only exchange first
    assert ta.exchange_plan(tb2)[0] == 'ok'
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    res_apply = ta.exchange_apply(tb2)
    torch.cuda.synchronize()
    dt_apply = time.perf_counter() - t0
    assert res_apply[0] == 'ok' and res_apply[1]['applied'] == len(mut2), res_apply
    assert ta.top_hash() == tb2.top_hash(), 'exchange did not converge the trees'
    ta.close()
    tb2.close()
    gbs = algo / dt / 1e9
    return {'tree_compares_per_s': round(1.0 / dt, 1), 'ms_per_compare': round(dt * 1e3, 4),
            'diff_keys': nd, 'diff_keys_per_s': round(nd / dt, 1),
            'kernel_ms_per_compare': kern,
            'visited_per_level': vis[1:tree_a.height + 2],
            'roofline': {'bound': 'hbm', 'achieved': round(gbs, 2), 'peak': HBM_PEAK_GBS, 'unit': 'GB/s',
                         'frac': round(gbs / HBM_PEAK_GBS, 6), 'bytes_per_compare': int(algo),
                         'note': 'latency-bound: ~1 MB of algorithmic traffic per compare; the bound that binds is '
                                 'the dependent chain frontier -> verify/merge -> scan -> write'},
            'ms_per_compare_records_to_host_c': round(c_times[len(c_times) // 2] * 1e3, 4),
            'ms_per_compare_records_to_host_c_what': 'st_compare through ctypes: compare + the ordered diff records '
                                                     '(keys, both values, kinds, segments) in host memory; median of '
                                                     '%d calls' % reps,
            'ms_per_compare_incl_python_decode': round(dt_host * 1e3, 4),
            'exchange_apply_ms': round(dt_apply * 1e3, 4),
            'exchange_apply': 'st_exchange_apply: compare + valid_obj_hash select + one batched insert/3 of the %d '
                              'newer remote values (dirty-path rehash); trees converge (equal top hashes); one call, '
                              'the local tree\'s compare state warmed by an exchange_plan first' % len(mut2),
            'what': 'config3: 10M vs 10M keys, every 1000th non-empty segment differs; K3 in one launch (frontier, '
                    'verify + merge-join, each wave\'s records placed after the higher waves\' by their published '
                    'counts) with the ordered diff records left on the device; one host round trip per compare'}


def _bench_verify(tree, n, reps=20):
    """verify_upper/1 and verify/1 (synctree.erl:549-571) of the 10M-key tree.
    verify_upper is the exchange's own precheck (riak_ensemble_exchange.erl:
    58-65): every exchange runs it before its compare.  §8(d) bytes: the 17-B
    entries every verified node's message holds (a node's hash input is its
    children's entries; verify/1 adds every segment's values, 17 B per key)
    plus the 17-B parent entry each node is checked against.  Wall time per
    C-ABI call (the call returns the boolean: one host round trip), kernel
    times from HIP events in a second pass."""
    H = tree.height
    pres = [None] + [tree.level_entries(l)[0] for l in range(1, H + 2)]
    inner_nodes = sum(int(pres[l].sum()) for l in range(1, H + 1))     # present nodes of levels 1..H
    child_entries = sum(int(pres[l].sum()) for l in range(2, H + 2))   # their message entries
    out = {}
    for name, upper in (('verify_upper', True), ('verify', False)):
        assert tree.verify(upper=upper) is True
        ts = []
        for _ in range(reps):
            t0 = time.perf_counter()
            tree.verify(upper=upper)
            ts.append(time.perf_counter() - t0)
        ts.sort()
        tree.set_timing(True)
        tree.kernel_stats('*reset*')
        for _ in range(reps):
            tree.verify(upper=upper)
        kms = {}
        for k in ('verify_upper', 'mark_reachable', 'segment_verify', 'level_verify'):
            c, ms = tree.kernel_stats(k)
            if c:
                kms[k] = round(ms / c, 4)
        tree.set_timing(False)
        ms = ts[len(ts) // 2] * 1e3
        alg = 17 * (child_entries + inner_nodes) + (0 if upper else 17 * (n + int(pres[H + 1].sum())))
        gbs = alg / (ms / 1e3) / 1e9
        out[name] = {'ms': round(ms, 4), 'kernel_ms': kms,
                     'roofline': {'bound': 'hbm', 'achieved': round(gbs, 1), 'peak': HBM_PEAK_GBS, 'unit': 'GB/s',
                                  'frac': round(gbs / HBM_PEAK_GBS, 4), 'bytes_per_call': alg,
                                  'formula': '17 B x (child entries of the %d verified inner nodes + their parent '
                                             'entries)%s, over the wall ms of one call'
                                             % (inner_nodes, '' if upper else ' + 17 B x (keys + segments)')}}
    out['what'] = ('median of %d C-ABI calls on the config-2 tree (10M keys); verify_upper/1 = the exchange '
                   'precheck (riak_ensemble_exchange.erl:58-65)' % reps)
    return out


def _bench_leveldb(synctree_hip, tree, local, torch, reps=5):
    """synctree_leveldb format of the 10M-key tree:
    device encode of every node record, the host-inclusive snapshot (D2H of
    the records), and restore into a fresh tree from those host records."""
    import ctypes
    from riak_ensemble_amd import _lib
    L = _lib.load()
    tid = b'ens-1'
    tree.snapshot_leveldb_device(tid)   # warm-up
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        n, kb, vb = tree.snapshot_leveldb_device(tid)
    dt = (time.perf_counter() - t0) / reps
    tree.set_timing(True)   # kernel times in a second pass (events add host time per launch)
    kn = ('snap_entry_sizes', 'snap_sizes', 'snap_write', 'snap_entries')
    k0 = [tree.kernel_stats(k) for k in kn]
    for _ in range(reps):
        n, kb, vb = tree.snapshot_leveldb_device(tid)
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
            'entries_roofline': _entries_roof(tree, vb, kms[3]),
            'encode_GB_per_s_written': round((kb + vb) / dt / 1e9, 1),
            'snapshot_to_host_ms': round(host_s * 1e3, 1),
            'restore_from_host_ms': round(restore_s * 1e3, 1),
            'restore_same_top_hash': bool(same),
            'what': 'config2 tree (10M keys): every node as <<0,Id,Level,encode_unsigned(Bucket)>> => '
                    'term_to_binary(Node) (synctree_leveldb.erl:104-152); restore = new/5 + reload_top_hash'}


def _entries_roof(tree, vb, ms):
    """k_snap_entries per entry: koff 8 + key record 9 + voff 8 + value 17 +
    entry offset 8 read, the entry's ETF bytes written."""
    ne = tree.num_entries()
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


def _dev_keys(seed, start, n, dev, torch):
    """splitmix64(seed + i), i = start+1 .. start+n, masked to 63 bits, on the
    device (a bijection before the mask: distinct keys with overwhelming
    probability; inserts are last-writer-wins anyway)."""
    return _dev_keys_at(seed, torch.arange(start, start + n, dtype=torch.int64, device=dev), dev, torch)


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


def _dev_values(seq, dev, torch, epoch=1):
    """<<0, Epoch:64, Seq:64>> rows for an int64 seq tensor (device)."""
    v = torch.zeros((seq.numel(), 17), dtype=torch.uint8, device=dev)
    v[:, 8] = epoch
    for b in range(8):
        v[:, 9 + b] = ((seq >> (56 - 8 * b)) & 0xFF).to(torch.uint8)
    return v


def _bench_ensembles(synctree_hip, dist, coll_dev, args, local, torch, trace=None, reps=5):
    """Config 4 on every rank: E ensembles x nk keys per GPU (ensemble e of rank
    r seeded SEED ^ (r * E + e + 1)), rehashed as ONE st_rehash_group batch,
    then every ensemble's top hash all-gathered across the ranks (RCCL
    all_gather_into_tensor of the 18-B records st_tops_to_device writes).
    Timed: batch rehash + tops + all-gather, max over ranks."""
    from riak_ensemble_amd import workload
    rank = dist.get_rank() if dist else 0
    world = dist.get_world_size() if dist else 1
    E, nk = args.ensembles, args.ensemble_keys
    dev = torch.device('cuda', local)
    trees = []
    t0 = time.perf_counter()
    vals = _dev_values(torch.arange(nk, dtype=torch.int64, device=dev), dev, torch)
    for e in range(E):
        k = _dev_keys(workload.SEED ^ (rank * E + e + 1), 0, nk, dev, torch)
        t = synctree_hip.DeviceTree(device=local)
        t.insert_int64_device(k.data_ptr(), vals.data_ptr(), nk, 17)
        trees.append(t)
        del k
    torch.cuda.synchronize()
    load_s = time.perf_counter() - t0
    mine = torch.empty(E * 18, dtype=torch.uint8, device=dev)
    allt = torch.empty(world * E * 18, dtype=torch.uint8, device=coll_dev)

    def step():
        synctree_hip.rehash_group(trees)
        synctree_hip.tops_to_device(trees, mine.data_ptr())
        if dist:
            dist.all_gather_into_tensor(allt, mine.to(coll_dev))
        else:
            allt.copy_(mine)

    for _ in range(3):   # warm-up (the first builds every tree's tiles)
        step()
    before = allt.cpu().numpy().copy()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(reps):
        step()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    el = time.perf_counter() - t0
    if dist:
        tt = torch.tensor([el], dtype=torch.float64, device=coll_dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        el = float(tt.item())
    stable = bool((allt.cpu().numpy() == before).all()) and int(before.reshape(-1, 18)[:, 0].sum()) == world * E
    # the group launch alone (HIP events on trees[0]'s stream) and its roofline:
    # per tree the same algorithmic bytes as the headline's launch
    # the group launch's GPU time: the span of reps group rehashes on trees[0]'s
    # stream (the launch's stream), no per-launch events; per-launch HIP
    # events beside it
    g_avg = _span_ms(trees[0], torch, dev, lambda: synctree_hip.rehash_group(trees), reps)
    trees[0].set_timing(True)
    trees[0].kernel_stats('*reset*')
    for _ in range(reps):
        synctree_hip.rehash_group(trees)
    g_n, g_ms = trees[0].kernel_stats('rehash_group')
    trees[0].set_timing(False)
    g_evt = g_ms / max(reps, 1)   # a group rehash: the fused launch + a level launch per level above level H
    S = trees[0].segments
    H = trees[0].height
    # SURVEY §8(d) bytes per tree: 17 B per key (values) + a 17-B entry per
    # present node (non-empty segments + present inner nodes), counted on a
    # sample of the trees (Poisson occupancy: every tree has the same
    # expectation; the sample's spread is a few hundred nodes)
    samp = trees[:4]
    nonempty = [int(t.level_entries(H + 1)[0].sum()) for t in samp]
    pinner = [_present_inner(t) for t in samp]
    tree_bytes = int(17 * nk + 17 * (sum(nonempty) + sum(pinner)) / len(samp))
    inner = sum(16 ** lv for lv in range(H))
    meta_bytes = 17 * nk + S * 8 + (S // 64) * 16 + S // 8 + S * 18 + inner * 18
    # the roofline's launch time: rocprof's mean of the group launch (a child
    # process traced on this box) when available, else the span below
    k_ms = trace['kernel_ms_mean'] if trace and 'kernel_ms_mean' in trace else g_avg
    k_src = ('rocprofv3 --kernel-trace mean of a group rehash\'s kernels (ensembles.kernel_trace)' if k_ms is not g_avg else
             'GPU span of %d back-to-back group rehashes on trees[0]\'s stream / %d (host preparation between them '
             'included: an upper bound of the launch)' % (reps, reps))
    g_gbs = E * tree_bytes / (k_ms / 1e3) / 1e9 if k_ms > 0 else 0.0
    mem0 = trees[0].mem_stats()
    perkey = _bench_perkey_multi(trees, synctree_hip, torch)
    # per-tree rehash for comparison (rank-local, untimed for the headline)
    t0 = time.perf_counter()
    for t in trees[:32]:
        t.rehash()
    for t in trees[:32]:
        t.sync()
    per_tree = (time.perf_counter() - t0) / min(32, E)
    for t in trees:
        t.close()
    return {'keys_per_s': round(world * E * nk * reps / el, 1), 'ms_per_batch': round(el * 1e3 / reps, 3),
            'ensembles_per_gpu': E, 'ensembles_total': world * E, 'keys_per_ensemble': nk, 'ranks': world,
            'tops_allgather_stable': stable, 'load_s': round(load_s, 2),
            'kernel_ms_per_batch': round(g_avg, 4), 'kernel_ms_per_batch_events': round(g_evt, 4),
            'roofline': {'bound': 'hbm', 'achieved': round(g_gbs, 1), 'peak': HBM_PEAK_GBS, 'unit': 'GB/s',
                         'frac': round(g_gbs / HBM_PEAK_GBS, 4), 'bytes_per_launch': E * tree_bytes,
                         'kernel_ms': round(k_ms, 4), 'kernel_time_source': k_src,
                         'bytes_per_tree': tree_bytes, 'bytes_per_tree_incl_metadata': meta_bytes,
                         'tile_bytes_per_tree': mem0['tiles'],
                         'sample_nonempty_segments': nonempty, 'sample_present_inner': pinner,
                         'kernel': K1_KERNEL + '<GROUP, 8 waves per window, 6 waves per SIMD> (K1 + level H) + k_level16_group '
                                   '(one launch per level above)',
                         'note': 'SURVEY §8(d): per tree 17 B of value per key + a 17-B entry per present node '
                                 '(non-empty segments + present inner nodes, mean of %d sampled trees)' % len(samp)},
            'kernel_trace': trace,
            'per_tree_rehash_keys_per_s_rank0': round(nk / per_tree, 1),
            'per_key_multi': perkey,
            'what': 'config4: %d ensembles x %d keys on each of %d GPU(s) (%d total); per step: st_rehash_group of '
                    'the rank\'s trees + st_tops_to_device + all_gather_into_tensor of every ensemble\'s top hash '
                    '(keys generated on device: splitmix64 masked to 63 bits)' % (E, nk, world, world * E)}


def _bench_perkey_multi(trees, synctree_hip, torch, rounds=40):
    """The per-key path of many ensembles at once (SURVEY §8f rank 4 in the
    config-4 shape): one insert/3 into EVERY tree per st_insert1_multi call
    (one device launch, a workgroup per tree), R rounds of new keys; then
    get/2 of the same keys per st_get1_multi call (values checked).  Beside
    it, st_insert1 on one tree (one launch per key).  Host arrays prepared
    before the timed loop (ctypes call, no Python packing inside it)."""
    import ctypes
    from riak_ensemble_amd import _lib
    L = _lib.load()
    E = len(trees)
    arr = (ctypes.c_void_p * E)(*[t.h.value for t in trees])
    rng = np.random.default_rng(404)
    kt = np.zeros(E, np.uint8)                                   # ST_KEY_INT
    ko = (np.arange(E + 1, dtype=np.uint64) * 8)
    vo = (np.arange(E + 1, dtype=np.uint64) * 17)
    rounds_k = [rng.integers(0, 1 << 62, E, dtype=np.int64) for _ in range(rounds)]
    rounds_v = []
    for r in range(rounds):
        v = np.zeros((E, 17), np.uint8)
        v[:, 8] = 9
        v[:, 9:17] = np.array(np.arange(E) + r * E, '>u8').view(np.uint8).reshape(-1, 8)
        rounds_v.append(v)
    kh = [np.ascontiguousarray(k.astype('>i8')).view(np.uint8) for k in rounds_k]
    st = np.zeros(E, np.int32)
    p = lambda a: ctypes.c_void_p(a.ctypes.data)   # noqa: E731

    def ins(r):
        _lib.check(L.st_insert1_multi(arr, E, p(kt), p(kh[r]), p(ko), p(rounds_v[r]), p(vo), p(st), None, None),
                   'st_insert1_multi')
        assert not st.any()
    ins(0)                                                      # warm-up (per-tree request slots)
    torch.cuda.synchronize()
    lat = []
    t0 = time.perf_counter()
    for r in range(1, rounds):
        tb = time.perf_counter()
        ins(r)
        lat.append(time.perf_counter() - tb)
    el = time.perf_counter() - t0
    lat.sort()
    # gets of the last round's keys, values checked
    vout = np.zeros(E * 17 + 64, np.uint8)
    vof = np.zeros(E + 1, np.uint64)
    tg = time.perf_counter()
    _lib.check(L.st_get1_multi(arr, E, p(kt), p(kh[rounds - 1]), p(ko), p(vout), len(vout), p(vof), p(st), None, None),
               'st_get1_multi')
    get_s = time.perf_counter() - tg
    assert not st.any() and (vout[:E * 17].reshape(E, 17) == rounds_v[rounds - 1]).all(), 'multi get values differ'
    # one tree, one launch per key
    t1 = trees[0]
    one = []
    for r in range(50):
        tb = time.perf_counter()
        assert t1.insert1(int(rng.integers(0, 1 << 62)), bytes(rounds_v[0][r % E])) is None
        one.append(time.perf_counter() - tb)
    one.sort()
    # the crossover with a host-side path: one insert/3 into each of N trees
    # per call, N = 1 .. E (ctypes included, median of 15 calls), beside the
    # C port's insert on the host (config1.per_key_latency_us.cpu_insert_in_c)
    curve = {}
    for N in [x for x in (1, 2, 4, 8, 16, 32, 64, 128, 256) if x < E] + [E]:
        sub = (ctypes.c_void_p * N)(*[t.h.value for t in trees[:N]])
        ko_n = np.ascontiguousarray(ko[:N + 1])
        vo_n = np.ascontiguousarray(vo[:N + 1])
        lat_n = []
        for r in range(15):
            kk = np.ascontiguousarray(rng.integers(0, 1 << 62, N, dtype=np.int64).astype('>i8')).view(np.uint8)
            vv = np.ascontiguousarray(rounds_v[r % rounds][:N])
            tb = time.perf_counter()
            _lib.check(L.st_insert1_multi(sub, N, p(kt), p(kk), p(ko_n), p(vv), p(vo_n), p(st), None, None),
                       'st_insert1_multi')
            lat_n.append(time.perf_counter() - tb)
            assert not st[:N].any()
        lat_n.sort()
        curve[N] = round(lat_n[len(lat_n) // 2] * 1e6, 1)
    return {'inserts_per_s': round(E * (rounds - 1) / el, 1), 'trees_per_launch': E,
            'us_per_call_by_trees': curve,
            'us_per_call_by_trees_what': 'st_insert1_multi with one insert/3 into each of N trees per call (one '
                                         'launch), median of 15 calls, ctypes included',
            'ms_per_launch_median': round(lat[len(lat) // 2] * 1e3, 4), 'ms_per_launch_max': round(lat[-1] * 1e3, 4),
            'get_ms_per_launch': round(get_s * 1e3, 4),
            'single_tree_insert1_us_median': round(one[len(one) // 2] * 1e6, 1),
            'what': 'st_insert1_multi: one insert/3 into each of the %d trees per call (one k_small_multi launch, '
                    'a workgroup per tree), %d calls; latency = one call (every tree answered); st_get1_multi of '
                    'the last round checked; single_tree = st_insert1 on one tree (ctypes included)' % (E, rounds - 1)}


def _bench_partition(synctree_hip, dist, coll_dev, args, local, torch):
    """Config 5: one tree of part_keys keys partitioned by segment range over
    the ranks (st_set_partition); timed: part_batches write batches of
    part_batch_keys keys (50 % overwrites with Seq + 1, 50 % new keys), each an
    insert/3 batch with dirty-path rehash on every rank + the all-gather of the
    level-2 entries and level 1 + top (parallel.PartitionedTree.combine)."""
    from riak_ensemble_amd import parallel
    dev = torch.device('cuda', local)
    world = dist.get_world_size() if dist else 1
    grp = dist if dist else _SoloGroup()
    pt = parallel.PartitionedTree(synctree_hip.DeviceTree(device=local), grp, device=coll_dev)
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
    for j in range(2 * K + 2):
        old = torch.from_numpy(rng.integers(0, N, B // 2)).to(dev)          # overwrites: Seq + 1 of a loaded key
        k = torch.cat([_dev_keys_at(seed, old, dev, torch), _dev_keys(seed, N + j * B, B - B // 2, dev, torch)])
        seq = torch.cat([old + 1, torch.arange(N + j * B, N + j * B + (B - B // 2), device=dev)])
        batches.append((k.contiguous(), _dev_values(seq, dev, torch).contiguous()))
    torch.cuda.synchronize()
    # two warm-up batches (the first of a run merges into the CSR, the second
    # builds the pages), then K timed: each batch timed on its own (a device
    # synchronisation around it) so the batches that rebuild the pages show;
    # the reported rate is the amortised one (all K)
    for k, v in batches[:2]:
        pt.tree.insert_int64_device(k.data_ptr(), v.data_ptr(), B, 17)
        pt.combine()
    torch.cuda.synchronize()
    ps0 = pt.tree.page_stats()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    per = []
    t0 = time.perf_counter()
    for j in range(2, K + 2):
        k, v = batches[j]
        tb = time.perf_counter()
        pt.tree.insert_int64_device(k.data_ptr(), v.data_ptr(), B, 17)
        pt.combine()
        torch.cuda.synchronize()
        per.append(time.perf_counter() - tb)
    if dist:
        dist.barrier()
    el = time.perf_counter() - t0
    ps1 = pt.tree.page_stats()
    # the same workload with the pages off: K more batches,
    # each merged into the canonical CSR (the whole CSR rewritten)
    from riak_ensemble_amd import _lib
    pt.tree.debug_knob(_lib.ST_DBG_PAGES, -1)
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    dper = []
    t1 = time.perf_counter()
    for j in range(K + 2, 2 * K + 2):
        k, v = batches[j]
        tb = time.perf_counter()
        pt.tree.insert_int64_device(k.data_ptr(), v.data_ptr(), B, 17)
        pt.combine()
        torch.cuda.synchronize()
        dper.append(time.perf_counter() - tb)
    el_delta = time.perf_counter() - t1
    pt.tree.debug_knob(_lib.ST_DBG_PAGES, 0)
    dper.sort()
    top = pt.top_hash()
    same = True
    if dist:
        t = torch.tensor([el], dtype=torch.float64, device=coll_dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
        tops = parallel.gather_tops(dist, [top], device=coll_dev)
        same = all(x == top for x in tops)
    per.sort()
    entries = pt.tree.num_entries()
    pt.tree.close()
    # roofline on the touched segments (the batch's floor): their values are
    # read by the path verification, read by the dirty-path hash and written
    # once by the merge -- 3 x their bytes (st_page_stats out[5], before each
    # merge), over the wall time per batch (everything in it)
    tv = (ps1[5] - ps0[5]) / max(K, 1)
    alg = 3 * tv
    gbs = alg / (el / K) / 1e9
    roof = {'bound': 'hbm', 'achieved': round(gbs, 1), 'peak': HBM_PEAK_GBS, 'unit': 'GB/s',
            'frac': round(gbs / HBM_PEAK_GBS, 4), 'traffic': None, 'bytes_per_batch': int(alg),
            'touched_value_bytes_per_batch': int(tv),
            'formula': '3 x the value bytes of the segments a batch touches (verify read + hash read + merge '
                       'write), per batch, over the wall ms_per_batch (all kernels and host work of the batch)'}
    return {'batch_keys_per_s': round(K * B / el, 1), 'ms_per_batch': round(el * 1e3 / K, 4), 'batches': K,
            'roofline': roof,
            'ms_per_batch_median': round(per[len(per) // 2] * 1e3, 4), 'ms_per_batch_max': round(per[-1] * 1e3, 4),
            'pages': {'batches': ps1[1] - ps0[1], 'page_builds': ps1[2] - ps0[2],
                      'moved_entry_slots': ps1[4] - ps0[4],
                      'what': 'st_page_stats over the timed batches: batches through the pages, page rebuilds '
                              '(append region full), entry slots of segments moved to new pages'},
            'csr_merge_mode': {'ms_per_batch': round(el_delta * 1e3 / K, 4), 'ms_per_batch_median': round(dper[len(dper) // 2] * 1e3, 4),
                               'ms_per_batch_max': round(dper[-1] * 1e3, 4),
                               'what': 'the next %d batches with the pages off (st_debug_knob ST_DBG_PAGES = -1; the first '
                                       'folds the pages): each merged into the canonical CSR, rewriting every entry; '
                                       'rank-local, not max over ranks' % K},
            'batch_keys': B, 'tree_keys': N, 'ranks': world, 'entries_on_rank0': entries,
            'tops_agree_across_ranks': same, 'load_s': round(load_s, 3),
            'what': 'config5: %d-key tree partitioned by segment range over %d rank(s); per batch: insert/3 of %d keys '
                    '(50%% overwrites Seq+1, 50%% new; verify + dirty-path rehash) on every rank, all-gather of the '
                    'level-2 entries, level 1 + top (keys generated on device: splitmix64 masked to 63 bits); each batch '
                    'rewrites the tails of the segments it touches in the paged layout (DESIGN.md 3.3); '
                    'ms_per_batch is the mean over the timed batches' % (N, world, B)}


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
    reference-faithful mode (n verified inserts in one C loop, then the DFS
    rehash over all 2^20 slots), one thread -- the reference Erlang cannot run
    here.  Plus the per-key get/insert latency."""
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
    # per-key verified-path calls (get/2, insert/3, synctree.erl:189-227) one at
    # a time through the C-ABI (ctypes), i.e. the low-batch latency path
    kl = [int(k) for k in keys[:200]]
    t.get1(kl[0])                                       # untimed warm-up
    t.insert1(kl[0], bytes(vals[0]))
    t0 = time.perf_counter()
    got = [t.get1(k) for k in kl]
    gpu_get_us = (time.perf_counter() - t0) / len(kl) * 1e6
    assert got == [bytes(vals[i]) for i in range(len(kl))], 'per-key get returned wrong values'
    newv = bytes(17)
    t0 = time.perf_counter()
    st = [t.insert1(k, newv) for k in kl]
    gpu_ins_us = (time.perf_counter() - t0) / len(kl) * 1e6
    assert all(s is None for s in st), 'per-key insert rejected'
    assert [t.get1(k) for k in kl[:20]] == [newv] * 20, 'per-key insert did not store'
    # the device part of those calls: the k_small kernel alone (HIP events)
    kern_us = {}
    for name, fn in (('get', lambda k: t.get1(k)), ('insert', lambda k: t.insert1(k, newv))):
        t.set_timing(True)
        t.kernel_stats('*reset*')
        for k in kl[:50]:
            fn(k)
        launches, ms = t.kernel_stats('small')
        t.set_timing(False)
        kern_us[name] = round(ms / max(launches, 1) * 1e3, 1)
    t.close()
    out = {'gpu_keys_per_s': round(n / best, 1), 'gpu_ms': round(best * 1e3, 3),
           'what': 'config1: 100k keys, build + rehash + top_hash (GPU: host arrays in, one insert batch)',
           'per_key_latency_us': {'gpu_get': round(gpu_get_us, 1), 'gpu_insert': round(gpu_ins_us, 1),
                                  'kernel_us': kern_us,
                                  'what': 'one get/2 or insert/3 per C-ABI call (st_get1 / st_insert1: verified '
                                          'path + dirty-path rehash on the device), 200 calls after a warm-up, '
                                          'ctypes overhead included; results checked; kernel_us: the k_small '
                                          'kernel alone'}}
    if cpu:
        sys.path.insert(0, os.path.join(ROOT, 'oracle'))
        import oracle_c
        ot = oracle_c.OTree()
        t0 = time.perf_counter()
        assert ot.insert_int64_seq(keys, vals) == 0
        ot.rehash()
        ctop = ot.top_hash()
        dt = time.perf_counter() - t0
        assert ctop == top, 'config1: CPU restatement and GPU disagree'
        ka = np.array(kl, np.int64)
        t0 = time.perf_counter()
        ot.insert_int64_seq(ka, np.zeros((len(kl), 17), np.uint8))
        cpu_ins = (time.perf_counter() - t0) / len(kl) * 1e6
        t0 = time.perf_counter()
        for k in kl:
            ot.get(k)
        cpu_get = (time.perf_counter() - t0) / len(kl) * 1e6
        out['per_key_latency_us']['cpu_insert_in_c'] = round(cpu_ins, 2)
        out['per_key_latency_us']['cpu_get_via_ctypes'] = round(cpu_get, 2)
        out['cpu'] = {'keys_per_s': round(n / dt, 1), 'seconds': round(dt, 3), 'cores': 1, 'kind': 'port',
                      'sample': 'oracle/synctree_oracle.c: 100k verified insert/3 calls in one C loop + rehash + '
                                'top_hash'}
    return out


def _host_cores():
    """Host cores this process may use: the CPU quota of its cgroup (cpu.max),
    else OMP_NUM_THREADS, else the affinity mask.  (On the GPU box the
    affinity mask shows the whole machine while the job's share is 16.)"""
    cands = []
    try:
        with open('/sys/fs/cgroup/cpu.max') as f:
            q, per = f.read().split()[:2]
        if q != 'max':
            cands.append(max(1, int(int(q) // int(per))))
    except (OSError, ValueError):
        pass
    if os.environ.get('OMP_NUM_THREADS', '').isdigit():
        cands.append(int(os.environ['OMP_NUM_THREADS']))
    aff = len(os.sched_getaffinity(0)) if hasattr(os, 'sched_getaffinity') else (os.cpu_count() or 1)
    cands.append(aff)
    return max(1, min(cands))


def _cpu_baseline(keys_h, vals_h, top0, reps=3):
    """The C port (oracle/synctree_oracle.c) rehashing the same 10M-key tree:
    (a) the reference-faithful DFS rehash (synctree.erl:497-543) on one host
    thread, and (b) the throughput-mode rehash (ot_rehash_par: level by level,
    every node of a level spread over OpenMP threads) on every host core.
    About 10-20 s of CPU work in total."""
    sys.path.insert(0, os.path.join(ROOT, 'oracle'))
    import oracle_c
    ncpu = _host_cores()
    t0 = time.perf_counter()
    ot = oracle_c.OTree().bulk_load_int64(keys_h, vals_h)
    load_s = time.perf_counter() - t0
    assert ot.top_hash() == top0, 'CPU port disagrees with the device top hash'
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        ot.rehash()
        ts.append(time.perf_counter() - t0)
    best1 = min(ts)
    ot.rehash_par(ncpu)   # warm-up (first-touch of the per-level arrays)
    tp = []
    for _ in range(reps):
        t0 = time.perf_counter()
        ot.rehash_par(ncpu)
        tp.append(time.perf_counter() - t0)
    bestp = min(tp)
    assert ot.top_hash() == top0
    n = len(keys_h)
    return {'value': round(n / best1, 1), 'unit': 'keys/s', 'cores': 1, 'kind': 'port',
            'sample': 'full synctree:rehash/1 restatement (oracle/synctree_oracle.c, DFS over all 2^20 segment '
                      'slots) of the same 10M-key tree, best of %d; tree load %.1f s untimed' % (reps, load_s),
            'seconds_per_rehash': round(best1, 3),
            'all_cores': {'value': round(n / bestp, 1), 'unit': 'keys/s', 'cores': ncpu, 'kind': 'port',
                          'seconds_per_rehash': round(bestp, 3),
                          'sample': 'ot_rehash_par: the same rehash level by level over flat entry arrays, every '
                                    'level\'s nodes spread over %d OpenMP threads (the host cores this job may use: '
                                    'cgroup quota / OMP_NUM_THREADS / affinity, the smallest), best of %d' % (ncpu, reps)}}


if __name__ == '__main__':
    main()
