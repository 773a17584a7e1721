"""Stress the per-key path (k_small) with the test_small_path pattern and
check every call against the C restatement; on the first divergence print
what the device returns now (transient vs persistent) and stop (diagnostic)."""
import os, sys, time
import numpy as np
R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, R)
sys.path.insert(0, os.path.join(R, 'oracle'))
import oracle_c as C
from riak_ensemble_amd import synctree_hip, workload


def _val(seq):
    return bytes([0]) + (1).to_bytes(8, 'big') + seq.to_bytes(8, 'big')


def trial(tn, W, S, steps=120):
    n = 20000 if S >= 4096 else 3000
    keys = workload.keys_int63(n, workload.SEED ^ (0x51 + tn))
    vals = workload.obj_hash_values(n)
    dev = synctree_hip.DeviceTree(W, S)
    ora = C.OTree(W, S)
    assert dev.insert_int64(keys, vals) == 0
    ora.bulk_load_int64(keys, vals)
    if dev.top_hash() != ora.top_hash():
        print('FAIL initial top, trial', tn, 'geom', (W, S), 'verify', dev.verify(), 'entries', dev.num_entries(), flush=True)
        got = dev.get_batch([int(k) for k in keys])
        bad = [i for i, g in enumerate(got) if g != ora.get(int(keys[i]))]
        segs = sorted(ora.segment_of(int(keys[i])) for i in bad)
        print('  bad keys', len(bad), 'segments', segs[:3], segs[-3:] if segs else None, 'kinds', [got[i] if not isinstance(got[i], bytes) else 'val' for i in bad[:4]], flush=True)
        return False
    rng = np.random.default_rng(tn)
    extra = workload.keys_int63(4000, workload.SEED ^ (0x52 + tn))
    seq = n
    junk = []
    touched = set()
    hist = {}
    model = {int(k): None for k in keys}
    for step in range(steps):
        m = int(rng.integers(1, 17))
        ks, vs = [], []
        for _ in range(m):
            k = int(keys[rng.integers(0, n)]) if rng.random() < 0.5 else int(extra[rng.integers(0, len(extra))])
            seq += 1
            ks.append(k)
            vs.append(_val(seq))
        touched.update(ora.segment_of(k) for k in ks)
        for k in ks:
            hist.setdefault(ora.segment_of(k), []).append((step, len(ks)))
        st = dev.insert_batch(ks, vs)
        for k, v in zip(ks, vs):
            ora.insert(k, v)
            model[k] = v
            INS.setdefault(k, []).append((step, v[-2:]))
        if CHECKALL and step >= CHECKALL:
            if not lost_report(dev, ora, model, 'after insert step %d' % step):
                return False
        if not all(x is None for x in st):
            print('FAIL insert trial', tn, 'geom', (W, S), 'step', step, 'n', len(ks), 'st', st, flush=True)
            print('  re-get of those keys:', dev.get_batch(ks) == [ora.get(k) for k in ks], flush=True)
            return False
        probe = [ks[0], int(keys[rng.integers(0, n)]), int(extra[rng.integers(0, len(extra))])]
        got = dev.get_batch(probe)
        exp = [ora.get(k) for k in probe]
        if got != exp:
            bad = [i for i in range(3) if got[i] != exp[i]]
            print('FAIL get trial', tn, 'geom', (W, S), 'step', step, 'idx', bad, 'got', [got[i] for i in bad],
                  'exp', [exp[i] for i in bad], flush=True)
            again = dev.get_batch(probe)
            print('  same get again:', again == exp, [again[i] for i in bad], flush=True)
            print('  get1 each:', [dev.get1(k) == ora.get(k) for k in probe], flush=True)
            print('  top equal:', dev.top_hash() == ora.top_hash(), flush=True)
            return False
        if JUNK and step % 10 == 9:      # other trees come and go (pool memory reuse)
            junk.append(synctree_hip.DeviceTree(16, 1 << 12))
            if len(junk) > 3:
                junk.pop(0).close()
        if step % 30 == 29:
            if step % 60 == 29:
                dev.rehash()
                touched = set()
                hist = {}
            else:
                vok = dev.verify()
                if not vok:
                    print('FAIL verify trial', tn, 'geom', (W, S), 'step', step, 'top equal', dev.top_hash() == ora.top_hash(),
                          'verify again', dev.verify(), flush=True)
                    segs = sorted(touched)
                    got = dev.exchange_get_batch(ora.height + 1, segs)
                    exp = [ora.node(ora.height + 1, x) for x in segs]
                    badsegs = [(x, g, e) for x, g, e in zip(segs, got, exp) if g != e]
                    print('  touched segments', len(segs), 'differing', len(badsegs), flush=True)
                    for x, g, e in badsegs[:4]:
                        print('   seg', x, 'touches', hist.get(x), '\n    dev', g, '\n    ora', e, flush=True)
                        for kk, vv in e:
                            print('     key', kk, 'dev get1 ok', dev.get1(kk) == vv, flush=True)
                    print('  entries dev', dev.num_entries(), 'ora', ora.num_entries(), flush=True)
                    lost_report(dev, ora, model, 'at verify failure')
                    multi = sum(1 for x in segs if len(hist.get(x, [])) > 1)
                    print('  touched more than once:', multi, 'of', len(segs), '; bad ones:',
                          [len(hist.get(x, [])) for x, _, _ in badsegs], flush=True)
                    for lvl in range(1, ora.height + 2):
                        pa, ha = dev.level_entries(lvl)
                        pb, hb = ora.level_entries(lvl)
                        d = np.nonzero((pa != pb) | np.any(ha != hb, axis=1))[0]
                        print('  level', lvl, 'differing buckets', len(d), d[:8], flush=True)
                    return False
            if dev.top_hash() != ora.top_hash():
                print('FAIL top after bulk op, trial', tn, 'step', step, 'verify', dev.verify(), 'entries dev',
                      dev.num_entries(), 'ora', ora.num_entries(), flush=True)
                lost_report(dev, ora, model, 'after bulk op')
                return False
    for j in junk:
        j.close()
    dev.close()
    return True


def lost_report(dev, ora, model, what):
    ks = list(model)
    got = dev.get_batch(ks)
    bad = [k for k, g in zip(ks, got) if g != ora.get(k)]
    if not bad:
        return True
    segs = sorted(ora.segment_of(k) for k in bad)
    print('  LOST', what, len(bad), 'of', len(ks), 'keys; segments', segs[0], '..', segs[-1], flush=True)
    h = {}
    for x in segs:
        h[x >> 14] = h.get(x >> 14, 0) + 1
    print('  per 16K-segment bin:', sorted(h.items()), flush=True)
    print('  first/last lost segs', segs[:6], segs[-6:], flush=True)
    shown = 0
    for k, g in zip(ks, got):
        if g != ora.get(k) and shown < 6:
            shown += 1
            print('   key', k, 'dev', g, 'ora', ora.get(k), 'hist', INS.get(k), flush=True)
    print('  sample kinds', [type(g).__name__ if not isinstance(g, tuple) else g[:2] for g in got if g is None or isinstance(g, tuple)][:6], flush=True)
    return False


INS = {}
CHECKALL = int(os.environ.get('STRESS_CHECKALL', '0'))
JUNK = int(os.environ.get('STRESS_JUNK', '1'))
t0 = time.time()
geoms = [(16, 1 << 20), (4, 4096), (16, 16)]
ok = True
for tn in range(int(sys.argv[1]) if len(sys.argv) > 1 else 30):
    for g in geoms:
        if not trial(tn, *g):
            ok = False
            break
    if not ok:
        break
    print('trial', tn, 'ok', round(time.time() - t0, 1), flush=True)
print('RESULT', 'ok' if ok else 'FAIL', flush=True)
