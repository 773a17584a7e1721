"""Per-window K1 timing of the fused rehash vs the window's modelled work and
its XCD (run with ST_LEVEL_STAMPS=1; diagnostic)."""
import os
import sys
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
dump = os.path.abspath('gpurun_out/stamp_dump.txt')
os.environ['ST_STAMP_DUMP'] = dump
if os.path.exists(dump):
    os.remove(dump)
import torch
from riak_ensemble_amd import synctree_hip, workload
n = 10_000_000
kh = workload.keys_int63(n)
k = torch.from_numpy(kh).cuda()
v = torch.from_numpy(workload.obj_hash_values(n)).cuda()
t = synctree_hip.DeviceTree()
t.insert_int64_device(k.data_ptr(), v.data_ptr(), n, 17)
for i in range(6):
    t.rehash()
    t.sync()
segs = np.concatenate([np.array(t.segments_of(kh[i:i + (1 << 21)].tolist()), np.int64) for i in range(0, n, 1 << 21)])
cnt = np.bincount(segs, minlength=1 << 20)
nb = np.where(cnt > 0, (17 * cnt + 8) // 64 + 1, 0)
W = -np.sort(-nb.reshape(256, 4096), axis=1)
tiles = W.reshape(256, 64, 64).max(axis=2)
wave = tiles.reshape(256, 4, 16).sum(axis=1)
simd = wave.reshape(256, 4, 4).sum(axis=1)
work_max_simd = simd.max(1)
work_max_wave = wave.max(1)
st = np.loadtxt(dump).reshape(-1, 256, 16)[2:] / 100.0     # skip 2 warm runs, us
k1 = st[:, :, 1].mean(0)
print('K1 done: mean %.2f min %.2f max %.2f' % (k1.mean(), k1.min(), k1.max()))
print('corr(K1, max-SIMD work) %.3f  corr(K1, max-wave work) %.3f  corr(K1, window total) %.3f' % (
    np.corrcoef(k1, work_max_simd)[0, 1], np.corrcoef(k1, work_max_wave)[0, 1], np.corrcoef(k1, tiles.sum(1))[0, 1]))
for x in range(8):
    sel = np.arange(256) % 8 == x
    print('XCD %d (blockIdx %% 8): K1 mean %.2f max %.2f' % (x, k1[sel].mean(), k1[sel].max()))
fit = np.polyfit(work_max_simd, k1, 1)
print('K1 ~ %.3f us per max-SIMD wave-block + %.2f' % (fit[0], fit[1]))
resid = k1 - np.polyval(fit, work_max_simd)
print('residual std %.2f us; run-to-run std %.2f us' % (resid.std(), st[:, :, 1].std(0).mean() / 100 * 100))
for kk, name in [(2, 'H hashed'), (4, 'H-1 hashed'), (6, 'H-2 hashed')]:
    d = (st[:, :, kk] - st[:, :, kk - 1 if kk == 2 else kk - 1]).mean(0)
    print('%s - previous stamp: mean %.2f max %.2f' % (name, d.mean(), d.max()))
