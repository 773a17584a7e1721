"""GPU box diagnostic: phase stamps of the per-key kernel (ST_SMALL_STAMPS=1)
for single-key get and insert on a 100k-key tree."""
import os
import sys

os.environ.setdefault('ST_SMALL_STAMPS', '1')
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from riak_ensemble_amd import synctree_hip, workload

keys = workload.keys_int63(100_000, workload.SEED ^ 0x100)
vals = workload.obj_hash_values(len(keys))
t = synctree_hip.DeviceTree()
t.insert_int64(keys, vals)
t.rehash()
for k in keys[:5]:
    t.get_batch([int(k)])
for k in keys[:5]:
    t.insert_batch([int(k)], [bytes(17)])
# the clock an insert finds: after 100 ms idle, and right behind a 10M-key-class
# load of work (20 rehashes of this tree queued just before)
import time
import sys as _s
for label in ('idle', 'busy'):
    for k in keys[5:10]:
        if label == 'idle':
            time.sleep(0.1)
        else:
            for _ in range(20):
                t.rehash()
        print('--- %s' % label, file=_s.stderr, flush=True)
        t.insert_batch([int(k)], [bytes(17)])
