"""Phase stamps of k_rehash_fused on ONE 1M-key tree (the config-4 tree
size): ST_LEVEL_STAMPS=1 prints per-phase min/median/max over the windows."""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from riak_ensemble_amd import synctree_hip, workload  # noqa: E402
n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
t = synctree_hip.DeviceTree()
t.insert_int64(workload.keys_int63(n, workload.SEED ^ 1), workload.obj_hash_values(n))
for _ in range(3):
    t.rehash()
t.sync()
print('done', flush=True)
