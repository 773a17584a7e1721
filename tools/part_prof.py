"""Profile helper: bench.py's config-5 leg alone (one rank)."""
import argparse
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import bench
from riak_ensemble_amd import synctree_hip

a = argparse.Namespace(part_keys=int(sys.argv[1]) if len(sys.argv) > 1 else 100_000_000, part_batches=5,
                       part_batch_keys=1_000_000)
print(bench._bench_partition(synctree_hip, None, torch.device('cuda', 0), a, 0, torch))
