"""Multi-GPU sharding of the synctree path.

Two ways to spread the path over the GPUs of one node, one process per GPU
(``torch.distributed``; backend ``nccl`` = RCCL over xGMI on MI355X, ``gloo``
in the CPU tests):

* **Ensemble sharding** (configs 2 and 4).  Every ensemble/peer owns its own
  tree (``riak_ensemble_peer.erl:1845-1846``), so ensemble ``e`` lives on rank
  ``e % world`` and the data path has no collective.  :func:`gather_tops`
  all-gathers the per-ensemble top hashes (17 B + presence each) afterwards.

* **Segment-range partition** of ONE huge tree (config 5).  Rank ``g`` owns
  segments ``[g*S/G, (g+1)*S/G)`` (G divides the 16 level-2 subtrees).  Every
  rank receives the same write batches and keeps its own keys
  (``st_set_partition``); a rehash hashes its subtrees up to level 2, one
  all-gather exchanges the 16 level-2 entries (18 B each), and every rank
  finishes level 1 + the top hash redundantly (``st_combine_upper``).  Inner
  levels are a reduction tree over independent segments, so this is the only
  exchange step.

The local tree is duck-typed (``set_partition``, ``insert_int64_device`` /
``insert_batch``, ``rehash``, ``level_entries``, ``combine_upper``,
``top_hash``): :class:`riak_ensemble_amd.synctree_hip.DeviceTree` in
production.
"""
import numpy as np


def partition_range(rank, world, segments, width=16):
    """Segment range [lo, hi) owned by `rank` of `world` (whole level-2 subtrees)."""
    if width != 16 or world < 1 or 16 % world:
        raise ValueError('segment-range partition needs width 16 and a world size dividing 16')
    per = segments // world
    return rank * per, (rank + 1) * per


def _allgather_bytes(dist, group, mine, device):
    """All-gather equal-length uint8 rows; returns a (world, len) numpy array."""
    import torch
    world = dist.get_world_size(group)
    t = torch.from_numpy(np.ascontiguousarray(mine, np.uint8)).to(device)
    out = torch.empty(world * t.numel(), dtype=torch.uint8, device=device)
    dist.all_gather_into_tensor(out, t, group=group)
    return out.cpu().numpy().reshape(world, -1)


class PartitionedTree:
    """One synctree partitioned by segment range across the ranks of `group`."""

    def __init__(self, local_tree, dist, group=None, device='cpu'):
        self.tree = local_tree
        self.dist = dist
        self.group = group
        self.device = device
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        self.lo, self.hi = partition_range(self.rank, self.world, local_tree.segments, local_tree.width)
        self.b2 = (self.lo * 16 // local_tree.segments, self.hi * 16 // local_tree.segments)
        if self.world > 1:
            local_tree.set_partition(self.lo, self.hi)

    def combine(self):
        """All-gather the owned level-2 entries; finish level 1 + top everywhere."""
        if self.world == 1:
            return
        pres, hashes = self.tree.level_entries(2)
        a, b = self.b2
        mine = np.concatenate([pres[a:b, None], hashes[a:b]], axis=1).reshape(-1)   # (b-a) x 18 B
        rows = _allgather_bytes(self.dist, self.group, mine, self.device).reshape(-1, 18)
        self.tree.combine_upper(rows[:, 0].copy(), rows[:, 1:].copy())

    def rehash(self):
        self.tree.rehash()
        self.combine()

    def top_hash(self):
        return self.tree.top_hash()


def gather_tops(dist, tops, group=None, device='cpu'):
    """Ensemble sharding: all-gather per-ensemble top hashes.

    `tops` is this rank's list of 17-byte hashes (or ``'undefined'``), one per
    local ensemble, the same count on every rank.  Returns the list of all
    ensembles' tops in (rank, local index) order."""
    rows = np.zeros((len(tops), 18), np.uint8)
    for i, h in enumerate(tops):
        if isinstance(h, (bytes, bytearray)):
            rows[i, 0] = 1
            rows[i, 1:] = np.frombuffer(bytes(h), np.uint8)
    allr = _allgather_bytes(dist, group, rows.reshape(-1), device).reshape(-1, 18)
    return [bytes(r[1:]) if r[0] else 'undefined' for r in allr]
