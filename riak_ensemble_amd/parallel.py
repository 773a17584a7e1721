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

* **Partitioned exchange** (config 3 over a config-5 tree).  Two trees
  partitioned alike (local and remote copy of the same segment ranges):
  every rank compares its own level-2 subtrees (``st_compare`` on a
  partitioned pair) with no collective; one all-gather of (first error,
  record-bytes length) and one of the padded record bytes then give every
  rank the reference's whole diff list: ``Keys ++ Acc`` over ascending
  segments (synctree.erl:373-375) = the highest rank's records first.  The
  first corruption is the minimum (level, bucket, side) over the ranks --
  the reference's level-by-level visiting order.  ``exchange`` applies the
  partition's own diffs (riak_ensemble_exchange.erl:71-97) and re-combines
  the upper levels.

The local tree is duck-typed (``set_partition``, ``insert_int64_device`` /
``insert_batch``, ``rehash``, ``level_entries``, ``combine_upper``,
``top_hash``, ``compare``, ``exchange_apply``):
:class:`riak_ensemble_amd.synctree_hip.DeviceTree` in production.
"""
import struct

import numpy as np

from . import terms

_NO_ERR = (1 << 64) - 1


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
    t = torch.from_numpy(np.array(mine, np.uint8, copy=True).reshape(-1)).to(device)
    out = torch.empty(world * t.numel(), dtype=torch.uint8, device=device)
    dist.all_gather_into_tensor(out, t, group=group)
    return out.cpu().numpy().reshape(world, -1)


def _allgather_var(dist, group, blob, device):
    """All-gather variable-length byte strings (lengths first, then the
    padded rows); returns the list of every rank's bytes."""
    lens = _allgather_bytes(dist, group, np.frombuffer(struct.pack('<q', len(blob)), np.uint8), device)
    lens = [struct.unpack('<q', r.tobytes())[0] for r in lens]
    mx = max(lens)
    if mx == 0:
        return [b''] * len(lens)
    rows = _allgather_bytes(dist, group, np.frombuffer(blob + bytes(mx - len(blob)), np.uint8), device)
    return [rows[r, :lens[r]].tobytes() for r in range(len(lens))]


def err_code(level, bucket, side):
    """(level, bucket, side) of a corrupted node as one orderable integer."""
    return (int(level) << 56) | (int(bucket) << 1) | (0 if side == 'local' else 1)


def pack_diffs(recs):
    """[(seg, key, (va, vb))...] -> bytes (seg u64, key type u8, value flags u8,
    three u32 lengths, then the key / value bytes)."""
    out = []
    for seg, key, (va, vb) in recs:
        kt, kb = terms.key_parts(key)
        fl = (1 if va == terms.NONE else 0) | (2 if vb == terms.NONE else 0)
        a = b'' if fl & 1 else bytes(va)
        b = b'' if fl & 2 else bytes(vb)
        out.append(struct.pack('<QBBIII', seg, kt, fl, len(kb), len(a), len(b)) + kb + a + b)
    return b''.join(out)


def unpack_diffs(blob):
    recs, o, hs = [], 0, struct.calcsize('<QBBIII')
    while o < len(blob):
        seg, kt, fl, kl, al, bl = struct.unpack_from('<QBBIII', blob, o)
        o += hs
        kb = blob[o:o + kl]
        o += kl
        va = terms.NONE if fl & 1 else blob[o:o + al]
        o += al
        vb = terms.NONE if fl & 2 else blob[o:o + bl]
        o += bl
        recs.append((seg, terms.key_from_parts(kt, kb), (va, vb)))
    return recs


def local_diff(tree, remote_tree, filt=0):
    """This partition's part of a partitioned compare: (first error code or
    ~0, packed records in reference order)."""
    res = tree.compare(remote_tree, filt)
    if res[0] == 'corrupted':
        _, side, (_, lvl, bkt) = res
        return err_code(lvl, bkt, side), b''
    return _NO_ERR, pack_diffs(res[1])


def merge_diffs(parts):
    """[(err, blob)] in rank order -> ('ok', records of the whole tree in
    reference order) or ('corrupted', side, (corrupted, L, B)) for the first
    corrupted node over all partitions."""
    e = min(p[0] for p in parts)
    if e != _NO_ERR:
        side = 'remote' if e & 1 else 'local'
        return ('corrupted', side, (terms.CORRUPTED, e >> 56, (e & ((1 << 56) - 1)) >> 1))
    out = []
    for _, blob in reversed(parts):   # highest segments (highest rank) first
        out.extend(unpack_diffs(blob))
    return ('ok', out)


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

    def compare(self, remote, filt=0):
        """Collective: the reference compare of the whole local tree against the
        whole remote tree (both partitioned alike, upper levels combined).
        Every rank returns the same result."""
        if self.world == 1:
            return merge_diffs([local_diff(self.tree, remote.tree, filt)])
        err, blob = local_diff(self.tree, remote.tree, filt)
        errs = _allgather_bytes(self.dist, self.group, np.frombuffer(struct.pack('<Q', err), np.uint8), self.device)
        errs = [struct.unpack('<Q', r.tobytes())[0] for r in errs]
        if min(errs) != _NO_ERR:   # no records travel when any partition is corrupted
            return merge_diffs([(e, b'') for e in errs])
        blobs = _allgather_var(self.dist, self.group, blob, self.device)
        return merge_diffs(list(zip(errs, blobs)))

    def exchange(self, remote):
        """Collective exchange of the whole local tree with the whole remote
        copy (riak_ensemble_exchange.erl:71-97).  Every rank first plans its
        partition (st_exchange_plan: compare + valid_obj_hash selection); a
        corruption anywhere aborts with nothing applied; otherwise the
        partitions apply in the reference's diff order -- highest segments
        (highest rank) first -- up to the first function_clause crash: ranks
        above the first crashing rank apply everything, that rank applies the
        diffs before its crash, ranks below apply nothing.  The upper levels
        are then re-combined.  Returns ('ok' | 'exchange_failed',
        {'diffs', 'applied', 'rejected'}) summed over the ranks, or the first
        ('corrupted', side, tuple); the same on every rank."""
        plan = self.tree.exchange_plan(remote.tree)
        if plan[0] == 'corrupted':
            row = (2, err_code(plan[2][1], plan[2][2], plan[1]))
        else:
            row = (1 if plan[0] == 'exchange_failed' else 0, 0)
        rows = [row]
        if self.world > 1:
            g = _allgather_bytes(self.dist, self.group, np.frombuffer(struct.pack('<BQ', *row), np.uint8), self.device)
            rows = [struct.unpack('<BQ', r.tobytes()) for r in g]
        bad = [e for t, e in rows if t == 2]
        if bad:
            e = min(bad)
            return ('corrupted', 'remote' if e & 1 else 'local', (terms.CORRUPTED, e >> 56, (e & ((1 << 56) - 1)) >> 1))
        crashing = [r for r, (t, _) in enumerate(rows) if t == 1]
        first = max(crashing) if crashing else -1   # first crash in application order
        if self.rank >= first:
            res = self.tree.exchange_apply(remote.tree)
            info = res[1]
        else:
            info = {'diffs': plan[1]['diffs'], 'applied': 0, 'rejected': 0}
        self.combine()
        tot = np.array([info['diffs'], info['applied'], info['rejected']], np.uint64)
        if self.world > 1:
            g = _allgather_bytes(self.dist, self.group, tot.view(np.uint8), self.device)
            tot = g.copy().view(np.uint64).reshape(self.world, 3).sum(axis=0)
        summary = {'diffs': int(tot[0]), 'applied': int(tot[1]), 'rejected': int(tot[2])}
        return ('exchange_failed' if crashing else 'ok', summary)


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
