"""Multi-GPU sharding of a BlockEnsemble: one process per GPU.

A global SamplingEnsemble of R recordings is split into contiguous recording shards, one per
rank.  Blocks never cross recordings, so the whole MCMC iteration (draw, Girsanov weight, MH
decision) is shard-local; the only exchange is ``fetch_ll``: every rank all-gathers its three
partials (ll, ll°, accepted count) and all ranks combine them with the same rank-order tree
(libdmt does this over RCCL in ``finish_reduction``, dmt_runtime.hip).  RNG streams are keyed
by GLOBAL segment ids (``Ensemble.set_shard``), so a shard draws exactly the variables its
recordings would get in the unsharded ensemble; with power-of-two blocks per rank the
reduction tree equals the single-GPU tree too, so sharded and unsharded runs are bit-identical.
"""
from __future__ import annotations

import numpy as np


def shard_range(n_recordings: int, world: int, rank: int):
    """Contiguous, balanced recording range [r0, r1) of ``rank``."""
    base, extra = divmod(n_recordings, world)
    r0 = rank * base + min(rank, extra)
    return r0, r0 + base + (1 if rank < extra else 0)


def segment_base(n_segments_per_recording, r0: int) -> int:
    """Global id of the first segment of recording r0 (the shard's ``seg_base``)."""
    return int(np.sum(np.asarray(n_segments_per_recording[:r0], dtype=np.int64)))


def rank_tree(values):
    """The rank-order reduction of libdmt's multi-rank fetch_ll: complete adjacent-pair tree
    over ranks padded to a power of two, + 0.0."""
    v = [float(x) for x in values]
    n2 = 1
    while n2 < len(v):
        n2 *= 2
    v += [0.0] * (n2 - len(v))
    while len(v) > 1:
        v = [v[2 * j] + v[2 * j + 1] for j in range(len(v) // 2)]
    return v[0] + 0.0


def combine_partials(partials, group=None):
    """Host-side restatement of the cross-rank step over a ``torch.distributed`` group
    (gloo on CPU): all-gather the 3 partials, combine in rank order on every rank."""
    import torch
    import torch.distributed as dist
    t = torch.tensor([float(x) for x in partials], dtype=torch.float64)
    out = [torch.empty_like(t) for _ in range(dist.get_world_size(group))]
    dist.all_gather(out, t, group=group)
    allv = torch.stack(out).numpy()
    return tuple(rank_tree(allv[:, c]) for c in range(allv.shape[1]))
