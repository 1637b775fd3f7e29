"""Multi-GPU sharding of constraint-set batches.

One process per GPU (torch.distributed, backend "nccl" = RCCL over xGMI on ROCm; "gloo" in
the CPU tests).  Sets are independent, so the data path has no collective: every rank
lowers the same list of sets, searches only its shard, and one all-gather of fixed-size
verdict records (set id, witness index) makes every rank's view complete.  Witness values
are then re-materialised locally where needed (a witness is a pure function of the set and
the candidate index).  The records are a few bytes per set — latency-bound messages, so
xGMI bandwidth is never the limit.
"""

from __future__ import annotations

from typing import Callable, List, Optional, Sequence, Tuple

import numpy as np

NOT_FOUND = 0xFFFFFFFF


def shard_bounds(costs: Sequence[int], world: int) -> List[Tuple[int, int]]:
    """Contiguous shards of ~equal total cost (bytecode length x budget per set)."""
    costs = np.asarray(costs, dtype=np.float64)
    n = len(costs)
    if n == 0:
        return [(0, 0)] * world
    cum = np.concatenate([[0.0], np.cumsum(costs)])
    total = cum[-1]
    bounds, start = [], 0
    for r in range(world):
        if r == world - 1:
            end = n
        else:
            target = total * (r + 1) / world
            end = int(np.searchsorted(cum, target, side="left"))
            end = max(start, min(end, n))
        bounds.append((start, end))
        start = end
    return bounds


def gather_found(local_found: np.ndarray, lo: int, n_total: int, group=None) -> np.ndarray:
    """All-gather per-set witness indices from every rank's shard [lo, lo+len)."""
    import torch
    import torch.distributed as dist

    world = dist.get_world_size(group)
    rec = np.full(n_total, NOT_FOUND, dtype=np.int64)
    rec[lo:lo + len(local_found)] = local_found.astype(np.int64)
    backend = dist.get_backend(group)
    dev = "cuda" if backend == "nccl" else "cpu"
    t = torch.from_numpy(rec).to(dev)
    parts = [torch.empty_like(t) for _ in range(world)]
    dist.all_gather(parts, t, group=group)
    out = np.full(n_total, NOT_FOUND, dtype=np.int64)
    for p in parts:
        p = p.cpu().numpy()
        mask = p != NOT_FOUND
        out[mask] = np.minimum(out[mask], p[mask])
    return out.astype(np.uint32)


def sharded_check(programs, search_fn: Optional[Callable] = None, budget: int = 65536,
                  seed: int = 0, flags: int = 2, group=None) -> np.ndarray:
    """Search `programs` across all ranks; returns the global found[] on every rank.

    ``search_fn(programs, budget, seed, flags) -> found`` runs the local shard (default: the
    GPU engine of this rank)."""
    import torch.distributed as dist

    rank, world = dist.get_rank(group), dist.get_world_size(group)
    costs = [p.sched_cost() for p in programs]
    lo, hi = shard_bounds(costs, world)[rank]
    if search_fn is None:
        from .engine import get_engine

        eng = get_engine()

        def search_fn(progs, budget, seed, flags):
            if not progs:
                return np.zeros(0, dtype=np.uint32)
            db = eng.upload(progs)
            r = eng.check(db, budget=budget, seed=seed, flags=flags)
            db.free()
            return r.found

    local = search_fn(programs[lo:hi], budget, seed, flags)
    return gather_found(np.asarray(local), lo, len(programs), group)
