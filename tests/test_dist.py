"""CPU, world_size 2 (gloo): sharding + the verdict all-gather of the multi-GPU path.

The per-rank search is the oracle here (tests may use it as the checker); on the GPU box the
same code path runs the engine with backend "nccl" (RCCL)."""

import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from mythril_amd.dist import NOT_FOUND, shard_bounds


def test_shard_bounds_balanced_and_complete():
    costs = [10, 1, 1, 1, 50, 3, 3, 30, 1, 1]
    for world in (1, 2, 3, 4, 8, 16):
        b = shard_bounds(costs, world)
        assert len(b) == world and b[0][0] == 0 and b[-1][1] == len(costs)
        assert all(b[i][1] == b[i + 1][0] for i in range(world - 1))
    assert shard_bounds([], 4) == [(0, 0)] * 4


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out_path):
    import torch.distributed as dist

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, "oracle")]
    import pyoracle as O

    from mythril_amd import ir, synth
    from mythril_amd.dist import sharded_check

    progs = [synth.random_dag_set(700 + i, plant=(i % 3 == 0))[0] for i in range(9)]

    def oracle_search(ps, budget, seed, flags):
        b = ir.Batch(ps) if ps else None
        out = []
        for i in range(len(ps)):
            first, _ = O.SetView.from_batch(b, i).check(budget, seed)
            out.append(NOT_FOUND if first is None else first)
        return np.array(out, dtype=np.uint32)

    found = sharded_check(progs, search_fn=oracle_search, budget=48, seed=11)
    np.save(f"{out_path}.{rank}.npy", found)
    dist.destroy_process_group()


def test_two_rank_gather_matches_single_process(tmp_path):
    port = _free_port()
    out = str(tmp_path / "found")
    mp.spawn(_worker, args=(2, port, out), nprocs=2, join=True)
    f0, f1 = np.load(out + ".0.npy"), np.load(out + ".1.npy")
    assert (f0 == f1).all()
    import pyoracle as O

    from mythril_amd import ir, synth

    progs = [synth.random_dag_set(700 + i, plant=(i % 3 == 0))[0] for i in range(9)]
    b = ir.Batch(progs)
    want = []
    for i in range(len(progs)):
        first, _ = O.SetView.from_batch(b, i).check(48, 11)
        want.append(NOT_FOUND if first is None else first)
    assert list(f0) == want
    assert (f0[::3] == 0).all()  # planted witnesses are candidate 0


def _gather_worker(rank, world, port, out_path):
    import torch.distributed as dist

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from mythril_amd.dist import gather_found

    res = []
    for sizes in ((7, 2), (9, 0), (0, 4)):
        lo = sum(sizes[:rank])
        mine = np.array([(lo + i) * 3 if (lo + i) % 2 else NOT_FOUND for i in range(sizes[rank])],
                        dtype=np.uint32)
        res.append(gather_found(mine, lo, sum(sizes)))
    np.save(f"{out_path}.{rank}.npy", np.concatenate(res))
    dist.destroy_process_group()


def test_gather_sends_shards_of_any_length(tmp_path):
    """gather_found all-gathers each rank's own shard (padded to the longest), not a
    full-length array per rank: uneven and empty shards reassemble into the global verdicts,
    u32 values above 2^31 included."""
    port = _free_port()
    out = str(tmp_path / "g")
    mp.spawn(_gather_worker, args=(2, port, out), nprocs=2, join=True)
    g0, g1 = np.load(out + ".0.npy"), np.load(out + ".1.npy")
    assert (g0 == g1).all()
    want = np.concatenate([np.array([i * 3 if i % 2 else NOT_FOUND for i in range(n)], dtype=np.uint32)
                           for n in (9, 9, 4)])
    assert (g0 == want).all()
