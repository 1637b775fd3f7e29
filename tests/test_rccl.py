"""The RCCL code path at world size 1 on the GPU box: torch.distributed with
backend "nccl" (RCCL on ROCm) and ``device_id=cuda:0``, initialised before any other GPU work
of the test process (the ``first`` marker), then

* ``bench.run``'s multi-rank branch — the evals sum, the step-time max, the early-exit
  reductions and the verdict all-gather over device tensors, exactly the code the driver's
  N-GPU run executes (bench.py ``main`` inits the same way);
* ``dist.gather_found``'s ``"cuda"`` branch and ``dist.sharded_check`` over RCCL, equal to a
  direct search of the same sets.

Everything else about N > 1 is covered by the gloo world-size-2 tests (test_bench_dist.py,
test_dist.py); a multi-GPU number needs the driver's 8-GPU node."""

import os
import socket

import numpy as np
import pytest

ARGV = ["--sets", "64", "--budget", "4096", "--steps", "2", "--warmup", "1", "--keccak-log2", "12",
        "--quick-sat-queries", "0", "--full-pass-dags", "0", "--corpus-scenarios", "0", "--no-cpu-baseline",
        "--seed", "3"]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.first
@pytest.mark.gpu
def test_gpu_rccl_world1_bench_branch_and_verdict_gather(monkeypatch):
    import torch
    import torch.distributed as dist

    import bench
    from mythril_amd import dist as pdist
    from mythril_amd import synth
    from mythril_amd.engine import get_engine

    monkeypatch.setenv("MASTER_ADDR", "127.0.0.1")
    monkeypatch.setenv("MASTER_PORT", str(_free_port()))
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    try:
        assert dist.get_backend() == "nccl"
        args = bench.parse(ARGV)
        line = bench.run(args, 0, 1, 0, dist)
        assert line["n_gpus"] == 1 and line["verdicts_gathered"] == args.steps * args.sets
        assert line["value"] > 0 and line["early_exit"]["planted"]["sets_with_witness"] == args.sets
        # the gathered verdicts of the timed steps equal a direct search of their sets
        progs = synth.random_dag_programs(args.warmup * args.sets, args.steps * args.sets, plant=False)[0]
        eng = get_engine(0)
        db = eng.upload(progs)
        direct = eng.check(db, budget=args.budget, seed=args.seed, flags=2).found
        db.free()
        assert int((direct != pdist.NOT_FOUND).sum()) == line["sets_with_witness"]
        g = pdist.gather_found(direct, 0, len(direct))        # the "cuda" branch
        assert np.array_equal(g, direct)
        sh = pdist.sharded_check(progs, budget=args.budget, seed=args.seed, flags=2)
        assert np.array_equal(sh, direct)
    finally:
        dist.destroy_process_group()
