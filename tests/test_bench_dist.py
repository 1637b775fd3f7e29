"""bench.py's multi-rank branch on CPU (gloo, world size 2), with the C oracle standing in
for the engine: the step-time max and evals sum over ranks, the verdict all-gather
(mythril_amd.dist.gather_found), the early-exit reductions and rank 0's JSON line — so the
driver's SCALE run is not that code's first execution.  On the GPU box the same ``run`` body
takes backend "nccl" (RCCL) with device tensors."""

import json
import os
import socket
import sys
import time

import numpy as np
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ARGV = ["--sets", "3", "--budget", "64", "--steps", "2", "--warmup", "1", "--keccak-log2", "0", "--quick-sat-queries", "0", "--full-pass-dags", "0",
        "--corpus-scenarios", "0", "--no-cpu-baseline", "--seed", "5"]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _engine():
    import oracle_engine
    from mythril_amd.engine import CheckResult

    class BenchOracleEngine(oracle_engine.OracleEngine):
        """check / check_each with a measured (nonzero) kernel time, as the bench reads."""

        def check(self, db, budget=65536, seed=0, flags=0, timeout_ms=0):
            t0 = time.perf_counter()
            r = super().check(db, budget, seed, flags, timeout_ms)
            return CheckResult(r.found, r.evals_full, r.cands_decided, r.ops,
                               1e3 * (time.perf_counter() - t0) + 1e-3)

        def check_each(self, dbs, budget=65536, seed=0, flags=0, timeout_ms=0):
            return [self.check(db, budget, seed, flags, timeout_ms) for db in dbs]

    return BenchOracleEngine()


def _worker(rank, world, port, out_path):
    import torch.distributed as dist

    sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import bench

    line = bench.run(bench.parse(ARGV), rank, world, 0, dist, engine=_engine(), cdev="cpu")
    if rank == 0:
        with open(out_path, "w") as f:
            json.dump(line, f)
    else:
        assert line is None
    dist.barrier()
    dist.destroy_process_group()


def test_bench_multirank_branch_gloo(tmp_path):
    out = str(tmp_path / "line.json")
    mp.spawn(_worker, args=(2, _free_port(), out), nprocs=2, join=True)
    line = json.load(open(out))
    import bench
    import pyoracle as O

    from mythril_amd import ir, synth

    a = bench.parse(ARGV)
    assert line["n_gpus"] == 2 and line["steps"] == a.steps and line["scaling"] == "weak"
    # every rank's timed sets, full sweep: evals = sets x budget x steps x ranks
    tot = 2 * a.steps * a.sets * a.budget
    assert abs(line["value"] - tot / (line["ms_per_step"] * a.steps / 1e3)) <= 1e-9 * line["value"]
    # the all-gathered verdicts are the oracle's over both ranks' DAG ids
    want = 0
    for k in range(a.warmup, a.warmup + a.steps):
        for r in range(2):
            progs = [synth.random_dag_set((k * 2 + r) * a.sets + i, plant=False)[0] for i in range(a.sets)]
            b = ir.Batch(progs)
            want += sum(O.SetView.from_batch(b, i).check(a.budget, a.seed)[0] is not None
                        for i in range(a.sets))
    assert line["verdicts_gathered"] == 2 * a.steps * a.sets
    assert line["sets_with_witness"] == want
    ee = line["early_exit"]
    assert ee["unplanted"]["sets"] == 2 * a.sets and ee["planted"]["sets_with_witness"] == 2 * a.sets


def _worker_fp(rank, world, port, out_path):
    import torch.distributed as dist

    sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import bench

    argv = [a for a in ARGV]
    i = argv.index("--full-pass-dags")
    argv[i + 1] = "21"
    argv += ["--full-pass-workers", "2"]
    line = bench.run(bench.parse(argv), rank, world, 0, dist, engine=_engine(), cdev="cpu")
    if rank == 0:
        with open(out_path, "w") as f:
            json.dump(line, f)
    dist.barrier()
    dist.destroy_process_group()


def test_bench_full_pass_sharded_over_ranks(tmp_path):
    """The full-pass leg at world size 2: each rank sweeps its contiguous shard of the DAG ids
    (10 + 11 of 21), evals and witnesses summed, times the slowest rank's."""
    out = str(tmp_path / "line.json")
    mp.spawn(_worker_fp, args=(2, _free_port(), out), nprocs=2, join=True)
    fp = json.load(open(out))["full_pass"]
    import bench
    import pyoracle as O

    from mythril_amd import ir, synth

    a = bench.parse(ARGV)
    assert fp["ranks"] == 2 and fp["dags"] == 21 and fp["evals"] == 21 * a.budget
    progs = [synth.random_dag_set(i, plant=False)[0] for i in range(21)]
    b = ir.Batch(progs)
    want = sum(O.SetView.from_batch(b, i).check(a.budget, a.seed)[0] is not None for i in range(21))
    assert fp["sets_with_witness"] == want
    assert fp["planted_early_exit"]["sets_with_witness"] == 21
    assert fp["kernel_s"] > 0 and fp["wall_s"] >= fp["kernel_s"]
