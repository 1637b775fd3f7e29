#!/usr/bin/env python3
"""Benchmark: constraint-candidate evaluations/sec on MI355X (BASELINE.json metric).

Workload (BASELINE.json configs[2]): synthetic random 256-bit
BitVec constraint DAGs (depth 32, MUL/DIV/EXP-heavy mix), 65,536 generated candidates each.
A *step* is one batch of `--sets` DAGs searched over the full candidate budget on one GPU
("full sweep": early exit off, every candidate evaluates the whole program — the unit of
work is one complete set-evaluation per candidate).  Inputs (bytecode) are uploaded to HBM
before the timed region; candidates are generated on device.

Multi-GPU: one process per GPU (torch.distributed.run); every rank searches its own DAG ids
(weak scaling, no data-path collective); the verdict bitmaps are all-gathered once after the
timed region (RCCL), which is the only collective the path has.

Prints one JSON line (rank 0) with roofline (integer VALU) and cpu_baseline objects.
"""

from __future__ import annotations

import argparse
import gc
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

# gfx950 integer VALU peak: 256 CUs x 4 SIMD-32 x 32 lanes x 2.4 GHz (MI355X_MICROARCH.md:
# FP32 vector 157.3 TFLOPS = 78.6 T lane-ops/s counting an FMA as one op)
INT32_PEAK_OPS = 256 * 4 * 32 * 2.4e9


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=8)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--sets", type=int, default=1024, help="DAGs per step per GPU")
    ap.add_argument("--budget", type=int, default=65536, help="candidates per DAG")
    ap.add_argument("--mode", choices=["full", "early"], default="full")
    # global candidate seed 0: candidate c of DAG d is Philox keyed by the set seed
    # 0x4D595448 ^ d alone (synth.CAND_SEED_BASE)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--cpu-sample-s", type=float, default=15.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--keccak-log2", type=int, default=24,
                    help="config 4: 2^k 64-byte key||slot messages per Keccak launch (0 = skip)")
    ap.add_argument("--lib", default=None, help="alternative build of libpathfeas.so (experiments)")
    ap.add_argument("--serial-steps", action="store_true",
                    help="one waited pf_check_batch call per step instead of all K enqueued at once")
    ap.add_argument("--corpus-scenarios", type=int, default=48,
                    help="LASER-shaped scenarios for the %% discharged half of the metric (0 = skip)")
    ap.add_argument("--full-pass-dags", type=int, default=1_000_000,
                    help="config 3 as specified: one pass over this many DAGs, split over the ranks (0 = skip)")
    ap.add_argument("--full-pass-workers", type=int, default=16)
    ap.add_argument("--quick-sat-queries", type=int, default=120,
                    help="queries of the quick-sat (100 cached models) and funnel legs (0 = skip)")
    return ap.parse_args(argv)


def cpu_baseline(programs, budget, seed, target_s):
    """Oracle on the host cores (rank 0, N=1 only): the C restatement if built, else Python."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    try:
        import coracle_py  # C restatement via ctypes (oracle/Makefile)

        return coracle_py.baseline(programs, budget, seed, target_s)
    except Exception as e:  # pragma: no cover - informative fallback for the baseline only
        err = str(e)
    import pyoracle as O
    from mythril_amd import ir

    b = ir.Batch(programs)
    t0 = time.perf_counter()
    evals = 0
    s = 0
    while time.perf_counter() - t0 < target_s and s < len(programs):
        sv = O.SetView.from_batch(b, s)
        n = 64
        assigns = sv.gen_assignments(np.arange(n, dtype=np.uint64), seed)
        for a in assigns:
            sv.evaluate(a)
        evals += n
        s += 1
    dt = time.perf_counter() - t0
    return {"value": evals / dt, "unit": "evals/s", "cores": 1, "kind": "port",
            "sample": f"python oracle, {s} sets x 64 candidates ({err[:60]})"}


def discharge(args):
    """The metric's second half, measured on the builder's LASER-shaped corpus — NOT the
    BASELINE population (z3 queries of ``myth analyze solidity_examples -t 3``, which needs
    z3 + solc, absent here): % of objective-free feasibility queries answered on the GPU.

    Queries: mythril_amd/corpus.py — LASER-shaped sets (both successors of every JUMPI fork
    and every tx-boundary state, svm.py:266-286,351-358) along planted 2-transaction
    scenarios over token / BECToken / EtherStore / Rubixi / KillBilly / WalletLibrary
    logic; the planted side of each fork is SAT by construction, the other side is open
    (z3 would decide it).  All queries go through the drop-in batched funnel in one call.
    Reported beside the rate:
    * provenance of the witnesses: ``hint_only`` (every bucket answered by candidate 0, the
      host's constraint-directed hint model) vs ``searched`` (a bucket's witness came from
      the GPU candidate search);
    * a labelled-UNSAT slice (the reference's UNSAT KATs + planted contradictions,
      corpus.labelled_unsat): ``unsat_labelled_false_positives`` must be 0;
    * ``single_query_ms``: cold latency of one query through check_sets (lowering + one
      launch + re-check), the live fork-prune path, beside the batched throughput."""
    from mythril_amd import corpus
    from mythril_amd.smt import gpu_check

    # the lowering workers are spawned once per analysis process: start them before the
    # clock, as a live run has them from its first batch on
    t_pool = time.perf_counter()
    n_workers = gpu_check.warm_pool()
    t_pool = time.perf_counter() - t_pool
    t0 = time.perf_counter()
    c = corpus.build(args.corpus_scenarios, 2, seed=2024)
    n_planted = corpus.validate(c)
    gc.collect()
    t1 = time.perf_counter()
    gpu_check.reset_cache()
    gpu_check.STATS.bucket_origin.clear()
    s0 = (gpu_check.STATS.kernel_ms, gpu_check.STATS.buckets, gpu_check.STATS.host_s)
    gpu_check.STATS.phase_s.clear()
    models = gpu_check.check_sets([q.constraints for q in c.queries], registry=c.kfm.registry)
    t2 = time.perf_counter()
    got = [m is not None for m in models]
    planted_hit = sum(1 for g, q in zip(got, c.queries) if g and q.label == "sat")
    n = len(c.queries)
    kinds = [m.origin for m in models if m is not None]
    stats_batch = (gpu_check.STATS.buckets - s0[1], gpu_check.STATS.kernel_ms - s0[0],
                   gpu_check.STATS.host_s - s0[2])
    bucket_origin = dict(gpu_check.STATS.bucket_origin)
    phase_s = {k: round(v, 4) for k, v in gpu_check.STATS.phase_s.items()}
    # the same corpus again with the answer caches cleared: its terms are now in the native
    # store with their bucket keys memoised — a live analysis's steady state, where each new
    # query shares all but its newest conjunct with earlier ones (the figure above is cold)
    gpu_check.reset_cache()
    gpu_check.STATS.phase_s.clear()
    # the cold call leaves a young generation full of its results: collect before the clock
    # so a gen-2 pass (0.1-0.2 s on the box's heap) does not land inside one leg at random
    gc.collect()
    t3 = time.perf_counter()
    gpu_check.check_sets([q.constraints for q in c.queries], registry=c.kfm.registry)
    t_rep = time.perf_counter() - t3
    phase_rep = {k: round(v, 4) for k, v in gpu_check.STATS.phase_s.items()}
    # soundness slice: UNSAT by construction, never answered sat
    unsat = corpus.labelled_unsat(c, n=256)
    fps = []
    for reg in {id(r): r for _, _, r in unsat}.values():
        group = [(cs, o) for cs, o, r in unsat if r is reg]
        ms = gpu_check.check_sets([cs for cs, _ in group], registry=reg)
        fps += [o for (cs, o), m in zip(group, ms) if m is not None]
    # the GPU search on its own: the same corpus with the host hint models switched off
    # (candidate 0 is then just the generator's first candidate)
    from dataclasses import replace as _replace

    gpu_check.reset_cache()
    ms_nh = gpu_check.check_sets([q.constraints for q in c.queries], registry=c.kfm.registry,
                                 config=_replace(gpu_check.CONFIG, hints=False))
    no_hints = sum(m is not None for m in ms_nh)
    # ... and in live order (fork pairs one call at a time, svm.py:351-358), where each new
    # bucket's search starts from the parent models of the queries answered before it
    gpu_check.reset_cache()
    cfg_live = _replace(gpu_check.CONFIG, hints=False, parents=True)
    t_live = time.perf_counter()
    live = []
    for g in corpus.live_order_groups(c.queries):
        live += gpu_check.check_sets([q.constraints for q in g], registry=c.kfm.registry, config=cfg_live)
    t_live = time.perf_counter() - t_live
    live_kinds = [m.origin for m in live if m is not None]
    # cold single-query latency (the fork-prune call site answers one query at a time)
    sample = [q for q in c.queries if q.label == "sat"][:96]
    lat = []
    gpu_check.STATS.phase_s.clear()
    slowest = (0.0, {})
    for q in sample:
        gpu_check.reset_cache()
        before = dict(gpu_check.STATS.phase_s)
        ts = time.perf_counter()
        gpu_check.check_sets([q.constraints], registry=c.kfm.registry)
        lat.append(1e3 * (time.perf_counter() - ts))
        if lat[-1] > slowest[0]:
            slowest = (lat[-1], {k: round(1e3 * (v - before.get(k, 0.0)), 3)
                                 for k, v in gpu_check.STATS.phase_s.items()})
    sq_phase = {k: round(1e3 * v / max(len(lat), 1), 3) for k, v in gpu_check.STATS.phase_s.items()}
    gpu_check.reset_cache()
    return {"population": "builder corpus (mythril_amd/corpus.py), not BASELINE's "
                          "solidity_examples -t 3 z3 queries (needs z3 + solc)",
            "queries": n, "planted_sat": n_planted, "gpu_sat": sum(got),
            "gpu_sat_planted": planted_hit,
            "pct_discharged_builder_corpus": 100.0 * sum(got) / max(n, 1),
            "pct_planted_discharged": 100.0 * planted_hit / max(n_planted, 1),
            # per set: "searched" = some bucket's witness is a later GPU candidate (index > 0);
            # "hint_only" = every bucket answered by candidate 0, at least one of them the
            # host hint model (the rest: an unhinted bucket's first generated candidate)
            "hint_only": kinds.count("hint"), "searched": kinds.count("search"),
            "first_candidate_only": kinds.count("first"), "from_cache": kinds.count("cache"),
            "bucket_witness_origin": bucket_origin,
            "pct_discharged_without_hints": 100.0 * no_hints / max(n, 1),
            "without_hints_live_order": {
                "pct_discharged": 100.0 * len(live_kinds) / max(n, 1),
                "searched": live_kinds.count("search"), "parent": live_kinds.count("parent"),
                "first_candidate_only": live_kinds.count("first"), "from_cache": live_kinds.count("cache"),
                "queries_per_s": n / max(t_live, 1e-9),
                "note": "hints off, parent models on; fork pairs posed one call at a time"},
            "recheck_failures": gpu_check.STATS.recheck_failures,
            "unsat_labelled": len(unsat), "unsat_labelled_false_positives": len(fps),
            "false_positive_origins": fps[:5],
            "single_query_ms": {"median": float(np.median(lat)) if lat else None,
                                "mean": float(np.mean(lat)) if lat else None,
                                "p95": float(np.percentile(lat, 95)) if lat else None,
                                "max": float(np.max(lat)) if lat else None, "queries": len(lat),
                                "phase_mean_ms": sq_phase, "max_phase_ms": slowest[1]},
            "buckets_searched": stats_batch[0], "kernel_ms": stats_batch[1], "host_s": stats_batch[2],
            "phase_s": phase_s, "lowering_workers": n_workers, "pool_start_s": round(t_pool, 3),
            "wall_s": t2 - t1, "corpus_build_s": t1 - t0,
            "queries_per_s": n / max(t2 - t1, 1e-9),
            "queries_per_s_terms_known": n / max(t_rep, 1e-9), "phase_s_terms_known": phase_rep,
            "corpus": f"mythril_amd/corpus.py, {args.corpus_scenarios} planted 2-tx scenarios "
                      f"(config-2 substitute: no z3/solc for --solver-log dumps)"}


def full_pass_leg(args, eng, rank=0, world=1, dist=None, cdev="cuda"):
    """BASELINE config 3 as specified: ONE pass over the 1,000,000 DAGs ×
    65,536 candidates, full sweep (plus the planted early-exit pass over the same ids), the
    host workers generating and lowering the next chunks while the device sweeps
    (tools/full_pass.py).  Two rates: over the kernel time (inputs resident, the headline's
    definition) and over the wall time (host generation included).  With N ranks the DAG ids
    are split into N contiguous shards (strong scaling of the fixed pass: no data-path
    collective; the per-rank figures are reduced afterwards — evals and witnesses summed,
    kernel and wall time the slowest rank's)."""
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import full_pass

    D = args.full_pass_dags
    lo, hi = rank * D // world, (rank + 1) * D // world
    gc.collect()
    if dist is not None:
        dist.barrier()
    res = full_pass.run_full_pass(eng, dags=hi - lo, first=lo, workers=args.full_pass_workers,
                                  budget=args.budget, seed=args.seed, mp_context="spawn")
    fs, pe = res["full_sweep"], res["planted_early_exit"]
    vals = [float(fs["evals_full"]), float(fs["sets_with_witness"]), float(pe["sets_with_witness"]),
            float(pe["cands_decided"]), fs["kernel_s"], res["total_wall_s"], pe["kernel_s"]]
    if dist is not None:
        import torch

        t_sum = torch.tensor(vals[:4], dtype=torch.float64, device=cdev)
        t_max = torch.tensor(vals[4:], dtype=torch.float64, device=cdev)
        dist.all_reduce(t_sum, op=dist.ReduceOp.SUM)
        dist.all_reduce(t_max, op=dist.ReduceOp.MAX)
        vals = [float(x) for x in t_sum.cpu().tolist()] + [float(x) for x in t_max.cpu().tolist()]
    evals, wit, pwit, pdec, ks, wall, pks = vals
    return {"dags": D, "candidates_per_dag": args.budget, "ranks": world,
            "evals": evals, "kernel_s": ks, "wall_s": wall,
            "evals_per_s_kernel": evals / ks if ks else None, "evals_per_s_wall": evals / wall if wall else None,
            "sets_with_witness": int(wit), "chunks_rank0": fs["chunks"],
            "host_wait_s_rank0": res["host_wait_s"], "upload_s_rank0": res.get("upload_s"),
            "host_workers_per_rank": res["host_workers"],
            "planted_early_exit": {"kernel_s": pks, "sets_with_witness": int(pwit), "cands_decided": int(pdec),
                                   "set_verdicts_per_s_kernel": D / pks if pks else None},
            "seeds": res["seeds"],
            "scaling": "strong: the 1,000,000 DAG ids split over the ranks" if world > 1 else None}


def quick_sat_leg(args):
    """The quick-sat loop before every objective-free query (support/model.py:95-98,
    support_utils.py:57-71) with 100 cached models — the reference loop (deep copy + eval per
    model) vs the GPU-resident ModelCache (mythril_amd/model_cache.py), same models, same
    queries, every choice compared — for a live-like cache of GPU witnesses and for a mixed
    one (GPU witnesses, z3-shaped models, empty models); then the whole funnel's per-query
    cost with the drop-in installed.  Runs in a Mythril-shaped process made of the test
    stand-ins (tests/fake_z3.py, tests/mythril_standin.py: Mythril and z3 are absent here),
    so z3's own eval / simplify costs are the stand-in's, not libz3's."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import model_cache_workload as W

    n = args.quick_sat_queries
    gc.collect()
    return {"witness_cache": W.quick_sat_profile(n_models=100, n_scenarios=24, n_queries=n,
                                                 gpu_frac=1.0, empty_frac=0.0),
            "mixed_cache": W.quick_sat_profile(n_models=100, n_scenarios=16, n_queries=n),
            "funnel": W.funnel_profile(n_scenarios=16, n_queries=2 * n)}


# Keccak-f[1600] = 6,500 int32 ops per permutation; a 64-byte key||slot
# preimage is one permutation and moves 64 B in + 32 B out of HBM.
KECCAK_OPS = 6500
KECCAK_BYTES = 64 + 32
# VALU instructions pf_keccak_fixed_kernel issues per wave (64 messages, one permutation per
# lane): the straight-line ISA count at this build (hipcc -S, 2,792 v_bitop3_b32 + 1,352
# v_alignbit_b32 + moves/loads), so the hardware view prices the kernel at what it issues,
# not at the §8(d) table's 6,500 ops
KECCAK_VALU_PER_WAVE = 4340
VALU_ISSUE_PER_S = 256 * 4 * 2.4e9 / 2   # wave64 VALU instructions per second (2 cycles each)
KECCAK_CYCLES_PER_WAVE = 2792 * 2.76 + 1352 * 4.69 + (4340 - 2792 - 1352) * 2.76


def keccak_leg(args, torch, rank, world):
    """Config 4 (BASELINE.json configs[3]): batched Keccak-256 over 2^k 64-byte mapping-slot
    preimages resident in HBM (pf_keccak_fixed_kernel), HIP-event time of each launch on
    the stream it runs on.  Weak scaling: every rank hashes its own 2^k messages."""
    import ctypes

    from mythril_amd import _lib

    n = 1 << args.keccak_log2
    g = torch.Generator(device="cuda").manual_seed(0x4B454343 + rank)
    data = torch.randint(0, 256, (n * 64,), dtype=torch.uint8, device="cuda", generator=g)
    out = torch.empty(n * 32, dtype=torch.uint8, device="cuda")
    stream = torch.cuda.current_stream().cuda_stream
    L = _lib.lib()
    ms = ctypes.c_float(0)
    kms = []
    for k in range(args.warmup + args.steps):
        _lib.check(L.pf_keccak256_fixed_dev(data.data_ptr(), 64, n, out.data_ptr(),
                                            ctypes.byref(ms), stream), "pf_keccak256_fixed_dev")
        if k >= args.warmup:
            kms.append(ms.value)
    torch.cuda.synchronize()
    t = float(np.mean(kms)) / 1e3
    if world > 1:
        import torch.distributed as dist

        x = torch.tensor([t], dtype=torch.float64, device="cuda")
        dist.all_reduce(x, op=dist.ReduceOp.MAX)
        t = float(x.item())
    ach = n * KECCAK_OPS / t
    return {"workload": "config-4 Keccak-256 of 64-byte key||slot preimages (HBM-resident)",
            "messages_per_launch_per_gpu": n, "value": world * n / t, "unit": "hashes/s",
            "kernel": "pf_keccak_fixed_kernel", "kernel_ms_avg": 1e3 * t,
            "roofline": {"bound": "valu", "achieved": ach / 1e12, "peak": INT32_PEAK_OPS / 1e12,
                         "unit": "Tops/s (int32)", "frac": ach / INT32_PEAK_OPS,
                         "hbm_GBps": n * KECCAK_BYTES / t / 1e9,
                         "valu_issue_frac": (n / 64) * KECCAK_VALU_PER_WAVE / t / VALU_ISSUE_PER_S,
                         # the same instructions priced at their measured issue costs at 8
                         # waves/SIMD (tools/movbench.hip, profiles/r04c_movbench.log: bitop3
                         # 2.76, alignbit 4.69 SIMD cycles) and the 2.25 GHz the dense loops
                         # run at — the rate this instruction mix can reach
                         "issue_frac_at_measured_rates": (n / 64) * KECCAK_CYCLES_PER_WAVE / (1024 * 2.25e9) / t,
                         "note": "frac prices 6,500 int32 ops per Keccak-f[1600] (SURVEY §8(d) "
                                 "table); valu_issue_frac is the hardware view: the 4,340 VALU "
                                 "instructions per wave the kernel issues over the SIMDs' issue "
                                 "slots (2 cycles per wave64 instruction at 2.4 GHz)"}}


def early_leg(args, eng, batch, torch, dist, first_id, cdev="cuda"):
    """SURVEY §8(d) config 3 asks for both sweeps: the same DAGs searched with ballot early
    exit and per-assert short-circuit on (the engine's production flags,
    pf_check_early_kernel).  Two launches:
    * ``unplanted`` — the timed batch itself: the search has to find a witness among the
      generated candidates; witness-free sets sweep the whole budget;
    * ``planted`` — the same DAG ids with their planted witness attached as the parent model
      (candidate 0 = the witness, SURVEY §8(d) "the planted candidate can be included"),
      so every set stops in its first wave: the engine's per-set verdict overhead.
    Reported per leg: candidates decided per second (a lane whose set is already false at an
    assert stops there), sets with a witness, set verdicts per second, kernel time."""
    from mythril_amd import ir, synth

    flags = ir.FLAG_EARLY_EXIT | ir.FLAG_SHORTCIRCUIT | ir.FLAG_COUNT_OPS
    planted = eng.upload([synth.random_dag_set(first_id + i, plant=True)[0] for i in range(args.sets)])
    out = {"flags": "early_exit|shortcircuit", "kernel": "pf_check_early_kernel"}
    for name, db in (("unplanted", batch), ("planted", planted)):
        eng.check(db, budget=args.budget, seed=args.seed, flags=flags)  # warm
        r = eng.check(db, budget=args.budget, seed=args.seed, flags=flags)
        vals = [float(r.cands_decided), r.kernel_ms / 1e3, float(int(r.sat.sum()))]
        if dist is not None:
            t = torch.tensor(vals, dtype=torch.float64, device=cdev)
            s_ = t[[0, 2]].clone()
            dist.all_reduce(s_, op=dist.ReduceOp.SUM)
            m_ = t[1:2].clone()
            dist.all_reduce(m_, op=dist.ReduceOp.MAX)
            vals = [float(s_[0]), float(m_[0]), float(s_[1])]
        n_sets = args.sets * (dist.get_world_size() if dist is not None else 1)
        out[name] = {"cands_decided_per_s": vals[0] / vals[1], "set_verdicts_per_s": n_sets / vals[1],
                     "sets_with_witness": int(vals[2]), "sets": n_sets, "kernel_ms": 1e3 * vals[1]}
    planted.free()
    return out


def pmc_traffic(args):
    """HBM bytes per launch of pf_check_kernel from the newest committed PMC summary
    (profiles/*_pmc.json, written by tools/pmc_summary.py from separate rocprofv3 --pmc
    FETCH_SIZE / WRITE_SIZE passes of this same default command) — None for other configs."""
    if (args.sets, args.budget, args.mode) != (1024, 65536, "full"):
        return None, None
    import glob
    files = sorted(glob.glob(os.path.join(os.path.dirname(os.path.abspath(__file__)), "profiles", "*_pmc.json")))
    if not files:
        return None, None
    with open(files[-1]) as f:
        d = json.load(f)
    return d, os.path.relpath(files[-1], os.path.dirname(os.path.abspath(__file__)))


# Issue cost of a wave64 VALU instruction by class, SIMD cycles at 4 waves/SIMD (the check
# kernel's occupancy), 16 independent instructions per wave (tools/movbench.hip,
# profiles/r04c_movbench.log, normalised at 2.4 GHz like the kernel time below): a simple
# 32-bit op (v_add_u32 2.95, v_mov 3.09, v_xor 2.89) costs ~3, not the 2 of the nominal
# issue rate; v_mad_u64_u32 5.13; f64 fma / cvt ~4.97 (v_mul_f64); v_rcp_f64 17.47.
VALU_COST_4W = {"simple": 2.95, "int64": 5.13, "fma_f64": 4.97, "cvt": 4.97, "trans_f64": 17.47}


def valu_view(pmc, kernel_s):
    """Hardware side of the roofline from the PMC summary: wave-level VALU instructions per
    launch (SQ_INSTS_VALU) over the SIMDs' VALU issue slots (a wave64 VALU instruction
    occupies its SIMD for 2 cycles; 1024 SIMDs, MI355X_MICROARCH.md "Wave scheduling"), at
    the effective clock of the PMC run (GRBM_GUI_ACTIVE / 8 XCDs) and, for reference, at
    2.4 GHz over the live kernel time.

    ``issue_frac_at_measured_rates`` prices the same instruction mix at the costs the
    microbenchmark measures for each class at 4 waves/SIMD (VALU_COST_4W: INT64 and the f64
    classes from their own PMC counters, every other VALU instruction at the simple-op cost —
    a lower bound, since carry chains, v_cndmask_e64 and 3-source ops cost 4.7-5.0) over
    1024 SIMDs x 2.4 GHz x the live kernel time.  At ~1 the SIMDs are issue-saturated by
    this mix: only fewer or cheaper instructions make the kernel faster."""
    if not pmc or "sq" not in pmc:
        return None
    v = pmc["sq"]["SQ_INSTS_VALU"]
    out = {"valu_instr_per_launch": v, "int64_instr_per_launch": pmc["sq"].get("SQ_INSTS_VALU_INT64"),
           "issue_frac_at_2400MHz": 2.0 * v / (1024 * 2.4e9 * kernel_s)}
    # the PMC workload is the default config (pmc_traffic): 1024 sets x 65,536 candidates =
    # 2^20 wave-level evaluations of a 64-candidate group
    out["valu_instr_per_eval_group"] = v / (1024 * 65536 / 64)
    f64 = pmc.get("f64") or {}
    i64 = pmc["sq"].get("SQ_INSTS_VALU_INT64")
    if i64 is not None and f64:
        fma = f64.get("SQ_INSTS_VALU_FMA_F64", 0.0) + f64.get("SQ_INSTS_VALU_MUL_F64", 0.0) + \
            f64.get("SQ_INSTS_VALU_ADD_F64", 0.0)
        cvt, trans = f64.get("SQ_INSTS_VALU_CVT", 0.0), f64.get("SQ_INSTS_VALU_TRANS_F64", 0.0)
        rest = max(0.0, v - i64 - fma - cvt - trans)
        cyc = (rest * VALU_COST_4W["simple"] + i64 * VALU_COST_4W["int64"] + fma * VALU_COST_4W["fma_f64"] +
               cvt * VALU_COST_4W["cvt"] + trans * VALU_COST_4W["trans_f64"])
        out["issue_frac_at_measured_rates"] = cyc / (1024 * 2.4e9 * kernel_s)
        out["measured_rates"] = dict(VALU_COST_4W, source="profiles/r04c_movbench.log (4 waves/SIMD)")
    clk = pmc.get("clk")
    if clk and clk.get("GRBM_GUI_ACTIVE"):
        cyc = clk["GRBM_GUI_ACTIVE"] / 8.0
        # both counts from the same PMC run: independent of this run's kernel time
        out["issue_frac_eff_clock"] = 2.0 * clk["SQ_INSTS_VALU"] / (1024 * cyc)
    return out


def main():
    args = parse()
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", str(args.gpus)))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    import torch

    dist = None
    if world > 1:
        import torch.distributed as dist_mod

        dist = dist_mod
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    line = run(args, rank, world, local, dist)
    if line is not None:
        print(json.dumps(line), flush=True)
    if dist is not None:
        # rank 0 spends a few seconds on the host-side legs: leave together
        dist.barrier()
        dist.destroy_process_group()


def run(args, rank, world, local, dist, engine=None, cdev="cuda"):
    """The bench body for one rank; returns rank 0's JSON line (None on other ranks).

    ``dist`` is torch.distributed with the process group already up (None at N = 1).  The
    engine and the collectives' device are parameters so that the multi-rank branch — the
    step-time max, the evals sum, the verdict all-gather, the early-exit reductions and
    rank 0's line — also runs in a CPU test under gloo with the oracle as the engine
    (tests/test_bench_dist.py), not first in the driver's SCALE run."""
    import torch

    from mythril_amd import _lib, ir, synth
    from mythril_amd.engine import Engine

    if args.lib:
        _lib.load_library(args.lib)

    eng = engine if engine is not None else Engine(local)
    flags = ir.FLAG_COUNT_OPS | (ir.FLAG_EARLY_EXIT | ir.FLAG_SHORTCIRCUIT if args.mode == "early" else 0)
    n_steps = args.warmup + args.steps
    batches, step_progs = [], []
    t_gen = time.perf_counter()
    for k in range(n_steps):
        first = (k * world + rank) * args.sets
        progs = synth.random_dag_programs(first, args.sets, plant=False)[0]
        step_progs.append(progs)
        batches.append(eng.upload(progs))
    t_gen = time.perf_counter() - t_gen

    def barrier():
        if cdev == "cuda":
            torch.cuda.synchronize()
        if dist is not None:
            dist.barrier()

    for k in range(args.warmup):
        eng.check(batches[k], budget=args.budget, seed=args.seed, flags=flags)
    barrier()
    t0 = time.perf_counter()
    evals = ops = 0
    kms = []
    founds = []
    # the K steps are enqueued back to back on the device stream (pf_check_batches) and read
    # afterwards — a stream of independent batches, as a batching caller would issue them —
    # so no host round trip sits between two steps' kernels (--serial-steps: one
    # pf_check_batch call per step, each waited for)
    if args.serial_steps:
        results = [eng.check(batches[k], budget=args.budget, seed=args.seed, flags=flags)
                   for k in range(args.warmup, n_steps)]
    else:
        results = eng.check_each(batches[args.warmup:n_steps], budget=args.budget, seed=args.seed,
                                 flags=flags)
    for r in results:
        evals += r.evals_full if args.mode == "full" else r.cands_decided
        ops += r.ops
        kms.append(r.kernel_ms)
        founds.append(r.found)
    barrier()
    dt = time.perf_counter() - t0

    tot_evals, max_dt = float(evals), dt
    if dist is not None:
        t = torch.tensor([float(evals), dt], dtype=torch.float64, device=cdev)
        ev = t[:1].clone()
        dist.all_reduce(ev, op=dist.ReduceOp.SUM)
        mx = t[1:].clone()
        dist.all_reduce(mx, op=dist.ReduceOp.MAX)
        tot_evals, max_dt = float(ev.item()), float(mx.item())
        # the path's one collective: all-gather the per-set SAT verdicts
        from mythril_amd.dist import gather_found

        mine = np.concatenate(founds)
        gathered = gather_found(mine, rank * len(mine), world * len(mine))

    # node evaluations of the timed steps: every instruction of every set runs for every
    # candidate in the full sweep (also report node-evals/s)
    nodes_per_step = [len(batches[k].batch.code) for k in range(args.warmup, n_steps)]
    tot_nodes = float(sum(nodes_per_step) * args.budget)
    if dist is not None:
        x = torch.tensor([tot_nodes], dtype=torch.float64, device=cdev)
        dist.all_reduce(x, op=dist.ReduceOp.SUM)
        tot_nodes = float(x.item())

    early = (early_leg(args, eng, batches[args.warmup], torch, dist, (args.warmup * world + rank) * args.sets,
                       cdev) if args.mode == "full" else None)
    kec = keccak_leg(args, torch, rank, world) if args.keccak_log2 > 0 else None

    # the SURVEY.md §8(d) op table's figure (prices EXP as 512 products and division as an
    # 8-digit schoolbook quotient, so its "achieved" can exceed the peak): kept as its own
    # field, computed on the host for the full sweep (every candidate runs every node)
    s8d = None
    if args.mode == "full":
        s8d_ops = float(sum(ir.op_cost_words(batches[k].batch.code) for k in range(args.warmup, n_steps))) * args.budget
        ks = sum(kms) / 1e3
        s8d = {"achieved": s8d_ops / ks / 1e12 if ks > 0 else 0.0,
               "frac": s8d_ops / ks / INT32_PEAK_OPS if ks > 0 else 0.0,
               "note": "SURVEY.md §8(d) per-op table (EXP 36,864, UDIV 256, SDIV 280); "
                       "not reachable-work pricing, so frac may exceed 1"}

    # the full pass on every rank (its own shard of the DAG ids), before rank 0's host legs
    fp = full_pass_leg(args, eng, rank, world, dist, cdev) if args.full_pass_dags > 0 else None

    if rank == 0:
        pmc, traffic_src = pmc_traffic(args)
        traffic = pmc.get("traffic_bytes") if pmc else None
        kernel_s = sum(kms) / 1e3
        achieved = ops / kernel_s if kernel_s > 0 else 0.0
        line = {
            "metric": "constraint-candidate evals/sec + % z3 queries discharged on-GPU",
            "value": tot_evals / max_dt,
            "unit": "evals/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": 1e3 * max_dt / args.steps,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u32 (256-bit as 8x32-bit limbs)",
            "data": "synthetic (config-3 random DAGs, on-device Philox candidates)",
            "config": {"workload": "synthetic-dags-depth32-muldivexp",
                       "sets_per_step_per_gpu": args.sets, "candidates_per_set": args.budget,
                       "mode": args.mode, "parallelism": f"sets sharded over {world} GPU(s)"},
            "roofline": {"bound": "valu", "achieved": achieved / 1e12,
                         "peak": INT32_PEAK_OPS / 1e12, "unit": "Tops/s (int32)",
                         "frac": achieved / INT32_PEAK_OPS, "traffic": traffic,
                         "traffic_unit": "bytes/launch", "traffic_source": traffic_src,
                         "kernel": "pf_check_kernel", "kernel_ms_avg": float(np.mean(kms)),
                         "op_table": "reachable (mythril_amd/ir.py _COST256_REACH: EXP 2,520, "
                                     "UDIV/UREM 96, SDIV/SREM/SMOD 120, MUL 72, HASH 120, "
                                     "cheap 8, shifts 16 int32 ops per 256-bit node)",
                         "s8d_table": s8d,
                         "hw": valu_view(pmc, float(np.mean(kms)) / 1e3)},
            "node_evals_per_s": tot_nodes / max_dt,
            "early_exit": early,
            "gen_upload_s": t_gen,
        }
        if args.keccak_log2 > 0:
            line["keccak"] = kec
            if pmc and "keccak" in pmc and args.keccak_log2 == 24:
                kec["roofline"]["traffic"] = pmc["keccak"]["traffic_bytes"]
                kec["roofline"]["traffic_unit"] = "bytes/launch (PMC)"
            if world == 1 and not args.no_cpu_baseline:
                sys.path.insert(0, os.path.join(ROOT, "oracle"))
                import coracle_py

                line["keccak"]["cpu_baseline"] = coracle_py.keccak_baseline(64, 5.0)
        if args.corpus_scenarios > 0:
            line["discharge"] = discharge(args)
        if args.quick_sat_queries > 0:
            line["quick_sat"] = quick_sat_leg(args)
        if fp is not None:
            line["full_pass"] = fp
        if world == 1 and not args.no_cpu_baseline:
            line["cpu_baseline"] = cpu_baseline(step_progs[args.warmup], args.budget, args.seed,
                                                args.cpu_sample_s)
        if dist is not None:
            line["verdicts_gathered"] = int(gathered.size)
            line["sets_with_witness"] = int((gathered != 0xFFFFFFFF).sum())
        return line
    return None


if __name__ == "__main__":
    main()
