#!/usr/bin/env python3
"""Config 3 as specified: ONE full pass over the 1,000,000 synthetic DAGs
(depth 32, MUL/DIV/EXP-heavy mix, dag ids 0..999,999, DAG generator seed 20260101, candidate
seed 0x4D595448 ^ dag_id), 65,536 candidates each = 6.55e10 constraint-candidate evals.

The DAGs are generated and lowered on the host by a pool of worker processes (chunks of
`--chunk` DAGs; the engine never sees the host side), each chunk is uploaded and swept
(early exit off, like bench.py's timed steps) while the workers build the next chunks.
Reported: total kernel time, wall time, evals/s over the kernel time and over the wall time,
sets with a witness among the 65,536 candidates, and a planted early-exit pass over the same
DAG ids (witness attached as the parent model, so every set stops at candidate 0).

    python tools/full_pass.py [--dags 1000000] [--chunk 65536] [--workers 16]
"""

from __future__ import annotations

import argparse
import json
import os
import sys
import time
from concurrent.futures import ProcessPoolExecutor

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _build(args):
    """DAGs [first, first+n): packed arrays of the unplanted programs and of the same
    programs with their planted witness attached as the parent model (identical code) —
    natively generated when libpflower.so has pflt_synth (synth.random_dag_programs)."""
    first, n = args
    from mythril_amd import ir, synth

    out = []
    for plant in (False, True):
        progs, _ = synth.random_dag_programs(first, n, plant=plant)
        b = ir.Batch(progs)
        out.append((b.code, b.consts, b.schema, b.parents, b.descs))
    return first, n, out


def _arrays_batch(arrs, n):
    from mythril_amd import ir

    b = ir.Batch.__new__(ir.Batch)
    b.programs = [None] * n
    b.code, b.consts, b.schema, b.parents, b.descs = arrs
    return b


def run_full_pass(eng, dags: int = 1_000_000, chunk: int = 65536, piece: int = 2048, workers: int = 16,
                  budget: int = 65536, seed: int = 0, progress=None, mp_context=None, first: int = 0) -> dict:
    """The full pass over DAG ids [first, first + dags) on ``eng``; returns the result dict.  The host
    workers (``mp_context``: "spawn" when the caller has already initialised the GPU) build
    the packed batches while the device sweeps the previous chunk."""
    import multiprocessing as mp

    import numpy as np

    from mythril_amd import ir

    ctx = mp.get_context(mp_context) if mp_context else None
    pool = ProcessPoolExecutor(workers, mp_context=ctx)
    list(pool.map(_build, [(0, 1)] * workers))
    t_wall = time.perf_counter()
    res = {"dags": dags, "first_dag": first, "candidates_per_dag": budget,
           "seeds": "DAG generator 20260101 (Philox key (seed << 32) | dag_id), candidate key "
                    "0x4D595448 ^ dag_id (global seed 0)"}
    legs = {"full_sweep": (0, 0), "planted_early_exit": (1, ir.FLAG_EARLY_EXIT | ir.FLAG_SHORTCIRCUIT)}
    acc = {k: dict(kernel_ms=0.0, evals=0, decided=0, sat=0) for k in legs}
    chunks = 0
    t_wait = 0.0   # wall time the packing loop spent waiting for the host workers
    # the device runs on its own thread (the engine's calls release the GIL): chunk k is
    # uploaded and swept while this thread waits for and packs chunk k + 1
    import queue
    import threading

    # One uploader thread per leg: pf_batch_create's host half (checks, device program,
    # staging) runs outside the library lock, but its copy is queued behind the search in
    # progress (the runtime's H2D copy waits for the busy CUs) — one thread per leg keeps the
    # next chunk's host work from waiting behind the previous leg's blocked copy.
    todos = {leg: queue.Queue(maxsize=2) for leg in legs}
    readys = {leg: queue.Queue(maxsize=2) for leg in legs}
    errors: list = []
    t_upload = [0.0]

    def put_checked(q, item) -> bool:
        while not errors:
            try:
                q.put(item, timeout=0.5)
                return True
            except queue.Full:
                continue
        return False

    def upload_loop(leg, which):
        try:
            while True:
                item = todos[leg].get()
                if item is None:
                    break
                k, n, packed = item
                tu = time.perf_counter()
                db = eng.upload(_arrays_batch(packed[which], n))
                t_upload[0] += time.perf_counter() - tu
                if progress is not None:
                    progress({"upload": leg, "chunk": k, "t0": tu - t_wall, "t1": time.perf_counter() - t_wall})
                if not put_checked(readys[leg], (k, n, db)):
                    db.free()
                    break
        except Exception as e:  # noqa: BLE001 - reported by the packing thread
            errors.append(e)
        finally:
            readys[leg].put(None)   # the device loop drains until it sees this

    def drain():
        for leg in legs:
            while True:
                it = readys[leg].get()
                if it is None:
                    break
                it[2].free()

    def device_loop():
        while True:
            items = [readys[leg].get() for leg in legs]
            if any(it is None for it in items):
                for leg, it in zip(legs, items):
                    if it is not None:
                        it[2].free()
                        while readys[leg].get() is not None:
                            pass
                return
            try:
                for (leg, (which, flags)), (k, n, db) in zip(legs.items(), items):
                    tc = time.perf_counter()
                    r = eng.check(db, budget=budget, seed=seed, flags=flags)
                    tc1 = time.perf_counter()
                    db.free()
                    a = acc[leg]
                    a["kernel_ms"] += r.kernel_ms
                    a["evals"] += r.evals_full
                    a["decided"] += r.cands_decided
                    a["sat"] += int(r.sat.sum())
                    if progress is not None:
                        progress({"leg": leg, "chunk": k, "sets": n, "kernel_ms": r.kernel_ms,
                                  "sat": int(r.sat.sum()), "t0": tc - t_wall, "t1": tc1 - t_wall})
            except Exception as e:  # noqa: BLE001 - reported by the packing thread
                errors.append(e)
                for _, _, db in items:
                    db.free()
                drain()
                return

    ups = [threading.Thread(target=upload_loop, args=(leg, which), daemon=True) for leg, (which, _) in legs.items()]
    for t in ups:
        t.start()
    dev = threading.Thread(target=device_loop, daemon=True)
    dev.start()
    with pool:
        tasks = [(first + f, min(piece, dags - f)) for f in range(0, dags, piece)]
        futs = [pool.submit(_build, t) for t in tasks]
        pending, n_pending = [], 0
        # the first chunks ramp up (chunk / 32, / 16, ... then chunk): the device starts after
        # one piece is built instead of a whole chunk's worth
        target = max(piece, chunk // 32)
        for i, fu in enumerate(futs):
            tw = time.perf_counter()
            pending.append(fu.result())
            t_wait += time.perf_counter() - tw
            if progress is not None and i + 1 == len(futs):
                progress({"built_all": time.perf_counter() - t_wall})
            n_pending += pending[-1][1]
            if n_pending < target and i + 1 < len(futs):
                continue
            target = min(chunk, 2 * target)
            chunks += 1
            packed = []
            for which in (0, 1):
                codes, consts, schemas, parents, descs = [], [], [], [], []
                oc = ok = os_ = op = 0
                for (_, nn, both) in pending:
                    c, k, s_, p, d = both[which]
                    d = d.copy()
                    d[:, 0] += oc
                    d[:, 2] += ok
                    d[:, 4] += os_
                    has = d[:, 7] != ir.NO_PARENT
                    d[has, 7] += op
                    s_ = s_.copy()   # schema parent slots are absolute parent indices
                    sp = s_[:, 3] != ir.NO_PARENT
                    s_[sp, 3] += op
                    codes.append(c); consts.append(k); schemas.append(s_); parents.append(p); descs.append(d)
                    oc += len(c); ok += len(k); os_ += len(s_); op += len(p)
                packed.append(tuple(np.concatenate(x) for x in (codes, consts, schemas, parents, descs)))
            if not all(put_checked(todos[leg], (chunks, n_pending, packed)) for leg in legs):
                break
            pending, n_pending = [], 0
    for leg, t in zip(legs, ups):
        while t.is_alive():
            try:
                todos[leg].put(None, timeout=0.5)
                break
            except queue.Full:
                continue
    for t in ups:
        t.join()
    dev.join()
    if errors:
        raise errors[0]
    for leg, a in acc.items():
        ks = a["kernel_ms"] / 1e3
        units = a["evals"] if leg == "full_sweep" else a["decided"]
        res[leg] = {"kernel_s": ks, "chunks": chunks, "evals_full": a["evals"],
                    "cands_decided": a["decided"], "sets_with_witness": a["sat"],
                    "evals_per_s_kernel": units / ks if ks else None,
                    "set_verdicts_per_s_kernel": dags / ks if ks else None}
    res["total_wall_s"] = time.perf_counter() - t_wall
    res["host_wait_s"] = t_wait
    res["upload_s"] = t_upload[0]   # pf_batch_create calls, overlapped with the searches
    res["host_workers"] = workers
    res["full_sweep"]["evals_per_s_wall"] = res["full_sweep"]["evals_full"] / res["total_wall_s"]
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dags", type=int, default=1_000_000)
    ap.add_argument("--chunk", type=int, default=65536)
    ap.add_argument("--piece", type=int, default=2048, help="DAGs per worker task")
    ap.add_argument("--workers", type=int, default=16)
    ap.add_argument("--budget", type=int, default=65536)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--out", default=None)
    args = ap.parse_args()

    from mythril_amd.engine import Engine

    # the workers are started (spawned) by run_full_pass; this process owns the GPU
    eng = Engine(0)
    import threading

    plock = threading.Lock()   # progress comes from the device and uploader threads

    def progress(d):
        with plock:
            print(json.dumps(d), flush=True)

    res = run_full_pass(eng, args.dags, args.chunk, args.piece, args.workers, args.budget, args.seed,
                        progress=progress, mp_context="spawn")
    line = json.dumps(res)
    print(line, flush=True)
    if args.out:
        with open(args.out, "w") as f:
            f.write(line + "\n")


if __name__ == "__main__":
    main()
