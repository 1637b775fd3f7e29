"""Host-side driver of the batched path-feasibility engine (one process per GPU).

This is the layer the SMT facade (mythril_amd.smt.solver) and the LASER plugin call.  It
replaces the two CPU paths of the reference's query funnel with one GPU batch:

* ``ModelCache.check_quick_sat`` — evaluate the conjunction under candidate models
  (mythril/support/support_utils.py:57-71), here 65,536 generated candidates per set
  instead of <= 100 cached z3 models;
* the objective-free ``Optimize.check`` (mythril/support/model.py:37-59, :99-125) whenever a
  witness is found; sets without a witness are left to z3 unchanged (soundness).
"""

from __future__ import annotations

import ctypes
from dataclasses import dataclass
from typing import List, Optional, Sequence

import numpy as np

from . import _lib
from .ir import LIMBS, Batch, Program, from_limbs

NOT_FOUND = 0xFFFFFFFF


@dataclass
class CheckResult:
    found: np.ndarray        # [n_sets] uint32 smallest witness index or NOT_FOUND
    evals_full: int
    cands_decided: int
    ops: int
    kernel_ms: float
    timed_out: bool = False   # the device deadline cut the search: NOT_FOUND is incomplete

    @property
    def sat(self) -> np.ndarray:
        return self.found != NOT_FOUND


class DeviceBatch:
    """A :class:`~mythril_amd.ir.Batch` resident in one device's HBM (pf_batch_create_on)."""

    def __init__(self, batch: Batch, device: int = -1):
        L = _lib.lib()
        self.batch = batch
        self.device = device
        h = ctypes.c_uint64(0)
        descs = np.ascontiguousarray(batch.descs, dtype=np.uint32)
        code = np.ascontiguousarray(batch.code, dtype=np.uint32)
        consts = np.ascontiguousarray(batch.consts, dtype=np.uint32)
        schema = np.ascontiguousarray(batch.schema, dtype=np.uint32)
        parents = np.ascontiguousarray(batch.parents, dtype=np.uint32)
        _lib.check(L.pf_batch_create_on(
            device,
            _lib.ptr_u32(code.reshape(-1)) if code.size else None, code.shape[0],
            _lib.ptr_u32(consts.reshape(-1)) if consts.size else None, consts.shape[0],
            _lib.ptr_u32(schema.reshape(-1)) if schema.size else None, schema.shape[0],
            _lib.ptr_u32(parents.reshape(-1)) if parents.size else None, parents.shape[0],
            _lib.ptr_u32(descs.reshape(-1)) if descs.size else None, descs.shape[0],
            ctypes.byref(h)), "pf_batch_create_on")
        self.handle = h.value

    def __len__(self):
        return len(self.batch)

    def free(self):
        if self.handle:
            _lib.lib().pf_batch_free(self.handle)
            self.handle = 0

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


class Engine:
    """The per-process engine: one GPU (one process per GPU) or several GPUs driven by one
    process (``devices``), one library stream per device."""

    def __init__(self, device: int = 0, devices: Optional[Sequence[int]] = None):
        self.devices = list(devices) if devices is not None else [device]
        if len(set(self.devices)) < len(self.devices):
            # a device named twice: one execution context (own stream) per entry, so the
            # node split (upload_sharded + check_many) runs its multi-device path on one GPU
            self.devices = _lib.init_contexts(self.devices)
        else:
            _lib.init(self.devices)
        self.device = self.devices[0]

    # ---- search -------------------------------------------------------------------
    def upload(self, programs: Sequence[Program] | Batch, device: Optional[int] = None) -> DeviceBatch:
        batch = programs if isinstance(programs, Batch) else Batch(programs)
        return DeviceBatch(batch, self.device if device is None else device)

    def check(self, db: DeviceBatch, budget: int = 65536, seed: int = 0, flags: int = 2,
              timeout_ms: int = 0) -> CheckResult:
        n = len(db)
        found = np.full(max(n, 1), NOT_FOUND, dtype=np.uint32)
        st = _lib.pf_stats()
        _lib.check(_lib.lib().pf_check_batch(db.handle, seed, budget, flags, timeout_ms,
                                            _lib.ptr_u32(found), None, ctypes.byref(st)),
                   "pf_check_batch")
        return CheckResult(found[:n], st.evals_full, st.cands_decided, st.ops, st.kernel_ms,
                           bool(st.timed_out))

    def upload_sharded(self, programs: Sequence[Program]) -> List[DeviceBatch]:
        """Size-balanced contiguous shards, one per device (mythril_amd.dist.shard_bounds
        over the bytecode cost model), each uploaded to its device."""
        from .dist import shard_bounds

        progs = list(programs)
        nd = len(self.devices)
        if nd == 1 or len(progs) < 2:
            return [self.upload(progs)]
        out = []
        for (lo, hi), d in zip(shard_bounds([p.sched_cost() for p in progs], nd), self.devices):
            if hi > lo:
                out.append(self.upload(progs[lo:hi], device=d))
        return out

    def check_many(self, dbs: Sequence[DeviceBatch], budget: int = 65536, seed: int = 0,
                   flags: int = 2, timeout_ms: int = 0) -> CheckResult:
        """One search over several device batches at once (pf_check_batches: every device
        launches before any result is read); verdicts concatenated in batch order, the
        kernel time is the slowest device's."""
        if len(dbs) == 1:
            return self.check(dbs[0], budget, seed, flags, timeout_ms)
        n = sum(len(db) for db in dbs)
        found = np.full(max(n, 1), NOT_FOUND, dtype=np.uint32)
        stats = (_lib.pf_stats * len(dbs))()
        handles = np.array([db.handle for db in dbs], dtype=np.uint64)
        _lib.check(_lib.lib().pf_check_batches(_lib.ptr_u64(handles), len(dbs), seed, budget, flags,
                                              timeout_ms, _lib.ptr_u32(found), stats),
                   "pf_check_batches")
        return CheckResult(found[:n], sum(s.evals_full for s in stats),
                           sum(s.cands_decided for s in stats), sum(s.ops for s in stats),
                           max(s.kernel_ms for s in stats), any(s.timed_out for s in stats))

    def check_each(self, dbs: Sequence[DeviceBatch], budget: int = 65536, seed: int = 0,
                   flags: int = 2, timeout_ms: int = 0) -> List[CheckResult]:
        """check() of every batch, all enqueued before any result is read (pf_check_batches):
        batches on one device run back to back on its stream, with no host round trip
        between them (a stream of independent batches, e.g. bench steps)."""
        if not dbs:
            return []
        n = sum(len(db) for db in dbs)
        found = np.full(max(n, 1), NOT_FOUND, dtype=np.uint32)
        stats = (_lib.pf_stats * len(dbs))()
        handles = np.array([db.handle for db in dbs], dtype=np.uint64)
        _lib.check(_lib.lib().pf_check_batches(_lib.ptr_u64(handles), len(dbs), seed, budget, flags,
                                              timeout_ms, _lib.ptr_u32(found), stats),
                   "pf_check_batches")
        out, off = [], 0
        for db, s in zip(dbs, stats):
            out.append(CheckResult(found[off:off + len(db)].copy(), s.evals_full, s.cands_decided,
                                   s.ops, s.kernel_ms, bool(s.timed_out)))
            off += len(db)
        return out

    def materialize(self, db: DeviceBatch, set_ids: Sequence[int], cand_ids: Sequence[int],
                    seed: int = 0) -> List[List[int]]:
        """Concrete variable values of the given (set, candidate) pairs."""
        set_ids = np.ascontiguousarray(set_ids, dtype=np.uint32)
        cand_ids = np.ascontiguousarray(cand_ids, dtype=np.uint32)
        nv = [int(db.batch.descs[s][5]) for s in set_ids]
        total = sum(nv)
        out = np.zeros(max(total, 1) * LIMBS, dtype=np.uint32)
        if len(set_ids):
            _lib.check(_lib.lib().pf_materialize(db.handle, seed, _lib.ptr_u32(set_ids),
                                                _lib.ptr_u32(cand_ids), len(set_ids),
                                                _lib.ptr_u32(out)), "pf_materialize")
        res, off = [], 0
        rows = out.reshape(-1, LIMBS)
        for k in nv:
            res.append([from_limbs(rows[off + i]) for i in range(k)])
            off += k
        return res

    def materialize_limbs(self, db: DeviceBatch, set_ids: Sequence[int], cand_ids: Sequence[int],
                          seed: int = 0) -> np.ndarray:
        """materialize() as limbs: the variables of every (set, candidate) pair back to back,
        one row of 8 little-endian u32 each (rows = sum of the sets' variable counts)."""
        set_ids = np.ascontiguousarray(set_ids, dtype=np.uint32)
        cand_ids = np.ascontiguousarray(cand_ids, dtype=np.uint32)
        total = int(db.batch.descs[set_ids, 5].sum()) if len(set_ids) else 0
        out = np.zeros(max(total, 1) * LIMBS, dtype=np.uint32)
        if len(set_ids):
            _lib.check(_lib.lib().pf_materialize(db.handle, seed, _lib.ptr_u32(set_ids),
                                                _lib.ptr_u32(cand_ids), len(set_ids),
                                                _lib.ptr_u32(out)), "pf_materialize")
        return out[:total * LIMBS].reshape(total, LIMBS)

    def eval_assignments(self, db: DeviceBatch, set_id: int, soa: np.ndarray) -> np.ndarray:
        """SAT flag of each explicit candidate; soa is [var][limb][cand] uint32."""
        soa = np.ascontiguousarray(soa, dtype=np.uint32)
        n_cand = soa.shape[-1]
        out = np.zeros(max(n_cand, 1), dtype=np.uint8)
        _lib.check(_lib.lib().pf_eval_assignments(db.handle, set_id, _lib.ptr_u32(soa.reshape(-1)),
                                                 n_cand, _lib.ptr_u8(out)), "pf_eval_assignments")
        return out[:n_cand].astype(bool)

    def eval_program(self, program: Program, soa: np.ndarray) -> np.ndarray:
        """SAT flag of each explicit candidate of one program, in one call (pf_eval_program:
        no batch object; the GPU-resident ModelCache's launch).  The packed arrays are kept
        on the program, so a second launch over it packs nothing."""
        pk = getattr(program, "_eval_pack", None)
        if pk is None:
            b = Batch([program])
            pk = (np.ascontiguousarray(b.code, dtype=np.uint32).reshape(-1),
                  np.ascontiguousarray(b.consts, dtype=np.uint32).reshape(-1),
                  np.ascontiguousarray(b.schema, dtype=np.uint32).reshape(-1))
            program._eval_pack = pk
        code, consts, schema = pk
        soa = np.ascontiguousarray(soa, dtype=np.uint32)
        n_cand = soa.shape[-1]
        out = np.zeros(max(n_cand, 1), dtype=np.uint8)
        z = np.zeros(8, dtype=np.uint32)
        _lib.check(_lib.lib().pf_eval_program(
            self.device, _lib.ptr_u32(code), code.size // 4,
            _lib.ptr_u32(consts if consts.size else z), consts.size // 8,
            _lib.ptr_u32(schema if schema.size else z), schema.size // 4,
            _lib.ptr_u32(soa.reshape(-1)), n_cand, _lib.ptr_u8(out)), "pf_eval_program")
        return out[:n_cand].astype(bool)

    def eval_programs(self, pack, soa: np.ndarray) -> np.ndarray:
        """SAT flags [program][candidate] of several programs over one call's explicit
        candidates (pf_eval_programs: one launch, a wave per program and 64 candidates).
        ``pack`` = the flat (code, consts, schema, descs) u32 arrays of an ir.Batch over the
        programs; ``soa`` = [var][limb][cand] over all programs' variables, program after
        program (their descriptors' var_off)."""
        code, consts, schema, descs = pack
        n_sets = descs.size // 8
        soa = np.ascontiguousarray(soa, dtype=np.uint32)
        n_cand = soa.shape[-1]
        out = np.zeros(max(n_sets * n_cand, 1), dtype=np.uint8)
        z = np.zeros(8, dtype=np.uint32)
        _lib.check(_lib.lib().pf_eval_programs(
            self.device, _lib.ptr_u32(code), code.size // 4,
            _lib.ptr_u32(consts if consts.size else z), consts.size // 8,
            _lib.ptr_u32(schema if schema.size else z), schema.size // 4,
            _lib.ptr_u32(descs), n_sets,
            _lib.ptr_u32(soa.reshape(-1) if soa.size else z), n_cand, _lib.ptr_u8(out)), "pf_eval_programs")
        return out[:n_sets * n_cand].reshape(n_sets, n_cand).astype(bool)

    # ---- keccak -------------------------------------------------------------------
    def keccak256(self, messages: Sequence[bytes]) -> List[bytes]:
        n = len(messages)
        if n == 0:
            return []
        offsets = np.zeros(n + 1, dtype=np.uint64)
        offsets[1:] = np.cumsum([len(m) for m in messages], dtype=np.uint64)
        data = np.frombuffer(b"".join(messages) or b"\0", dtype=np.uint8).copy()
        out = np.zeros(32 * n, dtype=np.uint8)
        _lib.check(_lib.lib().pf_keccak256_batch(_lib.ptr_u8(data), _lib.ptr_u64(offsets), n,
                                                _lib.ptr_u8(out)), "pf_keccak256_batch")
        return [out[32 * i:32 * i + 32].tobytes() for i in range(n)]


_engine: Optional[Engine] = None


def get_engine(device: Optional[int] = None) -> Engine:
    """The process's engine.  Device selection: an explicit ``device``; else ``PF_DEVICES``
    (comma-separated indices, or ``all``: one process driving every visible GPU — the live
    analysis, which Mythril runs as one process; an index named twice, e.g. ``0,0``, makes two
    execution contexts on that GPU); else ``LOCAL_RANK`` (one process per GPU)."""
    global _engine
    if _engine is None:
        import os
        if device is not None:
            _engine = Engine(device)
        else:
            spec = os.environ.get("PF_DEVICES", "").strip()
            if spec == "all":
                _engine = Engine(devices=list(range(_lib.lib().pf_device_count())))
            elif spec:
                _engine = Engine(devices=[int(x) for x in spec.split(",")])
            else:
                _engine = Engine(int(os.environ.get("LOCAL_RANK", "0")))
    return _engine
