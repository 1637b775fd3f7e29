"""Native term lowering: constraint terms -> program in libpflower.so (include/pf_lower.h).

The Python lowering (to_dag.TermLowering -> seed.apply_hints -> lower.lower) stays the
reference; this module hands the same bucket to the C++ port (csrc/pf_terms.cpp) and
rebuilds the host-side witness metadata (Lowered.var_terms / uf_apps / array_reads) from the
ids it returns, so ``gpu_check`` receives exactly what the Python path produces
(tests/test_native_terms.py compares node tables, variables, metadata and programs).

Terms are hash-consed and immortal (terms.Term._table), so each enters the native store once:
a per-process map Term -> store id, filled children-first on first use.  A lowering worker
process has its own store.
"""

from __future__ import annotations

import ctypes
import threading
from typing import Dict, List, Optional, Tuple

import numpy as np

from .. import ir
from ..lower import LoweringError, _native
from . import terms as T
from .to_dag import Lowered, UFRegistry

_OPS = {
    "bv": 1, "true": 2, "false": 3, "var": 4, "bvar": 5, "array": 6, "K": 7, "select": 8,
    "store": 9, "apply": 10, "extract": 11, "concat": 12, "zero_extend": 13, "ite": 14,
    "=": 15, "iff": 16, "and": 17, "or": 18, "not": 19, "xor": 20, "bvnot": 21, "bvneg": 22,
    "bvadd": 30, "bvsub": 31, "bvmul": 32, "bvudiv": 33, "bvurem": 34, "bvsdiv": 35,
    "bvsrem": 36, "bvsmod": 37, "bvand": 38, "bvor": 39, "bvxor": 40, "bvshl": 41,
    "bvlshr": 42, "bvashr": 43, "bvexp": 44,
    "bvult": 50, "bvule": 51, "bvslt": 52, "bvsle": 53, "bvuadd_noovfl": 54, "bvumul_noovfl": 55,
}
OTHER = 99
HINTS, PROGRAM, EXPLICIT = 1, 2, 4
GET_VARS, GET_VAR_TERMS, GET_UF_APPS, GET_READS, GET_CODE, GET_CONSTS, GET_NODES, GET_POOL, \
    GET_ROOTS, GET_FORCED, GET_IN_ROOTS = range(11)
VT_TERM, VT_SELECT, VT_EXTRACT = 0, 1, 2

_u32p = ctypes.POINTER(ctypes.c_uint32)
_U32_1, _U8_1, _I8_1 = ctypes.c_uint32 * 1, ctypes.c_uint8 * 1, ctypes.c_int8 * 1


# Pointer arguments: a one-element ctypes array over the numpy buffer (from_buffer) passes its
# address as T* for about a third of ndarray.ctypes.data_as's cost, which builds numpy's
# _ctypes helper on every call (a single query makes ~30 of these calls).  Read-only, empty
# and non-contiguous arrays take data_as.
def _p32(a: np.ndarray):
    try:
        return _U32_1.from_buffer(a)
    except (TypeError, ValueError):
        return a.ctypes.data_as(_u32p)


def _p8(a: np.ndarray):
    try:
        return _U8_1.from_buffer(a)
    except (TypeError, ValueError):
        return a.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8))


def _pi8(a: np.ndarray):
    try:
        return _I8_1.from_buffer(a)
    except (TypeError, ValueError):
        return a.ctypes.data_as(ctypes.POINTER(ctypes.c_int8))


def _limbs_of(v: int) -> List[int]:
    out = []
    while v:
        out.append(v & 0xFFFFFFFF)
        v >>= 32
    return out or [0]


def _limbs8(v: int) -> List[int]:
    v &= (1 << 256) - 1
    return [(v >> (32 * i)) & 0xFFFFFFFF for i in range(8)]


def _int_of(row) -> int:
    if isinstance(row, np.ndarray):
        return int.from_bytes(row.astype("<u4").tobytes(), "little")
    return sum(int(x) << (32 * i) for i, x in enumerate(row))


_SIGNED = False


def _bind(L):
    global _SIGNED
    if _SIGNED:
        return
    L.pflt_store_new.restype = ctypes.c_void_p
    L.pflt_store_free.argtypes = [ctypes.c_void_p]
    L.pflt_store_size.restype = ctypes.c_size_t
    L.pflt_store_size.argtypes = [ctypes.c_void_p]
    L.pflt_add.restype = ctypes.c_int64
    L.pflt_add.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32,
                           ctypes.c_uint32, _u32p, ctypes.c_uint32, ctypes.c_int64, ctypes.c_int64,
                           _u32p, ctypes.c_uint32, ctypes.c_char_p]
    L.pflt_lower.restype = ctypes.c_void_p
    L.pflt_lower.argtypes = [ctypes.c_void_p, _u32p, ctypes.c_size_t, _u32p, ctypes.c_size_t,
                             ctypes.c_char_p, _u32p, ctypes.c_size_t, _u32p, _u32p, ctypes.c_size_t,
                             ctypes.c_uint32, ctypes.c_uint32, ctypes.POINTER(ctypes.c_int)]
    L.pflt_last_error.restype = ctypes.c_char_p
    L.pflt_result_free.argtypes = [ctypes.c_void_p]
    L.pflt_result_info.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint64)]
    L.pflt_result_get.argtypes = [ctypes.c_void_p, ctypes.c_uint32, _u32p, ctypes.c_char_p]
    if hasattr(L, "pflt_result_candidate0"):
        L.pflt_result_candidate0.argtypes = [ctypes.c_void_p, _u32p]
        L.pflt_result_candidate0.restype = ctypes.c_int
    if hasattr(L, "pflt_lower_many"):
        vp, sz, u32 = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint32
        L.pflt_parent_new.restype = vp
        L.pflt_parent_new.argtypes = [ctypes.c_char_p, _u32p, sz, _u32p, _u32p, sz]
        L.pflt_parent_free.argtypes = [vp]
        L.pflt_parent_info.argtypes = [vp, ctypes.POINTER(ctypes.c_uint64)]
        L.pflt_parent_get.argtypes = [vp, ctypes.c_char_p, _u32p, _u32p, _u32p]
        L.pflt_recent_clear.argtypes = [vp]
        L.pflt_note_vars.argtypes = [vp, ctypes.c_char_p, _u32p, sz, sz]
        L.pflt_note_result.argtypes = [vp, vp, _u32p, sz]
        L.pflt_recent_parent.restype = vp
        L.pflt_recent_parent.argtypes = [vp, _u32p, sz]
        L.pflt_lower_many.argtypes = [vp, vp, sz, _u32p, sz, u32, ctypes.POINTER(vp)]
        L.pflt_result_status.argtypes = [vp]
        L.pflt_result_error.restype = ctypes.c_char_p
        L.pflt_result_error.argtypes = [vp]
        L.pflt_result_shrink.argtypes = [vp]
        if hasattr(L, "pflt_result_info_many"):
            L.pflt_result_info_many.argtypes = [ctypes.POINTER(vp), sz, ctypes.POINTER(ctypes.c_uint64)]
        L.pflt_pack_sizes.argtypes = [ctypes.POINTER(vp), sz, ctypes.POINTER(ctypes.c_uint64)]
        L.pflt_pack_batch.argtypes = [ctypes.POINTER(vp), sz, _u32p, _u32p, u32, _u32p, _u32p, _u32p, _u32p, _u32p]
        L.pflt_recheck_many.argtypes = [vp, ctypes.POINTER(vp), sz, _u32p, _u32p, sz, u32,
                                        ctypes.POINTER(ctypes.c_int8)]
    if hasattr(L, "pflt_witness_new"):
        vp, sz, u32, u64 = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint32, ctypes.c_uint64
        L.pflt_witness_new.restype = vp
        L.pflt_witness_new.argtypes = [vp, ctypes.POINTER(vp), sz, _u32p, _u32p, sz, u64]
        L.pflt_witness_free.argtypes = [vp]
        L.pflt_witness_values.argtypes = [ctypes.POINTER(vp), sz, _u32p, sz, _u32p, u64, _u32p, sz, u64, u32,
                                          _u32p, ctypes.POINTER(ctypes.c_uint8)]
    _SIGNED = True


class TermStore:
    """The process's native term store (one per process; terms enter once)."""

    def __init__(self, lib):
        _bind(lib)
        self.L = lib
        self.h = lib.pflt_store_new()
        self.ids: Dict[T.Term, int] = {}
        self.terms: List[T.Term] = []
        # (array id, index id) -> select term: var_terms' base-array reads, built once per
        # store (the quick-sat leaves of successive queries repeat most of them)
        self.selects: Dict[Tuple[int, int], T.Term] = {}
        # guards Store::t and the recent tables: pflt_add (export) may reallocate the term
        # vector that a concurrent recheck / recent-parent / lowering reads through pointers
        # (ctypes drops the GIL), so every call into the store holds it
        self.lock = threading.RLock()

    def __del__(self):
        # the C++ store goes with the last reference: results keep their own TermStore
        # (``_Result.st``), so a retired generation lives until its results are gone
        try:
            self.L.pflt_store_free(self.h)
        except Exception:  # noqa: BLE001
            pass

    def export_many(self, terms) -> List[int]:
        """Store ids of ``terms`` (export each): the stored ones by one C-level dict pass —
        a query exports its conjuncts several times (buckets, parents, lowering)."""
        out = list(map(self.ids.get, terms))
        if None in out:
            out = [i if i is not None else self.export(t) for i, t in zip(out, terms)]
        return out

    def export(self, root: T.Term) -> int:
        """Store id of ``root``, adding it and every new subterm (children first)."""
        nid = self.ids.get(root)
        if nid is not None:
            return nid
        ids, L, h = self.ids, self.L, self.h
        stack = [(root, False)]
        while stack:
            t, expanded = stack.pop()
            if t in ids:
                continue
            if not expanded:
                stack.append((t, True))
                for a in reversed(t.args):
                    if a not in ids:
                        stack.append((a, False))
                continue
            op = _OPS.get(t.op, OTHER)
            s = t.sort
            if s == T.BOOL:
                sk, w1, w2 = 0, 0, 0
            elif s[0] == "bv":
                sk, w1, w2 = 1, s[1], 0
            else:
                sk, w1, w2 = 2, s[1], s[2]
            args = (ctypes.c_uint32 * max(len(t.args), 1))(*[ids[a] for a in t.args])
            i0 = i1 = 0
            limbs = None
            nl = 0
            name = None
            v = t.val
            if op == 1:
                ls = _limbs_of(v)
                limbs, nl = (ctypes.c_uint32 * len(ls))(*ls), len(ls)
            elif op in (4, 5, 6):
                name = v.encode()
            elif op == 10:
                name = v[0].encode()
            elif op == 11:
                i0, i1 = v
            elif op == 13:
                i0 = v
            elif op == OTHER:
                name = t.op.encode()
            nid = L.pflt_add(h, op, sk, w1, w2, args, len(t.args), i0, i1, limbs, nl, name)
            if nid < 0:
                raise ValueError(L.pflt_last_error().decode(errors="replace"))
            ids[t] = nid
            self.terms.append(t)
        return ids[root]


_STORE: Optional[TermStore] = None
_STORE_LOCK = threading.Lock()


def store() -> Optional[TermStore]:
    """The process's store, or None when libpflower.so is not built."""
    global _STORE
    if _STORE is None:
        L = _native()
        if not L or not hasattr(L, "pflt_store_new"):
            return None
        with _STORE_LOCK:
            if _STORE is None:
                _STORE = TermStore(L)
    return _STORE


def synth_programs(first_id: int, n: int, plant: bool, cdf) -> Optional[Tuple[list, np.ndarray, np.ndarray]]:
    """Config-3 DAG programs first_id .. first_id + n - 1 natively (pflt_synth: the programs of
    synth.random_dag_set bit for bit), as NativePrograms, with the planted witnesses (n x 8 x 8
    u32 limbs) and variable counts; None when libpflower.so lacks it."""
    st = store()
    if st is None or not hasattr(st.L, "pflt_synth") or not (_features(st) & 2):
        return None
    L = st.L
    if not getattr(L, "_synth_bound", False):
        L.pflt_synth.restype = ctypes.c_int
        L.pflt_synth.argtypes = [ctypes.c_uint32, ctypes.c_size_t, ctypes.c_uint32,
                                 ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_void_p), _u32p, _u32p]
        L._synth_bound = True
    hs = (ctypes.c_void_p * max(n, 1))()
    wit = np.zeros((max(n, 1), 8, 8), dtype=np.uint32)
    nv = np.zeros(max(n, 1), dtype=np.uint32)
    c = np.ascontiguousarray(cdf, dtype=np.float64)
    rc = L.pflt_synth(first_id, n, 1 if plant else 0, c.ctypes.data_as(ctypes.POINTER(ctypes.c_double)), hs,
                      _p32(wit), _p32(nv))
    results = [_Result(st, hs[i]) for i in range(n) if hs[i]]
    if rc != 0:
        raise ValueError(L.pflt_last_error().decode(errors="replace"))
    progs = []
    for i, r in enumerate(results):
        p = NativeProgram(r, (0x4D595448 ^ (first_id + i)) & 0xFFFFFFFF)
        p.name = f"dag{first_id + i}"
        progs.append(p)
    return progs, wit[:n], nv[:n]


def _features(st) -> int:
    if not hasattr(st.L, "pflt_features"):
        return 0
    st.L.pflt_features.restype = ctypes.c_uint32
    return int(st.L.pflt_features())


def has_explicit() -> bool:
    """Whether libpflower.so has the explicit-model lowering (PFLT_EXPLICIT)."""
    st = store()
    if st is None or not hasattr(st.L, "pflt_features"):
        return False
    st.L.pflt_features.restype = ctypes.c_uint32
    return bool(st.L.pflt_features() & 1)


_BLOBS: Dict[tuple, np.ndarray] = {}


def new_generation(limit: int) -> bool:
    """Retire the process's store once it holds ``limit`` terms or more (over a
    long ``myth analyze`` every term ever exported stays in it).  The next export starts a
    fresh store; results lowered from the old one keep it alive through ``_Result.st`` and
    are re-checked / recorded against it, never against the new one.  The caller drops its
    caches of such results (gpu_check.check_sets: reset_cache).  True if retired."""
    global _STORE
    st = _STORE
    if st is None or len(st.terms) < limit:
        return False
    with _STORE_LOCK:
        if _STORE is not st:
            return False
        _STORE = TermStore(st.L)
    return True


def _registry_blob(reg: UFRegistry) -> np.ndarray:
    """The registry in pflt_lower's layout, cached per registry state (hashes only get added:
    the per-width counts and interval starts identify the state)."""
    return _registry_blob_serial(reg)[0]


_BLOB_SERIAL = [0]


def _registry_blob_serial(reg: UFRegistry):
    """(blob, serial): the serial is new for every blob built, so a native witness re-parses
    its hash specs exactly when the registry's state moved (pflt_witness_values)."""
    key = (id(reg), tuple(reg.actors),
           tuple((n, s.lo, len(s.concrete)) for n, s in reg.keccak.items()))
    ent = _BLOBS.get(key)
    if ent is None:
        if len(_BLOBS) > 64:
            _BLOBS.clear()
        _BLOB_SERIAL[0] += 1
        ent = _BLOBS[key] = (_registry_blob_build(reg), _BLOB_SERIAL[0])
    return ent


def _registry_blob_build(reg: UFRegistry) -> np.ndarray:
    blob: List[int] = [len(reg.actors)]
    for a in reg.actors:
        blob += _limbs8(a)
    blob.append(len(reg.keccak))
    for n, spec in reg.keccak.items():
        blob += [n, 1 if spec.lo is not None else 0]
        blob += _limbs8(spec.base if spec.lo is not None else 0)
        blob.append(len(spec.concrete))
        nl = (n + 31) // 32
        for c, dg in spec.concrete.items():
            c &= (1 << n) - 1
            blob += [(c >> (32 * i)) & 0xFFFFFFFF for i in range(nl)]
            blob += _limbs8(dg)
    return np.array(blob, dtype=np.uint32)


class _Result:
    """One pflt_lower result: the program, the variables and the witness metadata."""

    def __init__(self, st: TermStore, h, info: Optional[List[int]] = None):
        self.st, self.h = st, h
        if info is None:
            buf = (ctypes.c_uint64 * 17)()
            st.L.pflt_result_info(h, buf)
            info = [int(x) for x in buf]
        self.info = info

    def __del__(self):
        try:
            self.st.L.pflt_result_free(self.h)
        except Exception:  # noqa: BLE001
            pass

    def get(self, which: int, n: int, cols: int) -> np.ndarray:
        out = np.zeros(max(n * cols, 1), dtype=np.uint32)
        self.st.L.pflt_result_get(self.h, which, _p32(out), None)
        return out[:n * cols].reshape(n, cols) if cols > 1 else out[:n]

    def variables(self) -> List[ir.Var]:
        nv, nb = self.info[0], self.info[1]
        out = np.zeros(max(nv * 13, 1), dtype=np.uint32)
        names = ctypes.create_string_buffer(max(nb, 1))
        self.st.L.pflt_result_get(self.h, GET_VARS, _p32(out), names)
        labels = names.raw[:nb].split(b"\0")[:nv]
        rows = out[:13 * nv].reshape(nv, 13)
        pbytes = np.ascontiguousarray(rows[:, 5:13]).astype("<u4").tobytes()
        head = rows[:, :5].tolist()
        vs = []
        for i in range(nv):
            w_, k_, h0, h1, hp = head[i]
            parent = int.from_bytes(pbytes[32 * i:32 * i + 32], "little") if hp else None
            vs.append(ir.Var(labels[i].decode(), w_, k_, h0, h1, parent))
        return vs

    def var_terms(self) -> List[T.Term]:
        """The variables' terms alone (the explicit lowering's leaves)."""
        terms = self.st.terms
        out = []
        for typ, a, b, c in self.get(GET_VAR_TERMS, self.info[2], 4).tolist():
            if typ == VT_TERM:
                out.append(terms[a])
            elif typ == VT_SELECT:
                out.append(self._select(a, b))
            else:
                out.append(T.extract(c, b, terms[a]))
        return out

    def _select(self, a: int, b: int) -> T.Term:
        sel = self.st.selects
        t = sel.get((a, b))
        if t is None:
            terms = self.st.terms
            t = sel[(a, b)] = T.select(terms[a], terms[b])
        return t

    def lowered(self) -> Lowered:
        terms = self.st.terms
        vt = self.get(GET_VAR_TERMS, self.info[2], 4)
        var_terms = []
        for typ, a, b, c in vt.tolist():
            if typ == VT_TERM:
                var_terms.append(terms[a])
            elif typ == VT_SELECT:
                var_terms.append(self._select(a, b))
            else:
                var_terms.append(T.extract(c, b, terms[a]))
        uf_apps = []
        for a in self.get(GET_UF_APPS, self.info[3], 1).tolist():
            t = terms[a]
            uf_apps.append((t.val[0], t.args, t))
        na, nr = self.info[4], self.info[5]
        raw = self.get(GET_READS, na + 2 * nr, 1).tolist()
        counts, pairs = raw[:na], raw[na:]
        reads: Dict[str, list] = {}
        k = 0
        for cnt in counts:
            for _ in range(cnt):
                a, b = pairs[2 * k], pairs[2 * k + 1]
                reads.setdefault(terms[a].val, []).append((terms[b], self._select(a, b)))
                k += 1
        return Lowered(None, var_terms, uf_apps, reads)

    def program(self, seed: int) -> ir.PackedProgram:
        code = self.get(GET_CODE, self.info[6], 4)
        nc = self.info[7]
        raw = self.get(GET_CONSTS, nc, 8).astype("<u4").tobytes()
        consts = [int.from_bytes(raw[32 * i:32 * i + 32], "little") for i in range(nc)]
        return ir.PackedProgram(code.copy(), consts, self.variables(), seed, "")


def _parent_args(st: TermStore, parent: Optional[dict]):
    names: List[bytes] = []
    nvals: List[int] = []
    reads: List[int] = []
    rvals: List[int] = []
    for k, v in (parent or {}).items():
        if v is None:
            continue
        if isinstance(k, str):
            names.append(k.encode())
            ls = _limbs_of(int(v))
            nvals += [len(ls)] + ls
        elif isinstance(k, T.Term) and k.op == "select":
            reads += [st.export(k.args[0]), st.export(k.args[1])]
            rvals += _limbs8(int(v))
    blob = b"\0".join(names) + b"\0"
    return (blob, np.array(nvals or [0], dtype=np.uint32), len(names),
            np.array(reads or [0], dtype=np.uint32), np.array(rvals or [0], dtype=np.uint32), len(reads) // 2)


def lower_native(bucket: List[T.Term], reg: UFRegistry, parent: Optional[dict], flags: int,
                 seed: int = 0) -> _Result:
    """pflt_lower over the bucket's conjuncts; raises LoweringError like the Python path."""
    st = store()
    if st is None:
        raise RuntimeError("libpflower.so without the term store")
    with st.lock:
        roots = np.array(st.export_many(bucket) or [0], dtype=np.uint32)
        regb = _registry_blob(reg)
        pn, pnv, npn, pr, prv, npr = _parent_args(st, parent)
        rc = ctypes.c_int(0)
        h = st.L.pflt_lower(st.h, _p32(roots), len(bucket), _p32(regb),
                            len(regb), pn, _p32(pnv), npn, _p32(pr),
                            _p32(prv), npr, flags, seed & 0xFFFFFFFF, ctypes.byref(rc))
        if not h:
            msg = st.L.pflt_last_error().decode(errors="replace")
            if rc.value == -2:
                raise LoweringError(msg)
            raise ValueError(f"pflt_lower failed ({rc.value}): {msg}")
        return _Result(st, h)


def lower_bucket(bucket: List[T.Term], reg: UFRegistry, parent: Optional[dict], hints: bool,
                 seed: int) -> Tuple[Lowered, ir.PackedProgram]:
    """gpu_check._lower_bucket natively: (witness metadata, program)."""
    r = lower_native(bucket, reg, parent, PROGRAM | (HINTS if hints else 0), seed)
    return r.lowered(), r.program(seed)


def recheck(bucket: List[T.Term], lo: Lowered, values: List[int], reg: UFRegistry) -> Optional[bool]:
    """The host re-check of a bucket witness natively (pflt_recheck, csrc/pf_recheck.cpp):
    every conjunct true under the witness (interp.Witness's interpretation).  None when the
    library cannot evaluate some term (the caller re-checks in Python)."""
    st = store()
    if st is None or not hasattr(st.L, "pflt_recheck"):
        return None
    L = st.L
    if not getattr(L, "_recheck_bound", False):
        L.pflt_recheck.restype = ctypes.c_int
        L.pflt_recheck.argtypes = [ctypes.c_void_p, _u32p, ctypes.c_size_t, _u32p, _u32p, ctypes.c_size_t,
                                   _u32p, ctypes.c_size_t, _u32p, ctypes.c_size_t, _u32p, ctypes.c_size_t,
                                   ctypes.POINTER(ctypes.c_uint8)]
        L._recheck_bound = True
    with st.lock:
        ex = st.export
        desc: List[int] = []
        for t in lo.var_terms:
            if t.op == "select":
                desc += [VT_SELECT, ex(t.args[0]), ex(t.args[1]), 0]
            elif t.op == "extract" and t.args[0].op == "var":
                desc += [VT_EXTRACT, ex(t.args[0]), t.val[1], t.val[0]]
            else:
                desc += [VT_TERM, ex(t), 0, 0]
        vals = np.frombuffer(b"".join(((v or 0) & ((1 << 256) - 1)).to_bytes(32, "little") for v in values)
                             or b"\0" * 32, dtype="<u4").astype(np.uint32)
        ufs = [ex(app) for _, _, app in lo.uf_apps]
        reads: List[int] = []
        for entries in lo.array_reads.values():
            for idx, sel in entries:
                reads += [ex(sel.args[0]), ex(idx)]
        roots = [ex(c) for c in bucket]
        a = lambda xs: np.array(xs or [0], dtype=np.uint32)  # noqa: E731
        d_, u_, r_, ro_ = a(desc), a(ufs), a(reads), a(roots)
        regb = _registry_blob(reg)
        out = np.zeros(max(len(roots), 1), dtype=np.uint8)
        rc = L.pflt_recheck(st.h, _p32(d_), len(lo.var_terms), _p32(vals),
                            _p32(u_), len(ufs), _p32(r_), len(reads) // 2,
                            _p32(regb), len(regb), _p32(ro_), len(roots),
                            _p8(out))
    if rc != 0:
        return None
    return bool(out[:len(roots)].all())


def buckets(constraints: List[T.Term]) -> Optional[List[List[T.Term]]]:
    """independence.buckets natively (pflt_buckets: the same partition and order, keys
    memoised per stored term); None when the library lacks it."""
    st = store()
    if st is None or not hasattr(st.L, "pflt_buckets"):
        return None
    L = st.L
    if not getattr(L, "_buckets_bound", False):
        L.pflt_buckets.restype = ctypes.c_int64
        L.pflt_buckets.argtypes = [ctypes.c_void_p, _u32p, ctypes.c_size_t, _u32p, ctypes.c_size_t,
                                   _u32p, ctypes.c_size_t]
        L._buckets_bound = True
    with st.lock:
        roots = np.array(st.export_many(constraints) or [0], dtype=np.uint32)
        cap = 4 * len(constraints) + 256
        while True:
            ids = np.zeros(cap, dtype=np.uint32)
            sizes = np.zeros(cap, dtype=np.uint32)
            nb = L.pflt_buckets(st.h, _p32(roots), len(constraints), _p32(ids),
                                cap, _p32(sizes), cap)
            if nb != -1:
                break
            cap *= 4
        if nb < 0:
            return None
        terms = st.terms
        out, o = [], 0
        idl = ids.tolist()
        for n in sizes[:nb].tolist():
            out.append([terms[i] for i in idl[o:o + n]])
            o += n
        return out


def buckets_many(queries: List[List[T.Term]]) -> Optional[List[List[List[T.Term]]]]:
    """[buckets(q) for q in queries] in one native call (pflt_buckets_many: a batch's queries
    without a ctypes round trip and its arrays per query); None when the library lacks it."""
    st = store()
    if st is None or not hasattr(st.L, "pflt_buckets_many"):
        return None
    L = st.L
    if not getattr(L, "_buckets_many_bound", False):
        L.pflt_buckets_many.restype = ctypes.c_int64
        L.pflt_buckets_many.argtypes = [ctypes.c_void_p, _u32p, ctypes.POINTER(ctypes.c_uint64), ctypes.c_size_t,
                                        _u32p, ctypes.c_size_t, _u32p, ctypes.c_size_t,
                                        ctypes.POINTER(ctypes.c_int64)]
        L._buckets_many_bound = True
    n = len(queries)
    if n == 0:
        return []
    with st.lock:
        flat = st.export_many([c for q in queries for c in q])
        roots = np.array(flat or [0], dtype=np.uint32)
        offs = np.zeros(n + 1, dtype=np.uint64)
        np.cumsum(np.array([len(q) for q in queries], dtype=np.uint64), out=offs[1:])
        counts = np.zeros(n, dtype=np.int64)
        cap = 4 * len(flat) + 256
        while True:
            ids = np.zeros(cap, dtype=np.uint32)
            sizes = np.zeros(cap, dtype=np.uint32)
            nb = L.pflt_buckets_many(st.h, _p32(roots), offs.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)), n,
                                     _p32(ids), cap, _p32(sizes), cap,
                                     counts.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)))
            if nb != -1:
                break
            cap *= 4
        if nb < 0:
            return None
        terms = st.terms
        idl, szl = ids.tolist(), sizes[:nb].tolist()
        out: List[List[List[T.Term]]] = []
        o = g = 0
        for k in counts.tolist():
            qb = []
            for _ in range(k):
                m = szl[g]
                qb.append([terms[i] for i in idl[o:o + m]])
                o += m
                g += 1
            out.append(qb)
        return out


# ---- batches: parent models, concurrent lowering, native batch packing and re-check ---------
# (include/pf_lower.h "batches"; gpu_check.check_sets' native pipeline)

def batch_api() -> Optional[TermStore]:
    """The store when libpflower.so has the batch entry points, else None."""
    st = store()
    return st if st is not None and hasattr(st.L, "pflt_lower_many") else None


class NativeLowered:
    """to_dag.Lowered of a native result (the witness metadata), decoded on first use:
    check_sets re-checks and records witnesses natively, so most buckets never need it."""

    dag = None

    def __init__(self, res: "_Result"):
        self.res = res
        self._lo: Optional[Lowered] = None

    def _get(self) -> Lowered:
        if self._lo is None:
            self._lo = self.res.lowered()
        return self._lo

    var_terms = property(lambda self: self._get().var_terms)
    uf_apps = property(lambda self: self._get().uf_apps)
    array_reads = property(lambda self: self._get().array_reads)


def candidate0_limbs(prog) -> Optional[np.ndarray]:
    """Candidate 0 of a native program whose every variable has a parent value (the host
    hint model or a parent state's model), as materialize_limbs rows: the generator keeps
    every parented variable's parent at candidate 0, masked to its width
    (include/pf_bytecode.h; ``pf::gen_var``) — pflt_result_candidate0.  None when some
    variable has no parent (the generator then draws it)."""
    r = getattr(prog, "native_result", None)
    if r is None or not hasattr(r.st.L, "pflt_result_candidate0"):
        return None
    nv = int(r.info[0])
    out = np.empty((max(nv, 1), 8), dtype=np.uint32)
    if not r.st.L.pflt_result_candidate0(r.h, _p32(out)):
        return None
    return out[:nv]


class NativeProgram(ir.PackedProgram):
    """ir.PackedProgram of a native result: the batch is packed natively from the result
    (pack_batch); instructions, constants and variables are decoded only when read."""

    def __init__(self, res: "_Result", seed: int):
        self.native_result = res
        self.seed = seed
        self.name = ""
        self._code = None
        self._words = self._consts = self._vars = None

    @property
    def words(self):
        if self._words is None:
            self._words = self.native_result.get(GET_CODE, self.native_result.info[6], 4).copy()
        return self._words

    @property
    def consts(self):
        if self._consts is None:
            nc = self.native_result.info[7]
            raw = self.native_result.get(GET_CONSTS, nc, 8).astype("<u4").tobytes()
            self._consts = [int.from_bytes(raw[32 * i:32 * i + 32], "little") for i in range(nc)]
        return self._consts

    @property
    def vars(self):
        if self._vars is None:
            self._vars = self.native_result.variables()
        return self._vars

    @property
    def has_parent(self) -> bool:
        return bool(self.native_result.info[16])

    def decode(self) -> "NativeProgram":
        """Read everything now (before pflt_result_shrink frees the tables)."""
        self.words, self.consts, self.vars  # noqa: B018
        return self


def _parent_handle(st: TermStore, parent: dict):
    pn, pnv, npn, pr, prv, npr = _parent_args(st, parent)
    return st.L.pflt_parent_new(pn, _p32(pnv), npn, _p32(pr),
                                _p32(prv), npr)


def recent_parent_handle(bucket: List[T.Term], st: Optional[TermStore] = None):
    """The bucket's parent model from the store's recent values (pflt_recent_parent), as a
    handle for lower_many, or None when no value is known (gpu_check._recent_parent).

    ``st``: the store the caller pinned for its whole call: a handle's read keys
    are that store's term ids, so the handle must be read (parent_dict), lowered against
    (lower_many) and freed with the same store even if new_generation retires it meanwhile."""
    st = st or batch_api()
    with st.lock:
        roots = np.array(st.export_many(bucket) or [0], dtype=np.uint32)
        return st.L.pflt_recent_parent(st.h, _p32(roots), len(bucket)) or None


def parent_dict(h, st: Optional[TermStore] = None) -> dict:
    """A parent handle as gpu_check's parent dict (names -> value, select term -> value);
    ``st`` = the store the handle was made from (recent_parent_handle)."""
    st = st or batch_api()
    info = (ctypes.c_uint64 * 4)()
    st.L.pflt_parent_info(h, info)
    nn, nb, nw, nr = (int(x) for x in info)
    names = ctypes.create_string_buffer(max(nb, 1))
    nv = np.zeros(max(nw, 1), dtype=np.uint32)
    rd = np.zeros(max(2 * nr, 1), dtype=np.uint32)
    rv = np.zeros(max(8 * nr, 1), dtype=np.uint32)
    st.L.pflt_parent_get(h, names, _p32(nv), _p32(rd), _p32(rv))
    out: dict = {}
    labels = names.raw[:nb].split(b"\0")[:nn]
    o = 0
    for lab in labels:
        k = int(nv[o])
        out[lab.decode()] = _int_of(nv[o + 1:o + 1 + k])
        o += 1 + k
    for i in range(nr):
        out[T.select(st.terms[int(rd[2 * i])], st.terms[int(rd[2 * i + 1])])] = _int_of(rv[8 * i:8 * i + 8])
    return out


def free_parent(h, st: Optional[TermStore] = None) -> None:
    if h:
        (st or batch_api()).L.pflt_parent_free(h)


def note_vars(vals: Dict[str, int], recent_size: int) -> None:
    st = batch_api()
    if st is None:
        return
    names, words = [], []
    for k, v in vals.items():
        if v is None:
            continue
        names.append(k.encode())
        ls = _limbs_of(int(v))
        words += [len(ls)] + ls
    if names:
        w = np.array(words, dtype=np.uint32)
        with st.lock:
            st.L.pflt_note_vars(st.h, b"\0".join(names) + b"\0", _p32(w), len(names),
                                recent_size)


def note_result(lo: NativeLowered, limbs: np.ndarray, recent_size: int) -> None:
    st = lo.res.st          # the store the result's term ids belong to
    if not isinstance(limbs, np.ndarray):
        limbs = ir.limbs_array([int(x or 0) for x in limbs])
    v = np.ascontiguousarray(limbs, dtype=np.uint32)
    if v.size == 0:
        v = np.zeros(8, dtype=np.uint32)
    with st.lock:
        st.L.pflt_note_result(st.h, lo.res.h, _p32(v), recent_size)


def recent_clear() -> None:
    st = batch_api()
    if st is not None:
        with st.lock:
            st.L.pflt_recent_clear(st.h)


# pflt_job (include/pf_lower.h): roots pointer, n_roots, parents handle, flags, seed
_JOB = np.dtype([("roots", "<u8"), ("n", "<u8"), ("parents", "<u8"), ("flags", "<u4"), ("seed", "<u4")])


def lower_many(jobs: List[Tuple[List[T.Term], object]], reg: UFRegistry, hints: bool, seeds: List[int],
               threads: int, st: Optional[TermStore] = None, flags: Optional[int] = None) -> list:
    """[(bucket, parent handle or None)] -> [(NativeLowered, NativeProgram, None) or
    (None, None, error)], lowered concurrently on ``threads`` host threads.  ``st``: the
    store the parent handles were made from (the caller's pinned store); ``flags``: the
    pflt_lower flags (default PROGRAM, plus HINTS when ``hints``)."""
    st = st or batch_api()
    n = len(jobs)
    if n == 0:
        return []
    with st.lock:
        flat = st.export_many([c for b, _ in jobs for c in b])
        lens = np.array([len(b) for b, _ in jobs], dtype=np.uint64)
        offs = np.zeros(n, dtype=np.uint64)
        np.cumsum(lens[:-1], out=offs[1:])
        roots = np.array(flat or [0], dtype=np.uint32)
        arr = np.zeros(n, dtype=_JOB)
        arr["roots"] = roots.ctypes.data + 4 * offs
        arr["n"] = lens
        arr["parents"] = [h or 0 for _, h in jobs]
        arr["flags"] = flags if flags is not None else PROGRAM | (HINTS if hints else 0)
        arr["seed"] = np.array(seeds, dtype=np.uint64) & 0xFFFFFFFF
        regb = _registry_blob(reg)
        res = (ctypes.c_void_p * n)()
        st.L.pflt_lower_many(st.h, arr.ctypes.data, n, _p32(regb), len(regb),
                             max(1, threads), res)
    out = []
    rows = None
    if hasattr(st.L, "pflt_result_info_many"):
        # every result's status and sizes in one call (a _Result per job otherwise asks twice)
        info = np.zeros((n, 18), dtype=np.uint64)
        st.L.pflt_result_info_many(res, n, info.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)))
        rows = info.tolist()
    for j in range(n):
        h = res[j]
        rc = ctypes.c_int64(rows[j][0]).value if rows is not None else st.L.pflt_result_status(h)
        if rc != 0:
            msg = st.L.pflt_result_error(h).decode(errors="replace")
            st.L.pflt_result_free(h)
            out.append((None, None, msg if rc == -2 else f"ValueError: pflt_lower failed ({rc}): {msg}"))
            continue
        r = _Result(st, h, rows[j][1:] if rows is not None else None)
        out.append((NativeLowered(r), NativeProgram(r, seeds[j]), None))
    return out


def pack_batch(programs: List[NativeProgram]):
    """ir.Batch's arrays (code, consts, schema, parents, descs) packed natively."""
    st = batch_api()
    n = len(programs)
    hs = (ctypes.c_void_p * n)(*[p.native_result.h for p in programs])
    sz = (ctypes.c_uint64 * 4)()
    st.L.pflt_pack_sizes(hs, n, sz)
    ni, nc, nv, np_ = (int(x) for x in sz)
    code = np.zeros((max(ni, 1), 4), dtype=np.uint32)
    consts = np.zeros((max(nc, 1), 8), dtype=np.uint32)
    schema = np.zeros((max(nv, 1), 4), dtype=np.uint32)
    parents = np.zeros((max(np_, 1), 8), dtype=np.uint32)
    descs = np.zeros((max(n, 1), 8), dtype=np.uint32)
    seeds = np.array([p.seed & 0xFFFFFFFF for p in programs] or [0], dtype=np.uint32)
    lut = ir.reach_lut()
    st.L.pflt_pack_batch(hs, n, _p32(seeds), _p32(lut), lut.shape[1],
                         _p32(code), _p32(consts), _p32(schema),
                         _p32(parents), _p32(descs))
    return code[:ni], consts[:nc], schema[:nv], parents[:np_], descs[:n]


def recheck_many(los: List[NativeLowered], limbs: np.ndarray, reg: UFRegistry, threads: int) -> np.ndarray:
    """Status per bucket witness: 1 every conjunct true, 0 some false, -1 not evaluable
    natively (re-check in Python).  limbs = the witnesses' variables back to back."""
    n = len(los)
    if n == 0:
        return np.zeros(0, dtype=np.int8)
    st = los[0].res.st      # the store the results' term ids belong to
    if any(lo.res.st is not st for lo in los):
        # results of two store generations (a retirement between lowering and re-check):
        # each group against its own store
        v = np.ascontiguousarray(limbs, dtype=np.uint32).reshape(-1, 8)
        offs = np.cumsum([0] + [int(lo.res.info[0]) for lo in los])
        status = np.zeros(n, dtype=np.int8)
        for g in {id(lo.res.st) for lo in los}:
            idx = [k for k in range(n) if id(los[k].res.st) == g]
            rows = np.concatenate([v[offs[k]:offs[k + 1]] for k in idx] or [v[:0]])
            status[idx] = recheck_many([los[k] for k in idx], rows, reg, threads)
        return status
    hs = (ctypes.c_void_p * n)(*[lo.res.h for lo in los])
    v = np.ascontiguousarray(limbs, dtype=np.uint32).reshape(-1)
    if v.size == 0:
        v = np.zeros(8, dtype=np.uint32)
    regb = _registry_blob(reg)
    status = np.zeros(n, dtype=np.int8)
    with st.lock:
        st.L.pflt_recheck_many(st.h, hs, n, _p32(v), _p32(regb), len(regb),
                               max(1, threads), _pi8(status))
    return status


def shrink(lo: NativeLowered) -> None:
    """Free the program tables of a result whose program was uploaded (the cache keeps it)."""
    lo.res.st.L.pflt_result_shrink(lo.res.h)


def shrink_many(los: List[NativeLowered]) -> None:
    """shrink() of every result (one library: the entry point is looked up once)."""
    if los:
        f = los[0].res.st.L.pflt_result_shrink
        for lo in los:
            f(lo.res.h)


def ints_of(limbs: np.ndarray) -> List[int]:
    """Rows of 8 u32 limbs -> ints."""
    raw = np.ascontiguousarray(limbs, dtype="<u4").tobytes()
    return [int.from_bytes(raw[32 * i:32 * i + 32], "little") for i in range(len(raw) // 32)]


class NativeWitness:
    """A GPU witness's interpretation held natively (pflt_witness_new, csrc/pf_recheck.cpp):
    the bucket parts' lowering results with their values — interp.Witness.union of the parts'
    witnesses, evaluated by the re-check's evaluator with its memo kept between queries.  The
    GPU-resident ModelCache (mythril_amd/model_cache.py) reads quick-sat leaves through
    ``values_many``, all cached witnesses in one call."""

    __slots__ = ("st", "h", "parts", "__weakref__")

    def __init__(self, st: TermStore, h, parts):
        self.st, self.h, self.parts = st, h, parts   # parts keep the results (and store) alive

    @classmethod
    def build(cls, parts, reg: UFRegistry) -> Optional["NativeWitness"]:
        """parts = [(NativeLowered, values as limb rows or ints)] of one store; None when the
        build has no native witnesses or a part is not native."""
        if not parts or not all(isinstance(lo, NativeLowered) for lo, _ in parts):
            return None
        st = parts[0][0].res.st
        if any(lo.res.st is not st for lo, _ in parts) or not hasattr(st.L, "pflt_witness_new"):
            return None
        rows = []
        for lo, v in parts:
            nv = int(lo.res.info[0])
            r = np.ascontiguousarray(v, dtype=np.uint32).reshape(-1, 8) if isinstance(v, np.ndarray) \
                else ir.limbs_array(list(v)).reshape(-1, 8) if len(v) else np.zeros((0, 8), dtype=np.uint32)
            if len(r) != nv:
                return None
            rows.append(r)
        vals = np.concatenate(rows) if rows else np.zeros((0, 8), dtype=np.uint32)
        if vals.size == 0:
            vals = np.zeros((1, 8), dtype=np.uint32)
        vals = np.ascontiguousarray(vals).reshape(-1)
        blob, serial = _registry_blob_serial(reg)
        hs = (ctypes.c_void_p * len(parts))(*[lo.res.h for lo, _ in parts])
        with st.lock:
            h = st.L.pflt_witness_new(st.h, hs, len(parts), _p32(vals),
                                      _p32(blob), len(blob), serial)
        if not h:
            return None
        return cls(st, h, [lo for lo, _ in parts])

    def __del__(self):
        try:
            self.st.L.pflt_witness_free(self.h)
        except Exception:  # noqa: BLE001
            pass


# leaf slots: a dense number per term read through witness_values_many, under which each
# native witness keeps the value (33 bytes per slot per witness: at most ~0.5 MB each, ~50 MB
# for a full 100-model cache); renumbered (new epoch) when the table grows past _SLOTS_MAX
# The table is process-wide while the callers hold only their own store's lock, so it has a
# lock of its own, and the epoch is returned with the slots from the same snapshot: a caller
# that renumbers (new epoch) cannot hand another caller its epoch for older slot numbers.
_SLOTS: Dict[T.Term, int] = {}
_SLOT_EPOCH = [1]
_SLOTS_MAX = 1 << 14
_SLOTS_LOCK = threading.Lock()


def _slots_of(terms: List[T.Term]) -> Tuple[np.ndarray, int, int]:
    """(slots, how many of them are new, the epoch they belong to)."""
    with _SLOTS_LOCK:
        if len(_SLOTS) + len(terms) > _SLOTS_MAX:
            _SLOTS.clear()
            _SLOT_EPOCH[0] += 1
        out = np.empty(len(terms), dtype=np.uint32)
        n0 = len(_SLOTS)
        for i, t in enumerate(terms):
            s = _SLOTS.get(t)
            if s is None:
                s = _SLOTS[t] = len(_SLOTS)
            out[i] = s
        return out, len(_SLOTS) - n0, _SLOT_EPOCH[0]


def witness_values_many(ws: List[NativeWitness], terms: List[T.Term], reg: UFRegistry, threads: int = 1):
    """(values [model][term][8] u32 limbs, each masked to its term's width; ok [model][term]
    bool) of ``terms`` under every witness of ``ws`` (one store), natively in one call."""
    n, k = len(ws), len(terms)
    out = np.empty((n, k, 8), dtype=np.uint32)   # every (model, term) the call marks ok is written
    ok = np.zeros((n, k), dtype=np.uint8)
    if n == 0 or k == 0:
        return out, ok.astype(bool)
    st = ws[0].st
    blob, serial = _registry_blob_serial(reg)
    hs = (ctypes.c_void_p * n)(*[w.h for w in ws])
    with st.lock:
        ids = np.array(st.export_many(terms), dtype=np.uint32)
        slots, fresh, epoch = _slots_of(terms)
        if not fresh:
            # every term was read before: mostly 32-byte copies, cheaper than waking the pool
            threads = 1
        st.L.pflt_witness_values(hs, n, _p32(ids), k, _p32(slots), epoch,
                                 _p32(blob), len(blob),
                                 serial, max(1, threads), _p32(out),
                                 _p8(ok))
    return out, ok.astype(bool)
