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
HINTS, PROGRAM = 1, 2
GET_VARS, GET_VAR_TERMS, GET_UF_APPS, GET_READS, GET_CODE, GET_CONSTS, GET_NODES, GET_POOL, \
    GET_ROOTS, GET_FORCED = range(10)
VT_TERM, VT_SELECT, VT_EXTRACT = 0, 1, 2

_u32p = ctypes.POINTER(ctypes.c_uint32)


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
    _SIGNED = True


class TermStore:
    """The process's native term store (one per process; terms enter once)."""

    def __init__(self, lib):
        _bind(lib)
        self.L = lib
        self.h = lib.pflt_store_new()
        self.ids: Dict[T.Term, int] = {}
        self.terms: List[T.Term] = []
        self.lock = threading.Lock()

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


_BLOBS: Dict[tuple, np.ndarray] = {}


def _registry_blob(reg: UFRegistry) -> np.ndarray:
    """The registry in pflt_lower's layout, cached per registry state (hashes only get added:
    the per-width counts and interval starts identify the state)."""
    key = (id(reg), tuple(reg.actors),
           tuple((n, s.lo, len(s.concrete)) for n, s in reg.keccak.items()))
    blob = _BLOBS.get(key)
    if blob is None:
        if len(_BLOBS) > 64:
            _BLOBS.clear()
        blob = _BLOBS[key] = _registry_blob_build(reg)
    return blob


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

    def __init__(self, st: TermStore, h):
        self.st, self.h = st, h
        info = (ctypes.c_uint64 * 14)()
        st.L.pflt_result_info(h, info)
        self.info = [int(x) for x in info]

    def __del__(self):
        try:
            self.st.L.pflt_result_free(self.h)
        except Exception:  # noqa: BLE001
            pass

    def get(self, which: int, n: int, cols: int) -> np.ndarray:
        out = np.zeros(max(n * cols, 1), dtype=np.uint32)
        self.st.L.pflt_result_get(self.h, which, out.ctypes.data_as(_u32p), None)
        return out[:n * cols].reshape(n, cols) if cols > 1 else out[:n]

    def variables(self) -> List[ir.Var]:
        nv, nb = self.info[0], self.info[1]
        out = np.zeros(max(nv * 13, 1), dtype=np.uint32)
        names = ctypes.create_string_buffer(max(nb, 1))
        self.st.L.pflt_result_get(self.h, GET_VARS, out.ctypes.data_as(_u32p), names)
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

    def lowered(self) -> Lowered:
        terms = self.st.terms
        vt = self.get(GET_VAR_TERMS, self.info[2], 4)
        var_terms = []
        for typ, a, b, c in vt.tolist():
            if typ == VT_TERM:
                var_terms.append(terms[a])
            elif typ == VT_SELECT:
                var_terms.append(T.select(terms[a], terms[b]))
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
                arr, idx = terms[pairs[2 * k]], terms[pairs[2 * k + 1]]
                reads.setdefault(arr.val, []).append((idx, T.select(arr, idx)))
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
        roots = np.array([st.export(c) for c in bucket] or [0], dtype=np.uint32)
        regb = _registry_blob(reg)
        pn, pnv, npn, pr, prv, npr = _parent_args(st, parent)
        rc = ctypes.c_int(0)
        h = st.L.pflt_lower(st.h, roots.ctypes.data_as(_u32p), len(bucket), regb.ctypes.data_as(_u32p),
                            len(regb), pn, pnv.ctypes.data_as(_u32p), npn, pr.ctypes.data_as(_u32p),
                            prv.ctypes.data_as(_u32p), npr, flags, seed & 0xFFFFFFFF, ctypes.byref(rc))
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
        rc = L.pflt_recheck(st.h, d_.ctypes.data_as(_u32p), len(lo.var_terms), vals.ctypes.data_as(_u32p),
                            u_.ctypes.data_as(_u32p), len(ufs), r_.ctypes.data_as(_u32p), len(reads) // 2,
                            regb.ctypes.data_as(_u32p), len(regb), ro_.ctypes.data_as(_u32p), len(roots),
                            out.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)))
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
        roots = np.array([st.export(c) for c in constraints] or [0], dtype=np.uint32)
        cap = 4 * len(constraints) + 256
        while True:
            ids = np.zeros(cap, dtype=np.uint32)
            sizes = np.zeros(cap, dtype=np.uint32)
            nb = L.pflt_buckets(st.h, roots.ctypes.data_as(_u32p), len(constraints), ids.ctypes.data_as(_u32p),
                                cap, sizes.ctypes.data_as(_u32p), cap)
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
