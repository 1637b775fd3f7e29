"""Independence buckets — the GPU-side twin of mythril/laser/smt/solver/independence_solver.py.

The reference (``DependenceMap.add_condition``, independence_solver.py:38-83) groups the
conditions of a query into buckets that share no variable, solves each bucket on its own
and returns the union of the bucket models.  Here the same split happens before lowering:
every bucket becomes its own GPU program, so a candidate only has to satisfy the conditions
of one bucket (the hit rate of a conjunction of k independent parts is the product of the
parts' rates; split, it is the minimum).  The set is SAT iff every bucket has a witness.

Dependence keys are stricter than the reference's leaves, because the GPU interprets
arrays and UFs by construction (mythril_amd/smt/to_dag.py):
* a free BitVec/Bool symbol -> its name;
* a base array -> its name (all reads of one array must share one interpretation);
* ``keccak256_<n>`` and its inverse ``keccak256_<n>-1`` -> one family key per width n
  (injectivity side conditions and inverse lookups range over every application of n).
Other UFs (keyed hashes of their arguments, ``Power`` = EXP) are functions by construction
and couple nothing beyond their arguments.
"""

from __future__ import annotations

import re
from typing import Dict, FrozenSet, List

from . import terms as T

_KECCAK_RE = re.compile(r"^keccak256_(\d+)(?:-1)?$")

_keys_memo: Dict[T.Term, FrozenSet[str]] = {}


def dependence_keys(t: T.Term) -> FrozenSet[str]:
    """Symbols (and array / keccak-family keys) the value of ``t`` depends on."""
    r = _keys_memo.get(t)
    if r is not None:
        return r
    stack = [t]
    while stack:
        x = stack[-1]
        if x in _keys_memo:
            stack.pop()
            continue
        pend = [a for a in x.args if a not in _keys_memo]
        if pend:
            stack.extend(pend)
            continue
        stack.pop()
        own = set()
        if x.op in ("var", "bvar"):
            own.add("v:" + x.val)
        elif x.op == "array":
            own.add("a:" + x.val)
        elif x.op == "apply":
            m = _KECCAK_RE.match(x.val[0])
            if m:
                own.add("k:" + m.group(1))
        for a in x.args:
            own |= _keys_memo[a]
        _keys_memo[x] = frozenset(own)
    return _keys_memo[t]


def buckets(constraints: List[T.Term]) -> List[List[T.Term]]:
    """Partition ``constraints`` into variable-disjoint buckets (order kept inside each)."""
    parent: Dict[str, str] = {}

    def find(k: str) -> str:
        while parent[k] != k:
            parent[k] = parent[parent[k]]
            k = parent[k]
        return k

    keyed = []
    for c in constraints:
        ks = dependence_keys(c)
        keyed.append((c, ks))
        first = None
        for k in ks:
            if k not in parent:
                parent[k] = k
            if first is None:
                first = find(k)
            else:
                rk = find(k)
                if rk != first:
                    parent[rk] = first
    groups: Dict[str, List[T.Term]] = {}
    ground: List[T.Term] = []   # variable-free constraints (constant after folding)
    for c, ks in keyed:
        if not ks:
            ground.append(c)
            continue
        groups.setdefault(find(next(iter(ks))), []).append(c)
    out = list(groups.values())
    if ground:
        out.append(ground)
    return out
