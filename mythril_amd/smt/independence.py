"""Independence buckets — the GPU-side twin of mythril/laser/smt/solver/independence_solver.py.

The reference (``DependenceMap.add_condition``, independence_solver.py:38-83) groups the
conditions of a query into buckets that share no variable, solves each bucket on its own
and returns the union of the bucket models.  Here the same split happens before lowering:
every bucket becomes its own GPU program, so a candidate only has to satisfy the conditions
of one bucket (the hit rate of a conjunction of k independent parts is the product of the
parts' rates; split, it is the minimum).  The set is SAT iff every bucket has a witness.

Dependence keys follow the GPU's interpretation of arrays and UFs
(mythril_amd/smt/to_dag.py):
* a free BitVec/Bool symbol -> its name;
* a base array -> its name (all reads of one array must share one interpretation);
* ``keccak256_<n>`` is a fixed function of its argument's value (the registered concrete
  hash, else ``base_n + 64 * H(x)``), so its applications couple nothing beyond their
  arguments — except when the set also applies the inverse ``keccak256_<n>-1`` to a value
  that is not itself an application: that lookup ranges over every application of width
  n, so then all of them share one family key.
Other UFs (keyed hashes of their arguments) are functions by construction; ``Power`` couples
every constraint that applies it (its symbolic applications are shared candidate variables).
Top-level conjunctions are split first (``Constraints.get_all_constraints`` appends the
keccak manager's conditions as one big ``And``, constraints.py:132-133; its conjuncts
belong to different buckets).
"""

from __future__ import annotations

import re
from typing import Dict, FrozenSet, List

from . import terms as T

_KECCAK_RE = re.compile(r"^keccak256_(\d+)(?:-1)?$")

_keys_memo: Dict[T.Term, FrozenSet[str]] = {}
_free_inv_memo: Dict[T.Term, FrozenSet[str]] = {}


def free_inverse_widths(t: T.Term) -> FrozenSet[str]:
    """Widths n for which ``t`` applies ``keccak256_<n>-1`` to a non-application."""
    r = _free_inv_memo.get(t)
    if r is not None:
        return r
    stack = [t]
    while stack:
        x = stack[-1]
        if x in _free_inv_memo:
            stack.pop()
            continue
        pend = [a for a in x.args if a not in _free_inv_memo]
        if pend:
            stack.extend(pend)
            continue
        stack.pop()
        own = set()
        if x.op == "apply":
            m = _KECCAK_RE.match(x.val[0])
            if m and x.val[0].endswith("-1"):
                a = x.args[0]
                if not (a.op == "apply" and a.val[0] == f"keccak256_{m.group(1)}"):
                    own.add(m.group(1))
        for a in x.args:
            own |= _free_inv_memo[a]
        _free_inv_memo[x] = frozenset(own)
    return _free_inv_memo[t]


def dependence_keys(t: T.Term) -> FrozenSet[str]:
    """Symbols, arrays and keccak widths (``k:<n>``) the value of ``t`` depends on."""
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
            elif x.val[0] == "Power":
                # Power's symbolic applications are candidate variables kept functional
                # by argument value across the set (to_dag.TermLowering._power): every
                # constraint applying it, concrete table entries included, shares a bucket
                own.add("f:Power")
        for a in x.args:
            own |= _keys_memo[a]
        _keys_memo[x] = frozenset(own)
    return _keys_memo[t]


def _conjuncts(constraints: List[T.Term]) -> List[T.Term]:
    out: List[T.Term] = []
    stack = list(reversed(constraints))
    while stack:
        c = stack.pop()
        if c.op == "and":
            stack.extend(reversed(c.args))
        elif c is not T.TRUE:
            out.append(c)
    return out


def buckets(constraints: List[T.Term]) -> List[List[T.Term]]:
    """Partition ``constraints`` into variable-disjoint buckets (order kept inside each)."""
    constraints = _conjuncts(constraints)
    families = frozenset()
    for c in constraints:
        families |= free_inverse_widths(c)
    parent: Dict[str, str] = {}

    def find(k: str) -> str:
        while parent[k] != k:
            parent[k] = parent[parent[k]]
            k = parent[k]
        return k

    keyed = []
    for c in constraints:
        ks = dependence_keys(c)
        # keccak widths only couple when the set has a free inverse lookup of that width
        ks = frozenset(k for k in ks if not k.startswith("k:") or k[2:] in families)
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
