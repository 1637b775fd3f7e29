"""Term substitution (Bool.substitute / BaseArray.substitute in the reference,
mythril/laser/smt/bool.py:82-93, array.py:34-44)."""

from . import terms as T

_REBUILD = {
    "extract": lambda t, a: T.extract(t.val[0], t.val[1], a[0]),
    "concat": lambda t, a: T.concat(*a),
    "zero_extend": lambda t, a: T.zero_extend(t.val, a[0]),
    "ite": lambda t, a: T.ite(*a),
    "and": lambda t, a: T.and_(*a),
    "or": lambda t, a: T.or_(*a),
    "not": lambda t, a: T.not_(a[0]),
    "xor": lambda t, a: T.xor(*a),
    "=": lambda t, a: T.eq(*a),
    "iff": lambda t, a: T.eq(*a),
    "bvnot": lambda t, a: T.bvnot(a[0]),
    "bvneg": lambda t, a: T.bvneg(a[0]),
    "select": lambda t, a: T.select(*a),
    "store": lambda t, a: T.store(*a),
    "K": lambda t, a: T.const_array(t.sort[1], a[0]),
    "apply": lambda t, a: T.Term("apply", t.sort, tuple(a), t.val),
}


def substitute(t: T.Term, old: T.Term, new: T.Term, _memo=None) -> T.Term:
    """``t`` with every occurrence of ``old`` replaced by ``new``: an iterative post-order walk
    (LASER terms nest deeper than Python's recursion limit), each node rebuilt through its
    folding constructor only when one of its arguments changed."""
    memo = {} if _memo is None else _memo
    stack = [(t, False)]
    while stack:
        u, ready = stack.pop()
        if u is old or not u.args or u in memo:
            continue
        if not ready:
            stack.append((u, True))
            for a in u.args:
                if a is not old and a.args and a not in memo:
                    stack.append((a, False))
            continue
        args = [new if a is old else (memo.get(a, a) if a.args else a) for a in u.args]
        if all(x is y for x, y in zip(args, u.args)):
            r = u
        elif u.op in _REBUILD:
            r = _REBUILD[u.op](u, args)
        elif u.op in T._FOLD2:
            r = T.binop(u.op, *args)
        elif u.op in T._CMP:
            r = T.cmp(u.op, *args)
        else:
            raise ValueError(f"substitute: unknown op {u.op}")
        memo[u] = r
    if t is old:
        return new
    return memo.get(t, t) if t.args else t
