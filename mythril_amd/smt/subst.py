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
    memo = {} if _memo is None else _memo
    if t is old:
        return new
    if not t.args:
        return t
    r = memo.get(t)
    if r is not None:
        return r
    args = [substitute(a, old, new, memo) for a in t.args]
    if all(x is y for x, y in zip(args, t.args)):
        r = t
    elif t.op in _REBUILD:
        r = _REBUILD[t.op](t, args)
    elif t.op in T._FOLD2:
        r = T.binop(t.op, *args)
    elif t.op in T._CMP:
        r = T.cmp(t.op, *args)
    else:
        raise ValueError(f"substitute: unknown op {t.op}")
    memo[t] = r
    return r
