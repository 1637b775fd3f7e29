"""Test tooling: evaluate a mythril_amd.lower.Dag directly with the oracle's semantics.

Term-level twin of the bytecode evaluation: lowering (register allocation, remat) must not
change the value of the conjunction.
"""

import pyoracle as O

from mythril_amd import ir
from mythril_amd.lower import K_BCONST, K_BVAR, K_CONST, K_VAR

_W = {
    ir.W_ADD: O.bvadd, ir.W_SUB: O.bvsub, ir.W_MUL: O.bvmul, ir.W_UDIV: O.bvudiv,
    ir.W_UREM: O.bvurem, ir.W_SDIV: O.bvsdiv, ir.W_SREM: O.bvsrem, ir.W_SMOD: O.bvsmod,
    ir.W_AND: lambda a, b, w: a & b, ir.W_OR: lambda a, b, w: a | b,
    ir.W_XOR: lambda a, b, w: a ^ b, ir.W_SHL: O.bvshl, ir.W_LSHR: O.bvlshr,
    ir.W_ASHR: O.bvashr, ir.W_EXP: O.bvexp,
}
_B = {
    ir.B_EQ: lambda a, b, w: a == b, ir.B_ULT: O.ult, ir.B_ULE: O.ule, ir.B_SLT: O.slt,
    ir.B_SLE: O.sle, ir.B_UADD_NOOVF: O.uadd_noovf, ir.B_UMUL_NOOVF: O.umul_noovf,
}


def eval_dag(dag, values):
    val = eval_dag_values(dag, values)
    return all(val[r] for r in dag.roots)


def eval_dag_values(dag, values):
    """Value of every node."""
    val = {}
    for i, n in enumerate(dag.nodes):
        k, w = n.kind, n.width
        if k == K_VAR:
            v = values[n.aux] & O.M(w)
        elif k == K_CONST:
            v = n.aux & O.M(w)
        elif k == K_BCONST:
            v = bool(n.aux)
        elif k == K_BVAR:
            v = bool(values[n.aux] & 1)
        elif k in _W:
            v = _W[k](val[n.args[0]], val[n.args[1]], w)
        elif k == ir.W_HASH:
            v = O.uf_hash(val[n.args[0]], n.aux) & O.M(w)
        elif k == ir.W_NOT:
            v = O.bvnot(val[n.args[0]], w)
        elif k == ir.W_NEG:
            v = O.bvneg(val[n.args[0]], w)
        elif k == ir.W_MOV:
            v = val[n.args[0]] & O.M(w)
        elif k == ir.W_EXTRACT:
            v = O.extract(val[n.args[0]], n.aux, w)
        elif k == ir.W_CONCAT:
            v = O.concat(val[n.args[0]], val[n.args[1]], n.aux) & O.M(w)
        elif k == ir.W_SEXT:
            v = O.sign_extend(val[n.args[0]], n.aux, w)
        elif k == ir.W_ITE:
            v = val[n.args[1]] if val[n.args[0]] else val[n.args[2]]
        elif k in _B:
            v = bool(_B[k](val[n.args[0]], val[n.args[1]], w))
        elif k == ir.B_AND:
            v = val[n.args[0]] and val[n.args[1]]
        elif k == ir.B_OR:
            v = val[n.args[0]] or val[n.args[1]]
        elif k == ir.B_XOR:
            v = val[n.args[0]] != val[n.args[1]]
        elif k == ir.B_NOT:
            v = not val[n.args[0]]
        elif k == ir.B_ITE:
            v = val[n.args[1]] if val[n.args[0]] else val[n.args[2]]
        else:
            raise ValueError(k)
        val[i] = v
    return val

