"""mythril_amd.smt — drop-in for ``mythril.laser.smt`` (mythril/laser/smt/__init__.py:1-153).

Same exported names; ``Solver``/``Optimize.check()`` answer objective-free queries with the
MI355X batched search and leave everything else to z3 unchanged.
"""

from .expr import (  # noqa: F401
    UGE, UGT, ULE, ULT, And, Array, BaseArray, BitVec, Bool, BVAddNoOverflow,
    BVMulNoOverflow, BVSubNoUnderflow, Concat, Expression, Extract, Function, If, K, LShR,
    Not, Or, SMod, SRem, Sum, UDiv, URem, Xor, is_false, is_true, simplify, symbol_factory,
)
from .model import Model  # noqa: F401
from .solver import (  # noqa: F401
    BaseSolver, Optimize, Solver, SolverStatistics, sat, stat_smt_query, unknown, unsat,
)

SMTBool = Bool
