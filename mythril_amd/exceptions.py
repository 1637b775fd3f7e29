"""Exceptions of the query funnel (mirror of mythril/exceptions.py:16-28)."""


class UnsatError(Exception):
    """The constraints are unsatisfiable."""


class SolverTimeOutException(UnsatError):
    """The solver gave up (timeout / unknown)."""
