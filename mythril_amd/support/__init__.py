"""Mirror of mythril.support pieces on the hot path (the query funnel)."""
