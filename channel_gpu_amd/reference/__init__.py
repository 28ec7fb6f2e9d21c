"""NumPy fp64 oracle implementations (CPU reference path and test oracles)."""
from .oracle import OraclePlan, OracleSolver, build_ops, random_state, ygrid  # noqa: F401
