"""`reth.algorithm` (reth/reth/algorithm/__init__.py:17-21): the DQN solver only"""
from reth_amd.solver import DQNSolver, get_solver  # noqa: F401
