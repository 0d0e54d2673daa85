"""`reth.env` (reth/reth/env/__init__.py)"""
from reth_amd.envs import make  # noqa: F401
