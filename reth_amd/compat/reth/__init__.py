"""`reth` -> reth_amd (reth/reth/__init__.py: algorithm, buffer, env, presets, utils)"""
from . import algorithm, buffer, env, presets, utils  # noqa: F401
