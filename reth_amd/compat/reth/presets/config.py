"""`reth.presets.config` -> reth_amd.presets (reth/reth/presets/config.py:12-73)"""
from reth_amd.presets import get_env, get_replay_buffer, get_solver, get_trainer, get_worker  # noqa: F401
