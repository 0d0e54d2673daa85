"""`reth.presets` (reth/reth/presets/__init__.py)"""
from reth_amd.presets import Worker  # noqa: F401
from reth_amd.trainer import Trainer  # noqa: F401

from . import config  # noqa: F401
