"""`reth.utils` (reth/reth/utils/__init__.py:1-20)"""
from reth_amd.nstep import NStepAdder  # noqa: F401
from reth_amd.schedule import Interval, Schedule  # noqa: F401
from reth_amd.trainer import getLogger  # noqa: F401
