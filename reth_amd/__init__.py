"""reth_amd: MI355X-native Ape-X DQN rollout -> prioritized replay -> update hot path.

Host side of libreth_hip.so (hand-written gfx950 HIP kernels behind a C ABI,
include/reth_hip.h).  Modules mirror the reference's interfaces:

    reth_amd.reth_buffer   start_per / start_server / Client / NumpyLoader / TorchCudaLoader
    reth_amd.replay        SumTree (NumbaSumTree), PERSampler, HbmReplay
    reth_amd.solver        DQNSolver (reth.algorithm.DQNSolver), td_huber_loss
    reth_amd.trainer       Trainer (reth.presets.Trainer)
    reth_amd.actors        VecActors (the apex-dqn worker loop, vectorised on the GPU)
    reth_amd.apex          ApexDQN / ApexConfig (test/apex-dqn wiring, one process per GPU)
    reth_amd.schedule      Schedule, Interval
"""
from ._lib import HipExtensionMissing, RethHipError, lib  # noqa: F401

__all__ = ["lib", "HipExtensionMissing", "RethHipError"]
