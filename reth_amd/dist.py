"""Data-parallel learner support: one process per GPU, gradients averaged over RCCL.

The reference has no collective at all (one learner, ZeroMQ everywhere).
Ape-X shards naturally: every GPU owns its actors and its replay shard (the reference's
K shards of capacity C // K, test/apex-dqn/trainer.py:52-61), so the only exchange step is
the learner's gradient.  It is one flat fp32 bucket (1.69 M params = 6.7 MB for Pong)
all-reduced once per update -- on xGMI a ring all-reduce of 6.7 MB is ~80 us, small next
to the Q-net backward, so there is no bucketing/overlap machinery.
"""
import torch
import torch.distributed as dist


class GradAllReduce:
    """grad_hook for DQNSolver: average .grad over the process group in one collective.

    The flat buffer is allocated once; grads are copied in and out with two fused foreach
    copies (no per-parameter collectives)."""

    def __init__(self, group=None):
        self.group = group
        self._flat = None
        self._views = None

    def _bind(self, params):
        n = sum(p.numel() for p in params)
        dev = params[0].device
        self._flat = torch.empty(n, dtype=torch.float32, device=dev)
        self._views, off = [], 0
        for p in params:
            self._views.append(self._flat[off: off + p.numel()].view_as(p))
            off += p.numel()

    def __call__(self, params, grads=None):
        """grads: the gradient tensors to reduce (default: each parameter's .grad; a replayed
        HIP graph passes the buffers its captured backward writes)"""
        world = dist.get_world_size(self.group) if dist.is_initialized() else 1
        if world == 1:
            return
        if self._flat is None:
            self._bind(params)
        if grads is None:
            grads = [p.grad for p in params]
        torch._foreach_copy_(self._views, grads)
        if self._flat.is_cuda and dist.get_backend(self.group) != "nccl":
            # gloo stages CUDA tensors through the host: hand it a finished buffer (its
            # own stream bookkeeping against a busy non-default stream stalls for seconds)
            torch.cuda.current_stream(self._flat.device).synchronize()
        dist.all_reduce(self._flat, op=dist.ReduceOp.SUM, group=self.group)
        self._flat.div_(world)
        torch._foreach_copy_(grads, self._views)


def init_from_env(backend=None):
    """torch.distributed init from torchrun's env (RANK/WORLD_SIZE/MASTER_ADDR/...)."""
    import os

    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world == 1 or dist.is_initialized():
        return (dist.get_rank() if dist.is_initialized() else 0), world
    if backend is None:
        backend = os.environ.get("RTH_DIST_BACKEND")  # e.g. gloo for a multi-rank rehearsal on one GPU
    if backend is None:
        backend = "nccl" if torch.cuda.is_available() else "gloo"  # nccl == RCCL on ROCm
    dist.init_process_group(backend=backend)
    return dist.get_rank(), dist.get_world_size()
