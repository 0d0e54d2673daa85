"""Data-parallel learner support: one process per GPU, gradients averaged over RCCL.

The reference has no collective at all (one learner, ZeroMQ everywhere).
Ape-X shards naturally: every GPU owns its actors and its replay shard (the reference's
K shards of capacity C // K, test/apex-dqn/trainer.py:52-61), so the only exchange step is
the learner's gradient: 1.69 M fp32 params = 6.7 MB for Pong per update.  It goes in two
flat buckets: the merged dueling heads' gradients (95 % of the bytes, final right after the
FC backward) are all-reduced on a side stream while the conv backward runs, the conv
gradients on the learner's stream after it, and the final part of the update (heads split
+ clip + Adam) waits for both (ApexDQN._capture / _learner_replay).  The eager learner
reduces everything as one bucket.
"""
import gc

import torch
import torch.distributed as dist


class GradAllReduce:
    """grad_hook for DQNSolver: average gradients over the process group, one collective per
    bucket.

    Each bucket (a fixed list of gradient tensors) gets one flat buffer, allocated once;
    grads are copied in and out with two fused foreach copies (no per-parameter
    collectives).  The eager learner reduces everything as one bucket; the captured learner
    reduces the fully-connected gradients on a side stream while the conv backward runs
    (ApexDQN._capture)."""

    def __init__(self, group=None, force=False):
        self.group = group
        self.force = force  # run the collective in a one-rank group too (tests: RCCL on one GPU)
        self._flat = {}  # bucket key -> (flat buffer, views)

    def world(self):
        return dist.get_world_size(self.group) if dist.is_initialized() else 1

    def _active(self):
        return self.world() > 1 or (self.force and dist.is_initialized())

    def reduce(self, grads, key="all"):
        """all-reduce-average the tensors in `grads` in place, on the current stream"""
        world = self.world()
        if not self._active():
            return
        ent = self._flat.get(key)
        if ent is None or ent[1][0].shape != grads[0].shape or len(ent[1]) != len(grads):
            n = sum(g.numel() for g in grads)
            flat = torch.empty(n, dtype=torch.float32, device=grads[0].device)
            views, off = [], 0
            for g in grads:
                views.append(flat[off: off + g.numel()].view_as(g))
                off += g.numel()
            ent = self._flat[key] = (flat, views)
        flat, views = ent
        torch._foreach_copy_(views, grads)
        if flat.is_cuda and dist.get_backend(self.group) != "nccl":
            # gloo stages CUDA tensors through the host: hand it a finished buffer (its
            # own stream bookkeeping against a busy non-default stream stalls for seconds)
            torch.cuda.current_stream(flat.device).synchronize()
        dist.all_reduce(flat, op=dist.ReduceOp.SUM, group=self.group)
        flat.div_(world)
        torch._foreach_copy_(grads, views)

    def __call__(self, params, grads=None):
        """grads: the gradient tensors to reduce (default: each parameter's .grad)"""
        if not self._active():
            return
        self.reduce([p.grad for p in params] if grads is None else list(grads))


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


def shutdown(*owners):
    """orderly end of a data-parallel rank (bench.py, tests/test_rccl_gpu.py): drain the device,
    release the owners' captured graphs and streams (`close()`), then destroy the process group.
    The order matters: every RCCL call is issued eagerly between graph parts on the learner's
    side stream (ApexDQN._learner_replay), none is captured, so once the device is idle no
    graph references a communicator; the graphs are dropped while the HIP runtime and the
    communicator are both still alive, and the group is destroyed last, with nothing queued
    on any stream.  Returns normally -- the interpreter's own exit follows."""
    cuda = torch.cuda.is_available() and torch.cuda.is_initialized()
    if cuda:
        torch.cuda.synchronize()
    for o in owners:
        if o is not None:
            o.close()
    gc.collect()
    if cuda:
        torch.cuda.synchronize()
    if dist.is_initialized():
        dist.destroy_process_group()
