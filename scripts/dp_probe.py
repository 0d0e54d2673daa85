"""Probe: where the time goes in a multi-rank Ape-X step (development aid; run under
torch.distributed.run, RTH_SHARE_GPU/RTH_DIST_BACKEND for a one-GPU rehearsal)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from reth_amd.apex import ApexConfig, ApexDQN
from reth_amd.dist import init_from_env

local = int(os.environ.get("LOCAL_RANK", "0")) % torch.cuda.device_count()
torch.cuda.set_device(local)
rank, world = init_from_env()
dev = torch.device("cuda", local)
cfg = ApexConfig(n_actors=256, capacity=50000, batch_size=512, seed=0, hip_graph=os.environ.get("EAGER") is None)
ax = ApexDQN(cfg, device=dev, rank=rank, world=world)
ax.prefill(cfg.capacity)
hook = ax.solver.grad_hook
acc = {"hook": 0.0, "n": 0}


def timed_hook(params, grads=None):
    torch.cuda.synchronize()
    t = time.perf_counter()
    hook(params, grads=grads)
    torch.cuda.synchronize()
    acc["hook"] += time.perf_counter() - t
    acc["n"] += 1


if hook is not None:
    ax.solver.grad_hook = timed_hook
for _ in range(10):
    ax.iteration()
torch.cuda.synchronize()
acc.update(hook=0.0, n=0)
t0 = time.perf_counter()
for _ in range(20):
    ax.iteration()
torch.cuda.synchronize()
dt = time.perf_counter() - t0
print(f"rank {rank}/{world}: {dt / 20 * 1e3:.1f} ms/step, hook {acc['hook'] / max(acc['n'], 1) * 1e3:.1f} ms "
      f"x {acc['n']}, graphs={ax._graphs is not None}", flush=True)
