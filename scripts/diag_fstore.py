"""Development aid: the frame-store Ape-X loop against the full-row one in lockstep (eager),
reporting the first iteration where the actors' ring, actions, the replay rows, the learner's
batch slots or the parameters differ (tests/test_frame_store_gpu.py's failure triage)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from reth_amd.apex import ApexConfig, ApexDQN  # noqa: E402

dev = torch.device("cuda:0")
graph = len(sys.argv) > 1 and sys.argv[1] == "graph"


def make(fs):
    cfg = ApexConfig(n_actors=16, capacity=1024, batch_size=32, sample_start=64, p_done=0.25, seed=6, hip_graph=graph,
                     send_weights_interval=3, recv_weights_interval=4, update_target_interval=5, frame_store=fs)
    return ApexDQN(cfg, device=dev)


a, b = make(False), make(True)
seen = set()
for it in range(150):
    a.iteration()
    b.iteration()
    torch.cuda.synchronize()
    checks = {"ring": (a.actors.frames, b.actors.frames), "action": (a.actors.action, b.actors.action),
              "done": (a.actors.done, b.actors.done), "updates": (torch.tensor(a.updates), torch.tensor(b.updates))}
    n = a.replay.info()[0]
    if n:
        ca = a.replay.gather(torch.arange(n, device=dev))
        cb = b.replay.gather(torch.arange(n, device=dev))
        for name, x, y in zip(["s0", "a", "r", "s1", "done"], ca, cb):
            checks["rep_" + name] = (x, y)
        ta, tb = a.replay.tree.export(), b.replay.tree.export()
        checks["tree_val"] = (ta[2], tb[2])
    for k, (sa, sb) in enumerate(zip(a.loader._slots or [], b.loader._slots or [])):
        for j, (x, y) in enumerate(zip(sa[0], sb[0])):
            checks[f"slot{k}_col{j}"] = (x, y)
        checks[f"slot{k}_idx"] = (sa[1], sb[1])
    pa = torch.cat([p.detach().flatten() for p in a.solver._params])
    pb = torch.cat([p.detach().flatten() for p in b.solver._params])
    checks["params"] = (pa, pb)
    for name, (x, y) in checks.items():
        if name in seen:
            continue
        if x.shape != y.shape or not torch.equal(x, y):
            seen.add(name)
            extra = ""
            if x.shape == y.shape:
                d = (x != y)
                extra = f" {int(d.sum())} of {d.numel()} differ; first at {tuple(int(v) for v in d.nonzero()[0])}"
            print(f"iteration {it}: {name} differs{extra}", flush=True)
print("done; differing:", sorted(seen), flush=True)
