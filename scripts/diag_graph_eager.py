"""Development aid (r06): the Ape-X loop eager vs graph-replayed at lr = 0 (test_scale_gpu's
graph == eager check at Pong size): the tree's root sum after every iteration in both modes,
and the first iteration where they part.  usage: diag_graph_eager.py [iters] [blas]
(blas: the learner's FC1 forward on hipBLASLt instead of rth_fc_x9, to bisect)"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from reth_amd import fused_learner  # noqa: E402
from reth_amd.apex import ApexConfig, ApexDQN  # noqa: E402

iters = int(sys.argv[1]) if len(sys.argv) > 1 else 14
if "blas" in sys.argv:
    fused_learner.fc1_relu = lambda x, w, b, out=None, owner=None: torch._addmm_activation(b, x, w.t())
dev = torch.device("cuda", 0)
kw = dict(n_actors=256, num_actions=6, capacity=1_000_000)
prefill = (1_000_000 - 256 * 10) // 4
runs = {}
for graph in (False, True):
    ax = ApexDQN(ApexConfig(batch_size=512, hip_graph=graph, seed=4, learning_rate=0.0, **kw), device=dev)
    ax.prefill(prefill)
    rec = []
    for k in range(iters):
        ax.iteration()
        torch.cuda.synchronize()
        s, m, v = ax.replay.tree.export()
        rec.append((float(s[0]), ax.updates, ax._graphs is not None))
    runs[graph] = rec
    ax.close()
    del ax
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
for k, (e, g) in enumerate(zip(runs[False], runs[True])):
    print(k, "eager", e, "graph", g, "SAME" if e[0] == g[0] else "DIFF", flush=True)
