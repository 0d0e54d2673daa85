import sys, torch
sys.path.insert(0, ".")
from reth_amd.apex import ApexConfig, ApexDQN
for graph in (False, True):
    cfg = ApexConfig(n_actors=256, num_actions=6, capacity=100_000, batch_size=512, hip_graph=graph, seed=3)
    ax = ApexDQN(cfg, device="cuda:0")
    ax.prefill(50_000)
    torch.cuda.synchronize()
    print("graph", graph, "after prefill", ax.replay.info(), flush=True)
    for i in range(30):
        ax.iteration()
        torch.cuda.synchronize()
        print(i, ax.replay.info(), ax.actors.pushes, ax.updates, ax._graphs is not None, flush=True)
    ax.close()
