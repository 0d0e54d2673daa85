"""Data-parallel learner on the GPU: two ranks (gloo, both on cuda:0) run the captured Ape-X
loop on different data (rank-seeded actors and replay shards).  The learner graph is cut at
the gradient buckets and the merged heads' bucket is all-reduced on a side stream while the
conv backward replays (ApexDQN._learner_replay); if any bucket missed its reduce, or the
final part read a bucket before its reduce finished, the replicas would drift apart.  The
N > 1 contract: bit-identical parameters on every rank after every update."""
import os
import socket

import pytest
import torch

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _rank_main(rank, world, port, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    import torch.distributed as dist

    from reth_amd.apex import ApexConfig, ApexDQN
    from reth_amd.dist import init_from_env

    r, w = init_from_env(backend="gloo")
    assert (r, w) == (rank, world)
    torch.cuda.set_device(0)
    cfg = ApexConfig(n_actors=16, capacity=1024, batch_size=32, sample_start=64, seed=4, hip_graph=True,
                     update_target_interval=3)
    ax = ApexDQN(cfg, device="cuda:0", rank=rank, world=world)
    init = torch.cat([p.detach().flatten() for p in ax.solver._params]).clone()
    for _ in range(30):
        ax.iteration()
    torch.cuda.synchronize()
    G = ax._graphs
    parts = {v: len(G["learn"][v]) for v in G["learn"]} if G is not None else {}
    flat = torch.cat([p.detach().flatten() for p in ax.solver._params])
    torch.save({"params": flat.cpu(), "init": init.cpu(), "parts": parts, "updates": ax.updates,
                "modes": dict(ax.actor_modes)}, os.path.join(out_dir, f"rank{rank}.pt"))
    ax.close()
    dist.destroy_process_group()


def test_two_rank_graph_learner_keeps_replicas_identical(tmp_path):
    import torch.multiprocessing as mp

    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    mp.spawn(_rank_main, args=(2, _free_port(), str(tmp_path)), nprocs=2, join=True)
    res = [torch.load(tmp_path / f"rank{r}.pt", weights_only=True) for r in range(2)]
    for x in res:
        assert x["updates"] > 20
        assert x["parts"] and all(n == 3 for n in x["parts"].values()), x["parts"]  # graph replay, bucket cuts
        assert not torch.equal(x["params"], x["init"])
    assert torch.equal(res[0]["params"], res[1]["params"])
