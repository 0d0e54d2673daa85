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


def _rank_main(rank, world, port, out_dir, shape):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    import torch.distributed as dist

    from reth_amd.apex import ApexConfig, ApexDQN
    from reth_amd.dist import init_from_env

    r, w = init_from_env(backend="gloo")
    assert (r, w) == (rank, world)
    torch.cuda.set_device(0)
    iters = shape.pop("iters", 30)
    prefill = shape.pop("prefill", False)
    cfg = ApexConfig(sample_start=64, seed=4, hip_graph=True, update_target_interval=3, **shape)
    ax = ApexDQN(cfg, device="cuda:0", rank=rank, world=world)
    if prefill:
        ax.prefill(cfg.capacity)
    info0 = ax.replay.info()
    init = torch.cat([p.detach().flatten() for p in ax.solver._params]).clone()
    for _ in range(iters):
        ax.iteration()
    torch.cuda.synchronize()
    G = ax._graphs
    parts = {v: len(G["learn"][v]) for v in G["learn"]} if G is not None else {}
    flat = torch.cat([p.detach().flatten() for p in ax.solver._params])
    eps = ax.actors.eps.detach().cpu() if torch.is_tensor(getattr(ax.actors, "eps", None)) else None
    torch.save({"params": flat.cpu(), "init": init.cpu(), "parts": parts, "updates": ax.updates,
                "modes": dict(ax.actor_modes), "info0": list(info0), "info": list(ax.replay.info()),
                "env_steps": ax.env_steps, "pushes": ax.actors.pushes, "eps": eps},
               os.path.join(out_dir, f"rank{rank}.pt"))
    ax.close()
    dist.destroy_process_group()


def _run(tmp_path, world, shape):
    import torch.multiprocessing as mp

    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    mp.spawn(_rank_main, args=(world, _free_port(), str(tmp_path), shape), nprocs=world, join=True)
    return [torch.load(tmp_path / f"rank{r}.pt", weights_only=True) for r in range(world)]


def test_two_rank_graph_learner_keeps_replicas_identical(tmp_path):
    res = _run(tmp_path, 2, dict(n_actors=16, capacity=1024, batch_size=32))
    for x in res:
        assert x["updates"] > 20
        assert x["parts"] and all(n == 3 for n in x["parts"].values()), x["parts"]  # graph replay, bucket cuts
        assert not torch.equal(x["params"], x["init"])
    for r, x in enumerate(res[1:], 1):
        assert torch.equal(res[0]["params"], x["params"]), f"rank {r} drifted from rank 0"


@pytest.mark.parametrize("world", [2, 8])
def test_configs3_shape(tmp_path, world):
    """BASELINE configs[3] (bench.py --workload pong --faithful at N > 1): configs[1]'s 256
    actors and 1 M replay rows sharded over the ranks -- at world 8 the driver's 8-GPU shape,
    32 actors and a 125,000-row shard per rank (test/apex-dqn/trainer.py:52-61: K shards of
    C // K), pre-filled; the faithful global batch of 512 (64 per rank); actor_steps_per_update
    = world (each update paired with 256 env steps of its shard).  All ranks share cuda:0 over
    gloo (the one-GPU box; RCCL needs a GPU per rank).  Replicas bit-identical; each shard's
    counters are its own actors' rows and its own learner's samples; the ranks' actors take
    disjoint slices of the global epsilon ladder (worker.py:26 over all 256 actors)."""
    n_act, cap, B, iters = 256 // world, 1_000_000 // world, 512 // world, 12
    res = _run(tmp_path, world, dict(n_actors=n_act, capacity=cap, batch_size=B, actor_steps_per_update=world,
                                     iters=iters, prefill=True))
    for x in res:
        size0, tail0, cnt0, calls0, steps0 = x["info0"]
        size, tail, cnt, calls, steps = x["info"]
        assert size0 == size == cap and tail0 == 0  # prefilled to capacity: the FIFO wrapped to slot 0
        assert x["updates"] == iters and steps == x["updates"] and calls == x["updates"] + 1
        assert x["env_steps"] == n_act * world * iters
        appended = n_act * (x["pushes"] - 3 - 1)  # n-step warm-up, then one step of fused-actor lag
        assert tail == appended % cap
        assert x["parts"] and all(n == 3 for n in x["parts"].values())
        assert not torch.equal(x["params"], x["init"])
    for r, x in enumerate(res[1:], 1):  # every replica, not just the first pair
        assert torch.equal(res[0]["params"], x["params"]), f"rank {r} of {world} drifted from rank 0"
    if res[0]["eps"] is not None:
        from reth_amd.actors import apex_epsilons

        ladder = torch.as_tensor(apex_epsilons(n_act * world))
        for r, x in enumerate(res):
            assert torch.equal(x["eps"], ladder[r * n_act:(r + 1) * n_act].to(x["eps"].dtype))
