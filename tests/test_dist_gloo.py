"""N > 1 path on CPU: world_size-2 gloo.  Each rank computes gradients on its own shard's
batch; GradAllReduce (the learner's single exchange step) must leave identical gradients on
both ranks equal to the average, so clip + Adam keep the replicas bit-identical."""
import os
import socket

import numpy as np
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank_main(rank, world, port, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    from reth_amd.dist import GradAllReduce, init_from_env
    from reth_amd.model import MLP_DQNNetwork

    r, w = init_from_env(backend="gloo")
    assert (r, w) == (rank, world)
    torch.manual_seed(0)
    net = MLP_DQNNetwork((4,), 2)
    opt = torch.optim.Adam(net.parameters(), lr=1e-3, eps=1.5e-4)
    hook = GradAllReduce()
    params = list(net.parameters())
    for step in range(3):
        g = torch.Generator().manual_seed(100 * step + rank)  # different data per rank
        x = torch.randn(16, 4, generator=g)
        loss = net(x).pow(2).mean()
        opt.zero_grad()
        loss.backward()
        local = [p.grad.clone() for p in params]
        if step == 1:  # the captured learner's form: two buckets (heads | rest), reduced separately
            grads = [p.grad for p in params]
            hook.reduce(grads[:2], key=("bucket", 0))
            hook.reduce(grads[2:], key=("bucket", 1))
        else:
            hook(params)
        gathered = [[torch.empty_like(t) for _ in range(world)] for t in local]
        for t, buf in zip(local, gathered):
            dist.all_gather(buf, t)
        for p, buf in zip(params, gathered):
            torch.testing.assert_close(p.grad, sum(buf) / world, rtol=1e-6, atol=1e-7)
        torch.nn.utils.clip_grad_norm_(params, 40)
        opt.step()
    flat = torch.cat([p.detach().flatten() for p in params]).numpy()
    np.save(os.path.join(out_dir, f"rank{rank}.npy"), flat)
    dist.barrier()
    dist.destroy_process_group()


def test_grad_allreduce_world2(tmp_path):
    world = 2
    mp.spawn(_rank_main, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    a, b = np.load(tmp_path / "rank0.npy"), np.load(tmp_path / "rank1.npy")
    assert np.array_equal(a, b)  # replicas stay bit-identical


def test_grad_allreduce_forced_one_rank():
    """GradAllReduce(force=True) runs its collective in a one-rank group (the single-GPU RCCL
    rehearsal, tests/test_rccl_gpu.py) -- averaging over one rank leaves the gradients as they
    were; without force a one-rank group is skipped"""
    import socket

    import torch
    import torch.distributed as dist

    from reth_amd.dist import GradAllReduce

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1)
    try:
        g = [torch.randn(5, 3), torch.randn(7)]
        want = [t.clone() for t in g]
        hook = GradAllReduce(force=True)
        assert hook._active()
        hook.reduce(g)
        assert all(torch.equal(a, b) for a, b in zip(g, want))
        assert hook._flat  # the flat buffer was built: the collective ran
        assert not GradAllReduce()._active()
    finally:
        dist.destroy_process_group()
