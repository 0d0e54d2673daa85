"""End-to-end Ape-X on one GPU at a small size: actors -> HBM replay -> learner -> weights,
plus the graft smoke entry point."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_apex_small_end_to_end(dev):
    from reth_amd.apex import ApexConfig, ApexDQN

    cfg = ApexConfig(n_actors=16, capacity=4096, batch_size=32, sample_start=64, send_weights_interval=5,
                     recv_weights_interval=8, update_target_interval=10, p_done=0.05, seed=1)
    ax = ApexDQN(cfg, device=dev)
    for _ in range(60):
        ax.iteration()
    torch.cuda.synchronize()
    size, tail, cnt, calls = ax.replay.info()
    assert size == 16 * (60 - cfg.n_step) and ax.env_steps == 16 * 60
    assert ax.updates > 40 and ax.slot.version == ax.updates // 5
    assert ax.subscriber.loaded_version > 0
    assert all(torch.isfinite(p).all() for p in ax.solver.q_network.parameters())
    # the replay's a/r/done columns hold what the actors emitted last
    out = ax.replay.gather(torch.arange(tail - 16, tail, device=dev))
    assert torch.equal(out[1], ax.actors.row_a) and torch.equal(out[2], ax.actors.row_r)
    assert torch.equal(out[0], ax.actors.frames[ax.actors.row_s0].float())
    assert torch.equal(out[3], ax.actors.frames[ax.actors.row_s1].float())
    ax.close()


def test_prefill_then_learn(dev):
    from reth_amd.apex import ApexConfig, ApexDQN

    cfg = ApexConfig(n_actors=8, capacity=2000, batch_size=64, seed=2)
    ax = ApexDQN(cfg, device=dev)
    ax.prefill(2000, chunk=700)
    assert ax.replay.info()[0] == 2000 and ax.svc.ready()
    for _ in range(5):
        ax.iteration()
    assert ax.updates == 5
    ax.close()


def test_graft_smoke(dev):
    import __graft_entry__

    __graft_entry__.smoke()
