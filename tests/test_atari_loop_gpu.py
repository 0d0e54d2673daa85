"""SURVEY §8(f) row 2 on the loop's path: the Ape-X actors in the Atari env mode (raw
210x160 RGB frame pairs -> MaxAndSkip max, gray, INTER_AREA 84x84, FrameStack; reference
reth/reth/env/util.py:121-209, 259-274) write the stacks the acting batch and the replay
read.  Each step's stacks are checked against the oracle's OpenCV restatement
(oracle.warp_frame) driven through a FrameStack deque per actor; the captured loop equals the
eager one."""
from collections import deque

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _actor_net(dev):
    from reth_amd.model import DQNNetwork

    torch.manual_seed(0)
    net = DQNNetwork((4, 84, 84), 6).to(dev, memory_format=torch.channels_last)
    net.requires_grad_(False)
    net.hwc_features = True
    return net


@pytest.mark.parametrize("env", ["atari", "atari-h2d"])
def test_atari_actor_stacks_vs_oracle(dev, orc, env):
    from reth_amd.actors import VecActors

    N, T = 6, 14
    act = VecActors(N, 6, device=dev, seed=3, p_done=0.25, channels_last=True, env=env)
    net = _actor_net(dev)
    torch.cuda.synchronize()
    ring = act.ring
    fr = lambda h: act.frames[h].cpu().numpy()
    cur = act.cur_slot.cpu().numpy()
    stacks = [deque(fr(i * ring + cur[i]), maxlen=4) for i in range(N)]  # the initial observations
    dones = 0
    for t in range(T):
        act.step_fused(net)
        torch.cuda.synchronize()
        raw = act.raw.cpu().numpy()
        raw_reset = act.raw_reset.cpu().numpy()
        s0h, s1h = act.s0_h.cpu().numpy(), act.s1_h.cpu().numpy()
        done, cur = act.done.cpu().numpy(), act.cur_slot.cpu().numpy()
        for i in range(N):
            assert np.array_equal(fr(s0h[i]), np.stack(stacks[i])), (t, i, "s0")
            f = orc.warp_frame(raw[i, 0], raw[i, 1])
            stacks[i].append(f)
            assert np.array_equal(fr(s1h[i]), np.stack(stacks[i])), (t, i, "s1")
            if done[i]:
                dones += 1
                # env.reset(): MaxAndSkip.reset's screen (no pair max, util.py:129-130) warped, then
                # FrameStack.reset's k copies -- a fresh observation, not the terminal one
                rs = raw_reset[i]
                fr0 = orc.warp_frame(rs, rs)
                stacks[i].extend([fr0] * 4)
                assert np.array_equal(fr(i * ring + cur[i]), np.stack(stacks[i])), (t, i, "reset")
                assert not np.array_equal(fr0, f)
            else:
                assert cur[i] * 1 + i * ring == s1h[i]
    assert dones > 0
    if env == "atari-h2d":  # the frames came over PCIe from the pinned host buffer
        assert torch.equal(act.raw.cpu(), act.raw_host)


def test_atari_loop_graph_matches_eager(dev):
    """ApexDQN with env="atari": HIP-graph replay keeps every replay / tree op and every
    stack of the eager schedule (lr = 0 keeps the networks fixed)"""
    from reth_amd.apex import ApexConfig, ApexDQN

    def run(graph):
        cfg = ApexConfig(n_actors=16, capacity=1024, batch_size=32, sample_start=64, learning_rate=0.0, p_done=0.05,
                         seed=4, hip_graph=graph, send_weights_interval=3, recv_weights_interval=4,
                         update_target_interval=5, env="atari")
        ax = ApexDQN(cfg, device=dev)
        for _ in range(30):
            ax.iteration()
        torch.cuda.synchronize()
        assert (ax._graphs is not None) == graph
        s, m, v = ax.replay.tree.export()
        cols = ax.replay.gather(torch.arange(ax.replay.info()[0], device=dev))
        out = [s.cpu(), m.cpu(), v.cpu(), ax.actors.frames.cpu()] + [c.cpu() for c in cols]
        info = ax.replay.info()
        ax.close()
        return out, info

    a, ia = run(False)
    b, ib = run(True)
    assert ia == ib
    names = ["tree sums", "tree mins", "values", "frames", "s0", "a", "r", "s1", "done"]
    for name, x, y in zip(names, a, b):
        assert torch.equal(x, y), (name, int((x != y).sum()))
