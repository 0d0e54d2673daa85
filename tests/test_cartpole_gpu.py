"""C1: the reference's CartPole DQN example (examples/dqn/run.py) end to end on the device
path -- Worker + PrioritizedBuffer (HBM) + DQNSolver (MLP) + Trainer from the same YAML."""
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_cartpole_example_runs(dev):
    import sys

    sys.path.insert(0, os.path.join(ROOT, "examples"))
    import cartpole_dqn

    worker, trainer, buffer = cartpole_dqn.main(max_ts=40)
    assert trainer.cur_step == 40
    assert buffer.size == 1000 + 40 * 64 and worker.cur_step == buffer.size
    # alpha/beta stepped once per sample (prioritized_buffer.py:53-54), beta "0.4,1,100000"
    assert buffer.beta.value() == pytest.approx(0.4 + 0.6 * 40 / 100000)
    s, _, v = buffer.replay.tree.export()
    assert s[0].item() == pytest.approx(v[:buffer.size].sum().item(), rel=1e-9)


def test_cartpole_env_contract():
    from reth_amd.envs import CartPole

    env = CartPole(seed=0)
    s = env.reset()
    assert s.shape == (4,) and np.all(np.abs(s) <= 0.05)
    n = 0
    done = False
    while not done:
        s, r, done, _ = env.step(n % 2)
        n += 1
    assert r == 1.0 and 1 <= n <= 200
