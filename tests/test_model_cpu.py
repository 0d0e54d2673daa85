"""Q-network parity with the reference's torch model on CPU (architecture, parameter
names, seeded initialisation, forward values): the learner's network IS the reference's
network, so the GPU parity tests can start from identical weights."""
import numpy as np
import pytest
import torch

from reth_amd.model import DQNNetwork, MLP_DQNNetwork, make_q_network


@pytest.mark.parametrize("name", ["dqn_pong_b8.npz", "dqn_pong_b32.npz"])
def test_pong_net_init_and_forward(golden, name):
    g = golden(name)
    torch.manual_seed(int(g["seed"]))
    net = make_q_network((4, 84, 84), 6)
    make_q_network((4, 84, 84), 6)  # the reference builds the target net second
    sd = net.state_dict()
    assert list(sd.keys()) == [str(x) for x in g["param_names"]]
    sums = np.array([float(v.double().sum()) for v in sd.values()])
    np.testing.assert_allclose(sums, g["init_sum"], rtol=1e-12, atol=1e-15)  # threaded sum order
    with torch.no_grad():
        q = net(torch.as_tensor(g["s0"]).float()).numpy()
    # CPU conv summation order depends on the thread count: north_star's 1e-5 bar
    np.testing.assert_allclose(q, g["q_s0"], rtol=1e-5, atol=1e-5)
    assert sum(p.numel() for p in net.parameters()) == 1_685_927  # SURVEY §8(a) a14, A=6


def test_cartpole_mlp_init(golden):
    g = golden("dqn_cartpole_b64.npz")
    torch.manual_seed(int(g["seed"]))
    net = make_q_network((4,), 2)
    assert isinstance(net, MLP_DQNNetwork)
    for k, v in net.state_dict().items():
        np.testing.assert_array_equal(v.numpy(), g[f"init/{k}"])


def test_non_dueling_head_shapes():
    net = DQNNetwork((4, 84, 84), 4, dueling=False)
    assert net(torch.zeros(2, 4, 84, 84)).shape == (2, 4)
    assert "fc.2.weight" in net.state_dict()
