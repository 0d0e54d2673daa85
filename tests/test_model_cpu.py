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


def test_freeze_heads_refills_in_place():
    """the merged second layer of a shape rth_heads_fc2 does not build (H not a multiple of
    64) is refilled in the tensors the first freeze allocated: captured graphs keep reading
    the current weights after a target sync / weights reload"""
    net = DQNNetwork((4, 84, 84), 9, hidden_unit=48)
    assert not net._fc2_inplace()
    net.freeze_heads()
    w2, b2 = net._frozen[2], net._frozen[3]
    ptrs = (w2.data_ptr(), b2.data_ptr())
    with torch.no_grad():
        for p in net.parameters():
            p.add_(0.5)
    net.freeze_heads()
    assert (net._frozen[2].data_ptr(), net._frozen[3].data_ptr()) == ptrs
    A, H = 9, 48
    assert torch.equal(net._frozen[2][:A, :H], net.fc_adv[2].weight)
    assert torch.equal(net._frozen[2][A:, H:], net.fc_value[2].weight)
    assert torch.equal(net._frozen[3], torch.cat([net.fc_adv[2].bias, net.fc_value[2].bias]))
    assert net._frozen[0].data_ptr() == net.fc_adv[0].weight.data_ptr()  # FC1: the tied storage


def test_tie_survives_deepcopy_and_assign():
    """FC1's two branch parameters stay row slices of the storage the fast path multiplies by
    after copy.deepcopy and load_state_dict(assign=True)"""
    import copy

    net = DQNNetwork((4, 84, 84), 6)
    H = net.fc_adv[0].weight.shape[0]
    twin = copy.deepcopy(net)
    assert twin._w1s.data_ptr() == twin.fc_adv[0].weight.data_ptr() != net._w1s.data_ptr()
    assert twin.fc_value[0].weight.data_ptr() == twin._w1s[H:].data_ptr()
    sd = {k: v.clone() + 1 for k, v in net.state_dict().items()}
    net.load_state_dict(sd, assign=True)
    with torch.no_grad():
        w1, b1, _, _ = net._merged_head_weights()
    assert w1.data_ptr() == net.fc_adv[0].weight.data_ptr()
    assert torch.equal(w1[:H], sd["fc_adv.0.weight"]) and torch.equal(b1[H:], sd["fc_value.0.bias"])
