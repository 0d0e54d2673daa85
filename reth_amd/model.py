"""Q-networks (PyTorch-ROCm; MIOpen / hipBLASLt run the conv and linear GEMMs in fp32).

Parameter names, shapes and the order in which modules are constructed match
reth/reth/algorithm/dqn/dqn_model.py:6-71, so
  * state_dicts (and torch.save weight streams, dqn_solver.py:133-143) are interchangeable
    with the reference's, and
  * under the same torch.manual_seed the default initialisation is identical.
"""
import torch
from torch import nn


def conv_out(size, k, s):
    return (size - k) // s + 1


class DQNNetwork(nn.Module):
    """Nature-DQN torso + dueling heads (dqn_model.py:6-56): obs (C, H, W) -> Q[A]."""

    def __init__(self, obs_shape, num_actions, dueling=True, hidden_unit=256):
        super().__init__()
        c, h, w = obs_shape
        self.input_shape, self.num_actions, self.dueling = tuple(obs_shape), num_actions, dueling
        self.features = nn.Sequential(
            nn.Conv2d(c, 32, kernel_size=8, stride=4), nn.ReLU(),
            nn.Conv2d(32, 64, kernel_size=4, stride=2), nn.ReLU(),
            nn.Conv2d(64, 64, kernel_size=3, stride=1), nn.ReLU())
        fh = conv_out(conv_out(conv_out(h, 8, 4), 4, 2), 3, 1)
        fw = conv_out(conv_out(conv_out(w, 8, 4), 4, 2), 3, 1)
        nfeat = 64 * fh * fw
        if dueling:
            self.fc_adv = nn.Sequential(nn.Linear(nfeat, hidden_unit), nn.ReLU(), nn.Linear(hidden_unit, num_actions))
            self.fc_value = nn.Sequential(nn.Linear(nfeat, hidden_unit), nn.ReLU(), nn.Linear(hidden_unit, 1))
        else:
            self.fc = nn.Sequential(nn.Linear(nfeat, 512), nn.ReLU(), nn.Linear(512, num_actions))

    def forward(self, x):
        x = self.features(x).flatten(1)
        if not self.dueling:
            return self.fc(x)
        adv = self.fc_adv(x)
        value = self.fc_value(x)
        return value + adv - adv.mean(dim=1, keepdim=True)  # (value + adv) - mean, :192-193


class MLP_DQNNetwork(nn.Module):
    """dqn_model.py:59-71: obs (D,) -> Q[A] (CartPole)."""

    def __init__(self, obs_shape, num_actions):
        super().__init__()
        self.nn = nn.Sequential(nn.Linear(obs_shape[0], 128), nn.ReLU(inplace=True), nn.Linear(128, 128),
                                nn.ReLU(inplace=True), nn.Linear(128, num_actions))

    def forward(self, x):
        return self.nn(x)


def make_q_network(obs_shape, num_actions, dueling=True):
    """generate_dqn_network (dqn_model.py:74-83): conv net for 3-D observations, MLP otherwise"""
    if len(obs_shape) == 3:
        return DQNNetwork(obs_shape, num_actions, dueling=dueling)
    return MLP_DQNNetwork(obs_shape, num_actions)


def default_models(obs_shape, num_actions, dueling=True, learning_rate=5e-5, adam_epsilon=1e-8, fused_adam=True):
    """generate_dqn_default_models (dqn_model.py:86-99): online net, target net, Adam."""
    q = make_q_network(obs_shape, num_actions, dueling)
    tq = make_q_network(obs_shape, num_actions, dueling)
    return {"q_network": q, "target_q_network": tq, "learning_rate": learning_rate, "adam_epsilon": adam_epsilon,
            "fused_adam": fused_adam}
