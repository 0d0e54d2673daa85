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

    # ---------------------------------------------------------------- fused heads path
    # The same function with the two dueling branches merged: FC1 of both branches is one
    # 3136 -> 512 GEMM with the bias and ReLU fused into hipBLASLt's epilogue, and the two
    # output layers are one block-diagonal 512 -> A+1 GEMM.  It returns the raw heads
    # [B, A+1] = (advantages, value); the HIP consumers (rth_td_huber, rth_eps_greedy in
    # dueling mode) form Q = (V + A) - mean(A) themselves.  The parameters (and state_dict)
    # stay the reference's; the merged weights are either built per call (training, autograd
    # flows back into the branch parameters) or cached (`freeze_heads`, inference copies whose
    # weights change only at refresh points: target sync, actor weight reload).
    def _merged_head_weights(self):
        a0, v0, a2, v2 = self.fc_adv[0], self.fc_value[0], self.fc_adv[2], self.fc_value[2]
        w1 = torch.cat([a0.weight, v0.weight])
        b1 = torch.cat([a0.bias, v0.bias])
        A, H = a2.weight.shape
        w2 = torch.cat([torch.cat([a2.weight, a2.weight.new_zeros(A, H)], 1),
                        torch.cat([v2.weight.new_zeros(1, H), v2.weight], 1)])
        b2 = torch.cat([a2.bias, v2.bias])
        return w1, b1, w2, b2

    @torch.no_grad()
    def freeze_heads(self):
        """(re)build the cached merged weights in place (stable storage for graph replay)"""
        merged = self._merged_head_weights()
        if getattr(self, "_frozen", None) is None:
            self._frozen = [t.clone() for t in merged]
        else:
            for dst, src in zip(self._frozen, merged):
                dst.copy_(src)

    def forward_heads(self, x, merged=None):
        if not self.dueling:
            raise ValueError("forward_heads needs the dueling network")
        if merged is None:
            merged = self._frozen if getattr(self, "_frozen", None) is not None else self._merged_head_weights()
        w1, b1, w2, b2 = merged
        h = self.features(x).flatten(1)
        h = _LinearReLU.apply(h, w1, b1)
        return torch.addmm(b2, h, w2.t())


class _LinearReLU(torch.autograd.Function):
    """relu(x @ w.T + b) as ONE hipBLASLt GEMM with a bias+ReLU epilogue
    (torch._addmm_activation, which has no autograd formula of its own); the backward is
    the one autograd derives for linear -> relu (threshold on the output, addmm grads)."""

    @staticmethod
    def forward(ctx, x, w, b):
        out = torch._addmm_activation(b, x, w.t())
        ctx.save_for_backward(x, w, out)
        return out

    @staticmethod
    def backward(ctx, g):
        x, w, out = ctx.saved_tensors
        g = torch.ops.aten.threshold_backward(g, out, 0)
        gx = g.mm(w) if ctx.needs_input_grad[0] else None
        gw = g.t().mm(x) if ctx.needs_input_grad[1] else None
        gb = g.sum(0) if ctx.needs_input_grad[2] else None
        return gx, gw, gb


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
