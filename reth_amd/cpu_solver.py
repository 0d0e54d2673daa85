"""DQNSolver on host torch: the reference's CPU configurations.

BASELINE.json configs[0] (CartPole-v1, uniform replay, "CPU torch, no GPU") and the apex
worker's `get_solver(config, device="cpu")` (test/apex-dqn/worker.py:28: each actor process
keeps a CPU copy for act / calc_loss) run the solver on the host.  `DQNSolver(...,
device="cpu")` builds this class; every device other than the CPU gets the HIP solver
(solver.DQNSolver), which never falls back here.

Same interface and arithmetic as reth/reth/algorithm/dqn/dqn_solver.py:14-143: Q(s0)[a]
(a gather selects exactly what the one-hot product-sum does), the double-Q target
r + gamma^n * Q_tgt(s1)[argmax_a Q(s1)] * (1 - done) with gamma^n a python float applied to
an f32 tensor, smooth-L1 (beta 1) times the IS weights, mean, backward, clip_grad_norm_(clip)
and torch's Adam; the target network follows every `update_target_interval` updates.
"""
import io

import numpy as np
import torch
import torch.nn.functional as F

from .model import make_q_network
from .schedule import Interval


def _tensor(x, dtype):
    if torch.is_tensor(x):
        return x.to(device="cpu", dtype=dtype)
    return torch.as_tensor(np.asarray(x), dtype=dtype)


class CpuDQNSolver:
    def __init__(self, observation_space, action_space, models=None, gamma=0.99, clip_value=40, double_q=True,
                 dueling=True, learning_rate=5e-5, adam_epsilon=1e-8, update_target_interval=150, device="cpu",
                 n_step=1, **_ignored):
        self.device = torch.device("cpu")
        obs_shape = tuple(observation_space.shape)
        self.num_actions = int(action_space.n)
        if models is None:
            q = make_q_network(obs_shape, self.num_actions, dueling)
            tq = make_q_network(obs_shape, self.num_actions, dueling)
            models = {"q_network": q, "target_q_network": tq,
                      "optimizer": torch.optim.Adam(q.parameters(), lr=learning_rate, eps=adam_epsilon)}
        self.q_network = models["q_network"].to(self.device)
        self.target_q_network = models["target_q_network"].to(self.device)
        self.optimizer = models.get("optimizer") or torch.optim.Adam(
            self.q_network.parameters(), lr=models.get("learning_rate", learning_rate),
            eps=models.get("adam_epsilon", adam_epsilon))
        self.update_target()
        self.clip_value, self.double_q, self.gamma, self.n_step = clip_value, double_q, gamma, n_step
        self._update_target_interval = (Interval(self.update_target, update_target_interval)
                                        if update_target_interval is not None else None)

    def update_target(self):
        self.target_q_network.load_state_dict(self.q_network.state_dict())

    def _td_error(self, batch):
        s0, a, r, s1, done = batch
        s0, s1 = _tensor(s0, torch.float32), _tensor(s1, torch.float32)
        a, r, done = _tensor(a, torch.int64).view(-1), _tensor(r, torch.float32).view(-1), \
            _tensor(done, torch.float32).view(-1)
        q = self.q_network(s0).gather(1, a[:, None])[:, 0]
        q_next = self.target_q_network(s1)
        chooser = self.q_network(s1) if self.double_q else q_next
        best = q_next.gather(1, torch.argmax(chooser, 1)[:, None])[:, 0]
        target = r + (self.gamma ** self.n_step) * best * (1 - done)
        return q - target.detach()

    def calc_loss(self, batch):
        """|td| without an update (dqn_solver.py:100-102)"""
        with torch.no_grad():
            return self._td_error(batch).abs()

    def update(self, batch, weights=None):
        td = self._td_error(batch)
        out = td.detach().abs()
        loss = F.smooth_l1_loss(td, torch.zeros_like(td), reduction="none")
        if weights is not None:
            loss = loss * _tensor(weights, torch.float32).view(-1)
        loss = loss.mean()
        self.optimizer.zero_grad()
        loss.backward()
        if self.clip_value >= 0:
            torch.nn.utils.clip_grad_norm_(self.q_network.parameters(), self.clip_value)
        self.optimizer.step()
        if self._update_target_interval is not None:
            self._update_target_interval()
        return out

    def update_device(self, batch, weights=None):
        """Trainer.train's entry point (the device-resident result is the host one here)"""
        return self.update(batch, weights)

    @torch.no_grad()
    def act(self, state):
        x = _tensor(state, torch.float32).unsqueeze(0)
        return int(torch.argmax(self.q_network(x), dim=1).item())

    def load_weights(self, stream):
        self.q_network.load_state_dict(torch.load(stream, map_location="cpu", weights_only=True))
        self.update_target()

    def save_weights(self, stream=None):
        if stream is None:
            stream = io.BytesIO()
        torch.save(self.q_network.state_dict(), stream)
        return stream
