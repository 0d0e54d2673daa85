"""DQN solver on MI355X: reth.algorithm.DQNSolver's interface, fused HIP TD/Huber op.

Reference: reth/reth/algorithm/dqn/dqn_solver.py:14-143 (and algorithm/algorithm.py:6-30).

The Q-network's forward runs on hand-written HIP kernels (model.py: the conv torso in
rth_conv_bias_relu, FC1 in rth_fc_x9, FC2 in rth_heads_fc2); the dueling Nature-DQN's learner
update is the explicit kernel sequence of fused_learner.py (HIP data gradients, HIP weight
gradients of every conv layer, the fused TD / FC2 backward, clip + Adam with the norm from the
backward; only FC1's two backward GEMMs run on hipBLASLt), other networks go through
torch.autograd.  The TD error,
double-Q target, Huber loss, IS weighting, mean, |td| and the gradient with respect to Q(s0)
are ONE HIP kernel (rth_td_huber) wrapped as an autograd Function on the autograd path, so
  * the loss' backward starts from the kernel's d(loss)/d(Q(s0)) -- no chain of small torch
    ops and their backward kernels;
  * |td| stays in HBM for the priority update (update_device); the reference-compatible
    update() still returns it as a CPU tensor (`td_error.detach().cpu().abs()`, :109).
"""
import io

import numpy as np
import torch

from . import _lib, fused_learner
from ._lib import call, ptr, stream_ptr
from .model import default_models
from .optim import ClipAdam
from .replay import FrameStacks
from .schedule import Interval


class Discrete:
    """minimal gym.spaces.Discrete (gym is not part of this image)"""

    def __init__(self, n):
        self.n = int(n)


class Box:
    """minimal gym.spaces.Box"""

    def __init__(self, low, high, shape, dtype=None):
        self.low, self.high, self.shape = low, high, tuple(shape)


def _check_device(device):
    dev = torch.device(device if device is not None else "cuda")
    if dev.type != "cuda":
        raise ValueError(f"reth_amd.DQNSolver runs on the GPU (HIP) only, got device={dev}; "
                         "actors are vectorised on the device (reth_amd.actors)")
    if not torch.cuda.is_available():
        raise RuntimeError("no HIP device visible")
    return torch.device("cuda", dev.index if dev.index is not None else torch.cuda.current_device())


def td_huber_forward(q_s0, q_s1_online, q_s1_target, a, r, done, isw, gamma_n, double_q, want_dq, dueling=False):
    """One rth_td_huber launch -> (loss[1], td_abs[B], dq or None).  dueling: the q inputs are
    raw heads [B, A+1] (advantages, value) and dq is d(loss)/d(heads)."""
    B, W = q_s0.shape
    A = W - int(bool(dueling))
    for t, name in ((q_s0, "q_s0"), (q_s1_target, "q_s1_target")):
        if t.dtype != torch.float32 or not t.is_cuda or t.shape != (B, W):
            raise ValueError(f"{name} must be a float32 device tensor of shape {(B, W)}")
    if double_q and (q_s1_online is None or q_s1_online.shape != (B, W)):
        raise ValueError("double_q needs q_s1_online of the same shape")
    dev = q_s0.device
    q0 = q_s0.detach().contiguous()
    q1o = None if q_s1_online is None else q_s1_online.detach().contiguous()
    q1t = q_s1_target.detach().contiguous()
    a = a.to(device=dev, dtype=torch.int64).contiguous().view(-1)
    r = r.to(device=dev, dtype=torch.float32).contiguous().view(-1)
    done = done.to(device=dev, dtype=torch.float32).contiguous().view(-1)
    if isw is not None:
        isw = isw.to(device=dev, dtype=torch.float64).contiguous().view(-1)
    if a.numel() != B or r.numel() != B or done.numel() != B or (isw is not None and isw.numel() != B):
        raise ValueError("batch columns disagree in length")
    td_abs = torch.empty(B, dtype=torch.float32, device=dev)
    loss = torch.empty(1, dtype=torch.float32, device=dev)
    dq = torch.empty((B, W), dtype=torch.float32, device=dev) if want_dq else None
    call("rth_td_huber", ptr(q0), ptr(q1o), ptr(q1t), ptr(a), ptr(r), ptr(done), ptr(isw), B, A,
         float(gamma_n), int(bool(double_q)), int(bool(dueling)), None, ptr(td_abs), None, ptr(loss), ptr(dq),
         stream_ptr())
    return loss, td_abs, dq


class _TDHuber(torch.autograd.Function):
    @staticmethod
    def forward(ctx, q_s0, q_s1_online, q_s1_target, a, r, done, isw, gamma_n, double_q, dueling):
        loss, td_abs, dq = td_huber_forward(q_s0, q_s1_online, q_s1_target, a, r, done, isw, gamma_n, double_q,
                                            want_dq=True, dueling=dueling)
        ctx.save_for_backward(dq)
        ctx.mark_non_differentiable(td_abs)
        return loss.view(()), td_abs

    @staticmethod
    def backward(ctx, g_loss, g_td):
        (dq,) = ctx.saved_tensors
        return dq * g_loss, None, None, None, None, None, None, None, None, None


def td_huber_loss(q_s0, q_s1_online, q_s1_target, a, r, done, isw, gamma_n, double_q=True, dueling=False):
    """(mean IS-weighted Huber loss [differentiable w.r.t. q_s0], |td| [B])"""
    return _TDHuber.apply(q_s0, q_s1_online, q_s1_target, a, r, done, isw, gamma_n, double_q, dueling)


class Algorithm:
    """reth/reth/algorithm/algorithm.py:6-30 (device defaults to the current GPU)."""

    def __init__(self, device=None):
        self.device = _check_device(device)

    def update(self, batch, weights=None):
        raise NotImplementedError

    def act(self, state):
        raise NotImplementedError

    def load_weights(self, stream):
        raise NotImplementedError

    def save_weights(self, stream=None):
        raise NotImplementedError


class DQNSolver(Algorithm):
    def __new__(cls, *args, device=None, **kwargs):
        # device="cpu": the reference's host configuration (cpu_solver.CpuDQNSolver; BASELINE
        # configs[0], the apex worker's actor copy) -- an explicit choice, never a fallback
        if device is not None and torch.device(device).type == "cpu":
            from .cpu_solver import CpuDQNSolver

            return CpuDQNSolver(*args, device=device, **kwargs)
        return super().__new__(cls)

    """reth/reth/algorithm/dqn/dqn_solver.py:14-143 with the same constructor arguments.

    grad_hook(params) runs between backward and clip/Adam: the data-parallel learner uses it
    for the RCCL gradient all-reduce (reth_amd/dist.py).  channels_last keeps the conv
    weights NHWC (MIOpen's fp32 implicit-GEMM kernels are NHWC: no transposes)."""

    def __init__(self, observation_space, action_space, models=None, gamma=0.99, clip_value=40, double_q=True,
                 dueling=True, learning_rate=5e-5, adam_epsilon=1e-8, update_target_interval=150, device=None,
                 n_step=1, fused_adam=True, grad_hook=None, channels_last=False, capturable=False):
        super().__init__(device)
        obs_shape = tuple(observation_space.shape)
        self.num_actions = int(action_space.n)
        if models is None:
            models = default_models(obs_shape, self.num_actions, dueling, learning_rate, adam_epsilon, fused_adam)
        assert models["q_network"] is not None and models["target_q_network"] is not None
        fmt = torch.channels_last if channels_last and len(obs_shape) == 3 else torch.preserve_format
        self.q_network = models["q_network"].to(self.device, memory_format=fmt)
        self.target_q_network = models["target_q_network"].to(self.device, memory_format=fmt)
        self.target_q_network.requires_grad_(False)
        if channels_last and len(obs_shape) == 3:
            for net in (self.q_network, self.target_q_network):
                if hasattr(net, "hwc_features"):
                    net.hwc_features = True  # HIP conv torso on channels-last activations (model.py)
        if models.get("optimizer") is not None:
            self.optimizer = models["optimizer"]
        elif models.get("fused_adam", fused_adam):  # clip_grad_norm_ + Adam in one HIP call (optim.py)
            self.optimizer = ClipAdam(self.q_network.parameters(), lr=models.get("learning_rate", learning_rate),
                                      eps=models.get("adam_epsilon", adam_epsilon),
                                      max_norm=clip_value if clip_value >= 0 else None)
        else:  # torch's Adam (the reference's optimizer object)
            kw = {"capturable": True} if capturable else {}  # device step count: graph-capturable
            self.optimizer = torch.optim.Adam(self.q_network.parameters(), lr=models.get("learning_rate", learning_rate),
                                              eps=models.get("adam_epsilon", adam_epsilon), **kw)
        self._params = [p for p in self.q_network.parameters()]
        self._tparams = [p for p in self.target_q_network.parameters()]
        # dueling conv net: merged-heads forward, Q formed inside the TD kernel (model.py)
        self._heads = bool(getattr(self.q_network, "dueling", False) and hasattr(self.q_network, "forward_heads"))
        self.update_target()
        self.clip_value = clip_value
        self.double_q = double_q
        self.gamma = gamma
        self.n_step = n_step
        self.gamma_n = float(np.float32(gamma ** n_step))  # python float -> f32 scalar (:96)
        self.grad_hook = grad_hook
        self._update_target_interval = (Interval(self.update_target, update_target_interval)
                                        if update_target_interval is not None else None)
        # graph replay runs the (host-side) target-sync Interval outside the captured step
        self.auto_target_update = True
        # explicit kernel-sequence gradient pass (fused_learner.py) where it applies; False:
        # torch.autograd over the same forward (the A/B reference)
        self.fused_grads = True
        self.td_mean_acc = None  # Trainer's device mean-|td| accumulator (fused pass adds to it)

    # ------------------------------------------------------------------ target / weights
    @torch.no_grad()
    def update_target(self):
        """target <- online (:65-66), one fused device copy (+ the target's merged heads)"""
        self._target_syncs = getattr(self, "_target_syncs", 0) + 1
        torch._foreach_copy_(self._tparams, self._params)
        if self._heads:
            self.target_q_network.freeze_heads()

    def load_weights(self, stream):
        states = torch.load(stream, map_location=self.device, weights_only=True)
        self.q_network.load_state_dict(states)
        self.update_target()

    def save_weights(self, stream=None):
        if stream is None:
            stream = io.BytesIO()
        torch.save(self.q_network.state_dict(), stream)
        return stream

    # ------------------------------------------------------------------ TD
    def _tensors(self, batch):
        s0, a, r, s1, done = batch
        dev = self.device
        f = lambda x, dt: (x.to(device=dev, dtype=dt, non_blocking=True) if torch.is_tensor(x)
                           else torch.as_tensor(np.asarray(x), dtype=dt).to(dev, non_blocking=True))
        # uint8 frame stacks stay uint8 when the HIP conv torso reads them (the f32 frames the
        # reference feeds hold exactly these integers); anything else is cast as the reference does
        fr = lambda x: x if self._u8_frames(x) else f(x, torch.float32)
        return fr(s0), f(a, torch.int64), f(r, torch.float32), fr(s1), f(done, torch.float32)

    def _u8_frames(self, x):
        net = self.q_network
        return ((torch.is_tensor(x) or isinstance(x, FrameStacks)) and x.dtype == torch.uint8 and x.is_cuda
                and self._heads
                and getattr(net, "hwc_features", False) and getattr(net, "hip_conv", False))

    def target_heads(self, s1):
        """the target network's output on s1 (raw dueling heads with the HIP TD kernel): a
        function of the target weights only, so it may be computed ahead of the update that
        consumes it as long as no target sync falls in between (compute_grads(q1t=...))"""
        if not self._u8_frames(s1):
            s1 = (s1 if torch.is_tensor(s1) else torch.as_tensor(np.asarray(s1))).to(self.device, torch.float32)
        with torch.no_grad():
            return self.target_q_network.forward_heads(s1) if self._heads else self.target_q_network(s1)

    def _forward_targets(self, s1, merged=None, packed=None, q1t=None):
        with torch.no_grad():
            if self._heads:  # raw dueling heads; the TD kernel forms Q
                if q1t is None:
                    q1t = self.target_q_network.forward_heads(s1)
                q1o = None
                if self.double_q:
                    m = [t.detach() for t in merged] if merged is not None else None
                    q1o = self.q_network.forward_heads(s1, m, packed=packed)
            else:
                if q1t is None:
                    q1t = self.target_q_network(s1)
                q1o = self.q_network(s1) if self.double_q else None
        return q1o, q1t

    def calc_loss_device(self, batch):
        """|td| on the device without an update (:100-102)"""
        s0, a, r, s1, done = self._tensors(batch)
        with torch.no_grad():
            q0 = self.q_network.forward_heads(s0) if self._heads else self.q_network(s0)
        q1o, q1t = self._forward_targets(s1)
        _, td_abs, _ = td_huber_forward(q0, q1o, q1t, a, r, done, None, self.gamma_n, self.double_q, want_dq=False,
                                        dueling=self._heads)
        return td_abs

    def calc_loss(self, batch):
        return self.calc_loss_device(batch).cpu()

    def compute_grads(self, batch, weights=None, q1t=None, mid=None, probe=None, prenorm=False):
        """dqn_solver.py:104-117: forward passes, fused TD/Huber, backward -> |td| (device).
        q1t: the target network's output on this batch's s1 if already computed
        (target_heads), else it is computed here.  mid: gradient-bucket callback of the
        explicit pass (fused_learner.dueling_grads); the autograd path never calls it.
        prenorm: the caller runs apply_grads next on these gradients (no all-reduce in
        between): the explicit pass may write clip_grad_norm_'s partials and advance Adam's
        step count itself (fused_learner.NORM_IN_BACKWARD)"""
        s0, a, r, s1, done = self._tensors(batch)
        isw = None if weights is None else (weights if torch.is_tensor(weights) else torch.as_tensor(np.asarray(weights)))
        if self.fused_grads and self._heads and fused_learner.eligible(self.q_network, s0, s1):
            loss, td_abs = fused_learner.dueling_grads(self, s0, a, r, s1, done, isw, q1t, td_acc=self.td_mean_acc,
                                                        mid=mid, probe=probe, prenorm=prenorm)
            if self.td_mean_acc is not None:
                td_abs._rth_mean_tracked = True
            self.last_loss = loss.detach()
            return td_abs
        merged = packed = None
        if self._heads:  # merged dueling head weights (and packed conv weights of the HIP torso),
            # built once per weight version and shared by both online passes
            merged = self.q_network._merged_head_weights()
            if getattr(self.q_network, "hwc_features", False) and merged[0].is_cuda:
                with torch.no_grad():
                    packed = self.q_network.pack_convs()
            q0 = self.q_network.forward_heads(s0, merged, packed=packed)
        else:
            q0 = self.q_network(s0)
        q1o, q1t = self._forward_targets(s1, merged, packed, q1t)
        loss, td_abs = td_huber_loss(q0, q1o, q1t, a, r, done, isw, self.gamma_n, self.double_q, self._heads)
        # grads set to None: backward hands each parameter its gradient buffer directly
        # (no accumulate-add into a zeroed .grad, no zero fill); inside a captured HIP graph
        # the buffers come from the graph's pool at fixed addresses
        self.optimizer.zero_grad(set_to_none=True)
        loss.backward()
        self.last_loss = loss.detach()
        return td_abs

    def apply_grads(self, probe=None):
        """dqn_solver.py:118-123: clip_grad_norm_ -> Adam -> target Interval.  probe: as in
        fused_learner.dueling_grads, handed [("clip_adam", launch)] to issue itself -- with
        last=True when nothing follows it (no automatic target update), so a graph capture cut
        there does not open an empty part"""
        if isinstance(self.optimizer, ClipAdam):
            if probe is not None:
                tail = self.auto_target_update and self._update_target_interval is not None
                probe([("clip_adam", self.optimizer.step_launch())], last=not tail)
            else:
                self.optimizer.step()  # clips to optimizer.max_norm (= clip_value) itself
        else:
            if self.clip_value >= 0:
                torch.nn.utils.clip_grad_norm_(self._params, self.clip_value, foreach=True)
            self.optimizer.step()
        if self.auto_target_update and self._update_target_interval is not None:
            self._update_target_interval()

    def update_device(self, batch, weights=None, q1t=None):
        """DQNSolver.update (:104-124) returning |td| as a device tensor (no host sync)."""
        td_abs = self.compute_grads(batch, weights, q1t, prenorm=self.grad_hook is None)
        if self.grad_hook is not None:
            self.grad_hook(self._params)
        self.apply_grads()
        return td_abs

    def update(self, batch, weights=None):
        return self.update_device(batch, weights).cpu()

    # ------------------------------------------------------------------ acting
    @torch.no_grad()
    def act(self, state):
        x = torch.as_tensor(np.asarray(state), dtype=torch.float32).to(self.device).unsqueeze(0) \
            if not torch.is_tensor(state) else state.to(self.device, torch.float32).unsqueeze(0)
        return int(torch.argmax(self.q_network(x), dim=1).item())


def get_solver(name, **kwargs):
    """reth/reth/algorithm/__init__.py:17-21 (only the DQN path is rebuilt)"""
    if name != "dqn":
        raise NotImplementedError(f"solver {name!r}: only 'dqn' is on the Ape-X hot path")
    return DQNSolver(**kwargs)
