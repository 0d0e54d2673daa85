"""clip_grad_norm_ + Adam as one HIP call (rth_clip_adam) for the learner update.

Reference: reth/reth/algorithm/dqn/dqn_solver.py:118-121 (clip_grad_norm_(clip_value) then
torch.optim.Adam.step(), torch/optim/adam.py's single-tensor math with the reference's
defaults: betas (0.9, 0.999), no weight decay, no amsgrad).  The optimizer keeps Adam's
state layout (state[p]["exp_avg"], ["exp_avg_sq"], ["step"]) so it reads like torch's; the
step count is a device tensor, so the update is capturable in a HIP graph.
"""
import ctypes

import torch

from . import _lib
from ._lib import call, ptr, stream_ptr


class ParamTensor(ctypes.Structure):
    """rth_param_tensor"""
    _fields_ = [("param", _lib.c_vp), ("grad", _lib.c_vp), ("exp_avg", _lib.c_vp), ("exp_avg_sq", _lib.c_vp),
                ("n", _lib.c_i64)]


class ClipAdam(torch.optim.Optimizer):
    MAX_TENSORS = 32  # RTH_MAX_PARAM_TENSORS

    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, max_norm=None):
        super().__init__(params, dict(lr=lr, betas=tuple(betas), eps=eps))
        if len(self.param_groups) != 1:
            raise ValueError("ClipAdam takes one parameter group")
        ps = self.param_groups[0]["params"]
        if not ps or len(ps) > self.MAX_TENSORS:
            raise ValueError(f"ClipAdam: {len(ps)} parameter tensors (1..{self.MAX_TENSORS})")
        dev = ps[0].device
        for p in ps:  # elementwise over the storage: any dense layout (conv weights may be NHWC)
            dense = p.is_contiguous() or p.is_contiguous(memory_format=torch.channels_last)
            if p.dtype != torch.float32 or p.device != dev or not dense:
                raise ValueError("ClipAdam: parameters must be dense float32 tensors on one device")
        self.max_norm = max_norm
        self._step = torch.zeros(1, dtype=torch.int64, device=dev)
        self._ws = torch.zeros(_lib.lib().rth_clip_adam_workspace(), dtype=torch.uint8, device=dev)  # ticket = 0
        self.total_norm = torch.zeros(1, dtype=torch.float32, device=dev)
        self._prenormed = None  # norm partials of the next step written by the backward (prenorm)
        for p in ps:
            st = self.state[p]
            st["exp_avg"] = torch.zeros_like(p)  # same strides as the parameter
            st["exp_avg_sq"] = torch.zeros_like(p)
            st["step"] = self._step

    @torch.no_grad()
    def step(self, closure=None, max_norm=None):
        """max_norm (or the constructor's): clip the gradients' global 2-norm first;
        None: plain Adam.  Parameters without a gradient are skipped, as in torch."""
        loss = closure() if closure is not None else None
        g = self.param_groups[0]
        beta1, beta2 = g["betas"]
        mn = self.max_norm if max_norm is None else max_norm
        tensors = []
        for p in g["params"]:
            if p.grad is None:
                continue
            gr = p.grad
            if gr.stride() != p.stride():  # autograd keeps .grad in the parameter's layout; be safe
                gr = torch.empty_like(p).copy_(gr)
            st = self.state[p]
            tensors.append(ParamTensor(p.data_ptr(), gr.data_ptr(), st["exp_avg"].data_ptr(),
                                       st["exp_avg_sq"].data_ptr(), p.numel()))
        if not tensors:
            return loss
        arr = (ParamTensor * len(tensors))(*tensors)
        nparts, self._prenormed = self._prenormed, None
        if nparts is not None:  # the norm partials (and the step count) came from the backward
            call("rth_adam_prenormed", ctypes.cast(arr, _lib.c_vp), len(tensors), float(g["lr"]), float(beta1),
                 float(beta2), float(g["eps"]), -1.0 if mn is None or mn < 0 else float(mn), nparts, ptr(self._step),
                 ptr(self._ws), ptr(self.total_norm), stream_ptr())
            return loss
        call("rth_clip_adam", ctypes.cast(arr, _lib.c_vp), len(tensors), float(g["lr"]), float(beta1), float(beta2),
             float(g["eps"]), -1.0 if mn is None or mn < 0 else float(mn), ptr(self._step), ptr(self._ws),
             ptr(self.total_norm), stream_ptr())
        return loss

    # ---- the norm partials written by the learner's backward (rth_conv1_relu_wgrad_norm, one rank)
    def norm_tensors(self, grads):
        """(rth_param_tensor array, count) of the gradients whose squares the backward's launch
        sums (only .grad and .n are read)"""
        ts = [ParamTensor(gr.data_ptr(), gr.data_ptr(), gr.data_ptr(), gr.data_ptr(), gr.numel()) for gr in grads]
        return (ParamTensor * len(ts))(*ts), len(ts)

    def prenorm_scalars(self):
        """(lr, beta1, beta2, step, workspace) for the launch that advances the step count"""
        g = self.param_groups[0]
        beta1, beta2 = g["betas"]
        return float(g["lr"]), float(beta1), float(beta2), ptr(self._step), ptr(self._ws)

    def step_launch(self, max_norm=None):
        """the step() that would run now as a callable that may be issued again (a probe
        window replays it eagerly after the capture): a pending backward-written norm (prenorm)
        is bound to it"""
        nparts, self._prenormed = self._prenormed, None

        def launch():
            self._prenormed = nparts
            self.step(max_norm=max_norm)

        return launch

    def prenorm(self, nparts):
        """the next step() runs the update alone over `nparts` partials the backward wrote"""
        self._prenormed = int(nparts)
