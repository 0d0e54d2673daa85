"""Atari observation preprocessing on the device (reth/reth/env/util.py:121-209, 281-297).

The reference's wrappers run per actor on the host: MaxAndSkipEnv keeps the last two raw
210x160 RGB frames of the 4-frame skip window and returns their max, WarpFrame converts to
gray and resizes to 84x84 with cv2 (INTER_AREA), FrameStack keeps the last 4 (oldest
first, ImageToPyTorch: (4, 84, 84)).  AtariPreprocessor does all of it for every actor in
one HIP launch (rth_atari_step) and writes the new uint8 stack straight into the actors'
frame ring in HBM -- the stacks the acting batch and the replay appends read.
"""
import ctypes

import torch

from . import _lib
from ._lib import c_vp, call, ptr, stream_ptr
from .replay import _device


class AtariPreprocessor:
    def __init__(self, in_hw=(210, 160), out_hw=(84, 84), stack=4, device=None):
        self.in_hw, self.out_hw, self.stack = tuple(in_hw), tuple(out_hw), int(stack)
        self.device = _device(device)
        h = c_vp()
        with torch.cuda.device(self.device):
            call("rth_atari_create", in_hw[0], in_hw[1], out_hw[0], out_hw[1], self.device.index, ctypes.byref(h))
        self._h = h.value

    def __del__(self):
        if getattr(self, "_h", None):
            try:
                _lib.lib().rth_atari_destroy(self._h)
            except Exception:
                pass
            self._h = None

    def _check_raw(self, raw):
        H, W = self.in_hw
        if raw.dtype != torch.uint8 or not raw.is_cuda or raw.dim() != 5 or tuple(raw.shape[1:]) != (2, H, W, 3):
            raise ValueError(f"raw frames must be a uint8 device tensor [n, 2, {H}, {W}, 3]")
        return raw.contiguous()

    def warp(self, raw):
        """[n, 2, H, W, 3] -> [n, 84, 84]: max of the two frames, gray, INTER_AREA"""
        raw = self._check_raw(raw)
        out = torch.empty((raw.shape[0], *self.out_hw), dtype=torch.uint8, device=self.device)
        call("rth_atari_step", self._h, ptr(raw), raw.shape[0], None, 0, 0, None, None, None, ptr(out), stream_ptr())
        return out

    def step(self, raw, frames, ring, prev_slot, new_slot, reset=None, out_frame=None):
        """push the preprocessed frames onto each actor's stack: frames is the ring
        [n * ring (+ trailing stacks, e.g. VecActors' sink), stack, 84, 84] uint8; slot new_slot[i] <- slot prev_slot[i] shifted by one
        + the new frame (or the frame `stack` times where reset[i])"""
        raw = self._check_raw(raw)
        n = raw.shape[0]
        if frames.dtype != torch.uint8 or tuple(frames.shape[1:]) != (self.stack, *self.out_hw) or \
                frames.shape[0] < n * ring or not frames.is_contiguous():
            raise ValueError("frames must be a contiguous uint8 ring [>= n * ring, stack, 84, 84]")
        for t in (prev_slot, new_slot):
            if t.dtype != torch.int64 or t.numel() != n:
                raise ValueError("slots must be int64 [n]")
        if reset is not None:
            reset = reset.to(torch.uint8).contiguous()
        call("rth_atari_step", self._h, ptr(raw), n, ptr(frames), int(ring), self.stack, ptr(prev_slot),
             ptr(new_slot), ptr(reset), ptr(out_frame), stream_ptr())
