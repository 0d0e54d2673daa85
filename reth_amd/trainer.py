"""Learner wrapper: reth/reth/presets/trainer.py:9-74 (Trainer).

Same surface (step/print/cur_time/save_weights/load_weights/on_step_end).  The mean |td|
used for the periodic log line is accumulated on the device and only read when a line is
printed, so step() adds no host synchronisation beyond what the solver call itself does.
"""
import logging
import sys
import time

import torch

from .schedule import Interval


def getLogger(name, level=logging.DEBUG):
    """reth/reth/utils/__init__.py:8-20"""
    logger = logging.getLogger(name)
    logger.setLevel(level)
    if not logger.handlers:
        h = logging.StreamHandler(sys.stderr)
        h.setLevel(level)
        h.setFormatter(logging.Formatter("[%(asctime)s][%(name)s][%(levelname)s] %(message)s"))
        logger.addHandler(h)
    return logger


class Trainer:
    def __init__(self, solver, logger=None, print_interval=300):
        self.solver = solver
        self.logger = logger if logger is not None else getLogger("trainer")
        self.cur_step = 0
        self.start_time = None
        self.on_step_end = [Interval(self.print, int(print_interval))]
        self._err_acc = None  # persistent device accumulator (in-place: graph-replay safe)
        self._err_n = 0
        dev = getattr(solver, "device", None)
        if dev is not None and getattr(dev, "type", None) == "cuda" and hasattr(solver, "td_mean_acc"):
            # the solver's fused gradient pass adds mean |td| here itself (rth_heads_backward)
            self._err_acc = torch.zeros((), dtype=torch.float32, device=dev)
            solver.td_mean_acc = self._err_acc

    @property
    def cur_time(self):
        return 0 if self.start_time is None else time.monotonic() - self.start_time

    def print(self):
        if self.logger and self._err_n:
            mean = float(self._err_acc) / self._err_n
            self.logger.info(f"train_cnt: {self.cur_step}, mean_error: {mean:.3f}, time: {self.cur_time:.2f}")
        if self._err_acc is not None:
            self._err_acc.zero_()
        self._err_n = 0

    def load_weights(self, stream):
        self.solver.load_weights(stream)

    def save_weights(self, stream=None):
        return self.solver.save_weights(stream)

    def _track(self, td):
        if getattr(td, "_rth_mean_tracked", False):
            return
        if self._err_acc is None:
            self._err_acc = torch.zeros((), dtype=torch.float32, device=td.device)
        self._err_acc.add_(td.float().mean())

    def train(self, batch, **kwargs):
        """the device work of one step (capturable): update + error accounting"""
        td = self.solver.update_device(batch, **kwargs)
        self._track(td)
        return td

    def account(self, n=1):
        """host bookkeeping of n steps (eager or graph-replayed)"""
        if self.start_time is None:
            self.start_time = time.monotonic()
        for _ in range(n):
            self.cur_step += 1
            self._err_n += 1
            for f in self.on_step_end:
                f()

    def step(self, batch, device_result=False, **kwargs):
        """one learner update; returns |td| (CPU tensor like the reference, or the device
        tensor with device_result=True)."""
        td = self.train(batch, **kwargs)
        self.account()
        return td if device_result else td.cpu()
