"""Host n-step adder: reth/reth/utils/nstep_adder.py:5-28 (NStepAdder), for the CPU actors
of test/apex-dqn/worker.py:34,50 (`adder.push(s0, a, r, s1, done)` per env step).  The
GPU actors use the device form (k_nstep_push, actors.VecActors); this is the same algorithm
over host rows:

  * a deque of at most `step` pending rows, newest first;
  * push: when full, the oldest row is emitted; then every pending row up to (excluding)
    the first one already done takes r_k += gamma^j * r and s1_k = s1 (a done row stops the
    walk: rows older than an episode end keep their own s1); the new row goes in front.

The reward arithmetic of the reference depends on numpy's promotion rules (the rewards are
0-d float32 arrays, worker.py:47): numpy 1.19 (the reference's pin) adds the float64
product `t_gamma * r` and rounds once to float32 (`mode=0`, the default), numpy >= 2 (NEP 50)
computes it in float32 (`mode=1`).  Python-float rewards (the CartPole example) stay Python
floats, as in the reference.  The device adder implements the same two modes.
"""
from collections import deque

import numpy as np


def _add_discounted(acc, t_gamma, r, mode):
    if isinstance(acc, np.ndarray) or isinstance(acc, np.floating):
        if np.asarray(acc).dtype == np.float32:
            if mode == 0:
                return np.float32(np.float64(acc) + t_gamma * np.float64(r))
            return np.float32(np.float32(acc) + np.float32(t_gamma) * np.float32(r))
        return acc + t_gamma * r
    return acc + t_gamma * r


class NStepAdder:
    def __init__(self, gamma, step=3, mode=0):
        self.step = int(step)
        self.gamma = gamma
        self.mode = int(mode)
        self._buffer = deque(maxlen=self.step)

    def push(self, s0, a, r, s1, done, *extra_args):
        """one transition in; the row leaving the window (or None) out"""
        res = None
        if len(self._buffer) == self._buffer.maxlen:
            res = self._buffer.pop()
        t_gamma = self.gamma
        for item in self._buffer:
            if item[4]:
                break
            new = _add_discounted(item[2], t_gamma, r, self.mode)
            if isinstance(item[2], np.ndarray):
                item[2][...] = new  # in place, like `item[2] += ...` on the 0-d array
            else:
                item[2] = new
            t_gamma *= self.gamma
            item[3] = s1
        self._buffer.appendleft([s0, a, r, s1, done, *extra_args])
        return res
