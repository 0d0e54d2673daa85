"""Host-side schedules and intervals (scalar state; the device kernels take their values).

Same semantics as reth_buffer/reth_buffer/utils/schedule.py:4-52 (== reth/reth/utils/
schedule.py) and reth/reth/utils/interval.py:1-14, including the edge behaviour:
  * a Python number gives a constant schedule; a string must be "start,end,steps" (linear)
    or "method,start,end,steps" with method linear|exp.  A single-number *string* such as
    "0.5" raises, because the reference's len(parts) == 0 branch is unreachable (:16-17);
  * step() advances up to max_steps and returns the new value; value(step) clamps.
The arithmetic is evaluated in the reference's order so the floats are bit-identical
(tests/golden/schedule_fifo.json).
"""
import math

_METHODS = ("linear", "exp")


def _parse(spec):
    fields = spec.split(",")
    if len(fields) not in (3, 4):
        raise Exception(f"Invalid schedule string {spec}")
    method = "linear" if len(fields) == 3 else fields[0]
    lo, hi, n = fields[-3:]
    if method not in _METHODS:
        float(lo), float(hi), int(n)  # the reference converts before it checks the method
        raise Exception(f"Invalid schedule method {method}")
    return method, float(lo), float(hi), int(n)


class Schedule:
    def __init__(self, method, start=0.0, end=0.0, max_steps=1, const=None):
        self.method, self.start, self.end = method, start, end
        self.max_steps = max_steps
        self.const = const
        self.cur_step = 0

    @classmethod
    def from_str(cls, spec):
        if isinstance(spec, (int, float)):
            return cls("const", const=spec)
        method, lo, hi, n = _parse(spec)
        return cls(method, lo, hi, n)

    def _at(self, k):
        if self.method == "const":
            return self.const
        if self.method == "linear":
            return self.start + (self.end - self.start) * k / self.max_steps
        return self.end - (self.end - self.start) * math.exp(-1 * k / self.max_steps)

    def step(self):
        self.cur_step = min(self.cur_step + 1, self.max_steps) if self.cur_step < self.max_steps else self.cur_step
        return self._at(self.cur_step)

    def value(self, step=None):
        return self._at(self.cur_step if step is None else min(step, self.max_steps))


class Interval:
    """Invoke `f` once every `interval` calls (reth/reth/utils/interval.py:1-14)."""

    def __init__(self, f, interval=1):
        self.f, self.interval, self.cur = f, interval, 0

    def __call__(self, step=1):
        self.cur += step
        if self.cur >= self.interval:
            self.f()
            self.cur %= self.interval

    call = __call__
