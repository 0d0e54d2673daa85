"""ctypes wrapper of liboracle.so -- TEST INFRASTRUCTURE ONLY.

The CPU restatement of the reference's hot path (reth_oracle.c).  Imported only by tests/,
__graft_entry__.smoke() (as the checker) and bench.py's cpu_baseline leg.  The product
(reth_amd/) never imports it.
"""
import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(_HERE, "liboracle.so")
_lib = None

_p = ctypes.c_void_p
_i64, _i32, _f32, _f64, _u64, _u32 = (ctypes.c_int64, ctypes.c_int32, ctypes.c_float, ctypes.c_double,
                                      ctypes.c_uint64, ctypes.c_uint32)

NSTEP_MAX = 16


class NStepState(ctypes.Structure):
    _fields_ = [("n", _i32), ("count", _i32), ("s0", _i64 * NSTEP_MAX), ("a", _i64 * NSTEP_MAX),
                ("s1", _i64 * NSTEP_MAX), ("r", _f32 * NSTEP_MAX), ("done", _f32 * NSTEP_MAX)]


_SIGS = {
    "orc_tree_update": (None, [_i64, _p, _p, _p, _p, _p, _i64]),
    "orc_tree_find": (_i64, [_i64, _p, _p, _f64]),
    "orc_tree_sample": (None, [_i64, _p, _p, _i64, _p, _p, _p]),
    "orc_tree_min": (_f64, [_p, _p]),
    "orc_per_normalize": (None, [_p, _i64, _f32, _p]),
    "orc_per_normalize64": (None, [_p, _i64, _f64, _p]),
    "orc_per_is_weights": (None, [_p, _i64, _f64, _f64, _p]),
    "orc_schedule_value": (_f64, [_i32, _f64, _f64, _i64, _i64]),
    "orc_fifo_indices": (None, [_i64, ctypes.POINTER(_i64), _i64, _p]),
    "orc_nstep_init": (None, [ctypes.POINTER(NStepState), _i32]),
    "orc_nstep_push": (_i32, [ctypes.POINTER(NStepState), _f64, _i32, _i64, _i64, _f32, _i64, _f32,
                              ctypes.POINTER(_i64), ctypes.POINTER(_i64), ctypes.POINTER(_f32),
                              ctypes.POINTER(_i64), ctypes.POINTER(_f32)]),
    "orc_argmax_first": (_i64, [_p, _i64]),
    "orc_td_error": (None, [_p, _p, _p, _p, _p, _p, _i64, _i64, _f32, _i32, _p]),
    "orc_td_huber": (_f32, [_p, _p, _p, _i64, _i64, _p, _p]),
    "orc_eps_greedy": (None, [_p, _i64, _i64, _p, _p, _p, _p]),
    "orc_philox_uniform": (_f64, [_u64, _u64, _u32, _u32]),
    "orc_philox4x32": (None, [_p, _p, _p]),
}

STREAM_SAMPLE, STREAM_EXPLORE, STREAM_RANDACT, STREAM_ENV = 1, 2, 3, 4


def build():
    import subprocess

    subprocess.check_call(["make", "-s", "-C", _HERE])


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        L = ctypes.CDLL(LIB)
        for k, (r, a) in _SIGS.items():
            f = getattr(L, k)
            f.restype, f.argtypes = r, a
        _lib = L
    return _lib


def _a(x, dt):
    return np.ascontiguousarray(x, dtype=dt)


def P(x):
    return x.ctypes.data_as(_p) if x is not None else None


class Tree:
    """the reference NumbaSumTree state (three fp64 arrays) + its operations"""

    def __init__(self, capacity):
        self.capacity = int(capacity)
        self.sum = np.zeros(capacity)
        self.min_ = np.zeros(capacity)
        self.val = np.zeros(capacity)

    def update(self, idx, w):
        idx, w = _a(idx, np.int64), _a(w, np.float64)
        lib().orc_tree_update(self.capacity, P(self.sum), P(self.min_), P(self.val), P(idx), P(w), len(idx))

    def find(self, t):
        return lib().orc_tree_find(self.capacity, P(self.sum), P(self.val), float(t))

    def sample(self, uniforms):
        u = _a(uniforms, np.float64)
        idx = np.empty(len(u), np.int64)
        val = np.empty(len(u), np.float64)
        lib().orc_tree_sample(self.capacity, P(self.sum), P(self.val), len(u), P(u), P(idx), P(val))
        return idx, val

    def total(self):
        return float(self.sum[0])

    def min(self):
        return lib().orc_tree_min(P(self.sum), P(self.min_))


def per_normalize(w, alpha):
    w = np.asarray(w)
    if w.dtype == np.float64:
        out = np.empty(len(w), np.float64)
        lib().orc_per_normalize64(P(_a(w, np.float64)), len(w), float(alpha), P(out))
        return out
    w = _a(w, np.float32)
    out = np.empty(len(w), np.float32)
    lib().orc_per_normalize(P(w), len(w), float(np.float32(alpha)), P(out))
    return out


def per_is_weights(p, tree_min, beta):
    p = _a(p, np.float64)
    out = np.empty(len(p), np.float64)
    lib().orc_per_is_weights(P(p), len(p), float(tree_min), float(beta), P(out))
    return out


def schedule_value(method, start, end, max_steps, step):
    return lib().orc_schedule_value(0 if method == "linear" else 1, start, end, max_steps, step)


def fifo_indices(cap, tail, n):
    t = _i64(tail)
    out = np.empty(n, np.int32)
    lib().orc_fifo_indices(cap, ctypes.byref(t), n, P(out))
    return out, t.value


class NStep:
    def __init__(self, n, gamma, mode):
        self.st = NStepState()
        self.gamma, self.mode = float(gamma), int(mode)
        lib().orc_nstep_init(ctypes.byref(self.st), n)

    def push(self, s0, a, r, s1, done):
        o = [_i64(), _i64(), _f32(), _i64(), _f32()]
        e = lib().orc_nstep_push(ctypes.byref(self.st), self.gamma, self.mode, int(s0), int(a), float(r), int(s1),
                                 float(done), *[ctypes.byref(x) for x in o])
        if not e:
            return None
        return (o[0].value, o[1].value, np.float32(o[2].value), o[3].value, np.float32(o[4].value))


def td_error(q0, q1o, q1t, a, r, done, gamma_n, double_q=True):
    q0, q1t = _a(q0, np.float32), _a(q1t, np.float32)
    q1o = _a(q1o, np.float32) if q1o is not None else q1t
    a, r, done = _a(a, np.int64), _a(r, np.float32), _a(done, np.float32)
    B, A = q0.shape
    td = np.empty(B, np.float32)
    lib().orc_td_error(P(q0), P(q1o), P(q1t), P(a), P(r), P(done), B, A, float(np.float32(gamma_n)), int(double_q),
                       P(td))
    return td


def td_huber(td, w, a, A):
    td, a = _a(td, np.float32), _a(a, np.int64)
    w = None if w is None else _a(w, np.float32)
    B = len(td)
    le = np.empty(B, np.float32)
    dq = np.empty((B, A), np.float32)
    loss = lib().orc_td_huber(P(td), P(w), P(a), B, A, P(le), P(dq))
    return np.float32(loss), le, dq


def eps_greedy(q, eps, u, rand_action):
    q = _a(q, np.float32)
    N, A = q.shape
    out = np.empty(N, np.int64)
    lib().orc_eps_greedy(P(q), N, A, P(_a(eps, np.float64)), P(_a(u, np.float64)), P(_a(rand_action, np.int64)),
                         P(out))
    return out


def philox_uniform(seed, counter, lane, stream):
    return lib().orc_philox_uniform(seed, counter, lane, stream)


def philox4x32(ctr, key):
    c = _a(ctr, np.uint32)
    k = _a(key, np.uint32)
    o = np.empty(4, np.uint32)
    lib().orc_philox4x32(P(c), P(k), P(o))
    return o


# ---------------------------------------------------------------------------------------
# Samplers and in-process buffers (pure-Python restatements; small cases only)
# ---------------------------------------------------------------------------------------
class UniformSampler:
    """reth_buffer/reth_buffer/sampler/uniform_sampler.py:6-25 with the random draw injected:
    sample() maps uniforms u to positions floor(u * tail) (np.random.choice(tail, B) draws
    positions uniformly).  update() stops at capacity (the reference writes one entry past
    a full list and raises IndexError when an update straddles capacity)."""

    def __init__(self, capacity):
        self.indices = np.zeros(capacity, dtype="i8")
        self.capacity = capacity
        self.tail = 0

    def sample(self, uniforms):
        pos = np.minimum((np.asarray(uniforms, np.float64) * self.tail).astype(np.int64), self.tail - 1)
        return self.indices[pos], np.ones(len(pos), dtype="i8")

    def update(self, indices, weights=None):
        for idx in indices:
            if self.tail == self.capacity:
                return
            self.indices[self.tail] = idx
            self.tail += 1


class FIFOSampler:
    """reth_buffer/reth_buffer/sampler/fifo_sampler.py:8-29 (verbatim semantics)."""

    def __init__(self, capacity):
        from collections import deque

        self.buffer = deque(maxlen=capacity)

    def ready_sample(self, batch_size):
        return len(self.buffer) > batch_size

    def sample(self, batch_size):
        res_i, res_w = [], []
        for _ in range(batch_size):
            i, w = self.buffer.pop()
            res_i.append(i)
            res_w.append(w)
        return np.asarray(res_i, np.int64), np.asarray(res_w, np.float64)

    def update(self, indices, weights):
        for i, idx in enumerate(indices):
            self.buffer.appendleft((int(idx), float(weights[i])))


def numpy_buffer_indices(capacity, tail, size, batch_size):
    """reth/reth/buffer/buffer.py:55-85 (NumpyBuffer.append_batch): slots written and the new
    (tail, size); tail starts at -1"""
    size = min(size + batch_size, capacity)
    tail = (tail + 1) % capacity
    len1 = min(batch_size, capacity - tail)
    len2 = batch_size - len1
    if len2 == 0:
        idx = np.arange(tail, tail + len1)
        tail = tail + len1 - 1
    else:
        idx = np.concatenate((np.arange(tail, tail + len1), np.arange(len2)))
        tail = len2 - 1
    return idx, tail, size


class PrioritizedBuffer:
    """reth/reth/buffer/prioritized_buffer.py:8-74 on the C tree (indices only, uniforms
    injected into the tree sample; alpha/beta are Schedule specs)."""

    def __init__(self, capacity, alpha, beta):
        self.tree = Tree(capacity)
        self.capacity = capacity
        self.alpha, self.beta = _Sched(alpha), _Sched(beta)
        self.tail, self.size = -1, 0

    def _norm(self, w):
        w = np.asarray(w)
        return (w + 1e-6) ** self.alpha.value()

    def append_batch(self, n, weights=None):
        idx, self.tail, self.size = numpy_buffer_indices(self.capacity, self.tail, self.size, n)
        w = np.ones(n) if weights is None else self._norm(weights)
        self.tree.update(idx, np.asarray(w, np.float64))
        return idx

    def sample(self, uniforms):
        idx, p = self.tree.sample(uniforms)
        self.alpha.step()
        self.beta.step()
        return idx, (p / self.tree.min()) ** (-self.beta.value())

    def update_priorities(self, indices, weights):
        self.tree.update(np.asarray(indices, np.int64), np.asarray(self._norm(weights), np.float64))


class _Sched:
    """reth/reth/utils/schedule.py:4-52 (const or 'start,end,steps' linear)"""

    def __init__(self, spec):
        parts = str(spec).split(",")
        if len(parts) == 1:
            self.start = self.end = float(parts[0])
            self.steps = 1
            self.const = True
        else:
            self.start, self.end, self.steps = float(parts[0]), float(parts[1]), int(parts[2])
            self.const = False
        self.k = 0

    def step(self):
        self.k = min(self.k + 1, self.steps)

    def value(self):
        if self.const:
            return self.start
        return self.start + ((self.end - self.start) * self.k) / self.steps


# ---------------------------------------------------------------------------------------
# Atari preprocessing (reth/reth/env/util.py:121-209): MaxAndSkip max, cv2 RGB2GRAY,
# cv2.resize INTER_AREA (OpenCV's 8-bit algorithms restated; cv2 is absent -> parity with
# cv2 itself is unpinned), float32 operation order of resizeArea_
# ---------------------------------------------------------------------------------------
def area_tab(ssize, dsize, scale):
    """computeResizeAreaTab: per destination index, [(source index, float32 weight)]"""
    import math

    out = []
    for d in range(dsize):
        f1 = d * scale
        f2 = f1 + scale
        cell = min(scale, ssize - f1)
        s1, s2 = math.ceil(f1), math.floor(f2)
        s2 = min(s2, ssize - 1)
        s1 = min(s1, s2)
        taps = []
        if s1 - f1 > 1e-3:
            taps.append((s1 - 1, np.float32((s1 - f1) / cell)))
        for s in range(s1, s2):
            taps.append((s, np.float32(1.0 / cell)))
        if f2 - s2 > 1e-3:
            taps.append((s2, np.float32(min(min(f2 - s2, 1.0), cell) / cell)))
        out.append(taps)
    return out


def rgb2gray(rgb):
    """cv2.cvtColor(RGB2GRAY) on uint8: (R*4899 + G*9617 + B*1868 + 8192) >> 14"""
    c = rgb.astype(np.uint32)
    return ((c[..., 0] * 4899 + c[..., 1] * 9617 + c[..., 2] * 1868 + 8192) >> 14).astype(np.uint32)


def warp_frame(f0, f1, oh=84, ow=84):
    """WarpFrame(MaxAndSkip max of two raw frames) -> uint8 [oh, ow]"""
    H, W, _ = f0.shape
    gray = rgb2gray(np.maximum(f0, f1)).astype(np.float32)
    xt = area_tab(W, ow, 1.0 / (ow / W))
    yt = area_tab(H, oh, 1.0 / (oh / H))
    K = max(len(t) for t in xt)
    xs = np.zeros((ow, K), np.int64)
    xw = np.zeros((ow, K), np.float32)  # padded taps add S * 0 = +0: exact no-ops
    for d, taps in enumerate(xt):
        for k, (s, w) in enumerate(taps):
            xs[d, k], xw[d, k] = s, w
    out = np.empty((oh, ow), np.uint8)
    for dy, taps in enumerate(yt):
        acc = None
        for sy, beta in taps:
            row = gray[sy]
            buf = np.zeros(ow, np.float32)
            for k in range(K):
                buf = (buf + row[xs[:, k]] * xw[:, k]).astype(np.float32)
            term = (np.float32(beta) * buf).astype(np.float32)
            acc = term if acc is None else (acc + term).astype(np.float32)
        out[dy] = np.clip(np.rint(acc), 0, 255).astype(np.uint8)
    return out
