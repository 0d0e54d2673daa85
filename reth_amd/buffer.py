"""In-process replay buffers of `reth.buffer`, resident in HBM.

Reference: reth/reth/buffer/buffer.py:4-113 (NumpyBuffer, DynamicSizeBuffer) and
reth/reth/buffer/prioritized_buffer.py:8-74 (PrioritizedBuffer) -- the single-process
buffers of the reference's examples (examples/dqn/run.py: CartPole DQN with a
PrioritizedBuffer) and of its actors' staging batches (presets/worker.py:157-163).

Same constructors, methods and index semantics; the storage is device memory and every
row moves through the HIP kernels (rth_copy_rows for writes and gathers, the sum-tree
kernels for PrioritizedBuffer, rth_uniform_indices for the uniform draw).  What differs:
  * columns come back as torch device tensors, not numpy arrays (bool columns stay bool);
  * the uniform / prioritized draws come from counter-based Philox streams instead of
    numpy's global RandomState; `uniforms=` injects explicit draws (the parity hook).
"""
import numpy as np
import torch

from . import _lib
from ._lib import call, ptr, stream_ptr
from .replay import _TORCH_TO_RTH, Column, HbmReplay, _device

_NP_NAMES = {"bool": torch.bool, "uint8": torch.uint8, "int32": torch.int32, "int64": torch.int64,
             "float32": torch.float32, "float64": torch.float64}


def _torch_dtype(name):
    try:
        return _NP_NAMES[np.dtype(name).name]
    except KeyError:
        raise TypeError(f"unsupported column dtype {name}") from None


def _as_col(x, dtype, device):
    if torch.is_tensor(x):
        return x.to(device=device, dtype=dtype)
    return torch.as_tensor(np.asarray(x), device=device).to(dtype)


def _row_elems(shape):
    return int(np.prod(shape)) if shape else 1


def _copy_rows(dst, dst_rows, src, src_rows, n):
    """n rows src[src_rows] -> dst[dst_rows] (None = 0..n-1), one rth_copy_rows launch"""
    if n == 0:
        return
    elems = _row_elems(tuple(dst.shape[1:]))
    code = _TORCH_TO_RTH[dst.dtype]
    call("rth_copy_rows", ptr(dst), 0, ptr(dst_rows), ptr(src), 0, ptr(src_rows), n, elems, code, code, 0,
         stream_ptr())


class NumpyBuffer:
    """buffer.py:4-98.  struct: [(dtype name, row shape), ...] or detected on first append.
    device="cpu": the host buffer (host_buffer.HostNumpyBuffer: numpy columns, numpy draws)."""

    def __new__(cls, *args, device=None, **kwargs):
        if cls is NumpyBuffer and device is not None and torch.device(device).type == "cpu":
            from .host_buffer import HostNumpyBuffer

            return HostNumpyBuffer(*args, device=device, **kwargs)
        return super().__new__(cls)

    def __init__(self, capacity, struct=None, circular=True, device=None, seed=0):
        self._capacity = int(capacity)
        self._struct = struct
        self.circular = circular
        self.device = _device(device)
        self.seed, self._draws = int(seed), 0
        self._buffers = None
        self._size = 0
        self._tail = -1
        if self._struct is not None:
            self._create_buffer()

    def _create_buffer(self):
        assert self._struct is not None
        self._buffers = [torch.empty((self.capacity, *shape), dtype=_torch_dtype(dt), device=self.device)
                         for dt, shape in self._struct]

    def _detect_struct(self, trans):
        self._struct = []
        for col in trans:
            if torch.is_tensor(col):
                name = str(col.dtype).replace("torch.", "")
                self._struct.append((name, tuple(col.shape)))
            else:
                data = np.asarray(col)
                self._struct.append((data.dtype.name, data.shape))
        return self._struct

    def resize(self, new_capacity):
        assert new_capacity > self.size
        self._capacity = int(new_capacity)
        if self.struct is not None:
            old = self._buffers
            self._create_buffer()
            for new_buf, old_buf in zip(self._buffers, old):
                _copy_rows(new_buf, None, old_buf, None, self.size)

    def append(self, trans):
        if self._struct is None:
            self._detect_struct(trans)
            self._create_buffer()
        if not self.circular:
            assert self.size < self.capacity
        self._size = min(self.size + 1, self.capacity)
        self._tail = (self._tail + 1) % self.capacity
        dst = torch.tensor([self._tail], dtype=torch.int64, device=self.device)
        for buf, item in zip(self._buffers, trans):
            src = _as_col(item, buf.dtype, self.device).reshape(1, *buf.shape[1:]).contiguous()
            _copy_rows(buf, dst, src, None, 1)
        return self._tail

    def append_batch(self, trans):
        if self._struct is None:
            self._detect_struct([col[0] for col in trans])
            self._create_buffer()
        batch_size = len(trans[0])
        if not self.circular:
            assert self.size + batch_size <= self.capacity
        else:
            assert batch_size <= self.capacity
        self._size = min(self.size + batch_size, self.capacity)
        start = (self._tail + 1) % self.capacity
        indices = (start + np.arange(batch_size)) % self.capacity  # the reference's two slices
        self._tail = int(indices[-1]) if batch_size else self._tail
        dst = torch.as_tensor(indices, device=self.device)
        for buf, col in zip(self._buffers, trans):
            src = _as_col(col, buf.dtype, self.device).reshape(batch_size, *buf.shape[1:]).contiguous()
            _copy_rows(buf, dst, src, None, batch_size)
        return indices

    def sample_indices(self, batch_size, uniforms=None):
        """np.random.choice(size, batch_size) on the device (Philox, or explicit uniforms)"""
        idx = torch.empty(batch_size, dtype=torch.int64, device=self.device)
        u = None if uniforms is None else torch.as_tensor(uniforms, dtype=torch.float64, device=self.device)
        call("rth_uniform_indices", self.size, batch_size, ptr(u), self.seed, self._draws, None, ptr(idx),
             stream_ptr())
        self._draws += 1
        return idx

    def sample(self, batch_size, uniforms=None):
        return self.select(self.sample_indices(batch_size, uniforms))

    def select(self, indices):
        idx = torch.as_tensor(indices, dtype=torch.int64, device=self.device).reshape(-1)
        out = []
        for buf in self._buffers:
            o = torch.empty((idx.numel(), *buf.shape[1:]), dtype=buf.dtype, device=self.device)
            _copy_rows(o, None, buf, idx, idx.numel())
            out.append(o)
        return out

    def clear(self):
        self._size = 0
        self._tail = -1

    @property
    def data(self):
        return [buf[: self.size] for buf in self._buffers]

    @property
    def capacity(self):
        return self._capacity

    @property
    def struct(self):
        return self._struct

    @property
    def size(self):
        return self._size


class DynamicSizeBuffer(NumpyBuffer):
    """buffer.py:101-113: non-circular, doubles its capacity when full."""

    def __init__(self, init_capacity=64, struct=None, device=None):
        super().__init__(init_capacity, struct, False, device=device)

    def append(self, trans):
        if self.size == self.capacity and self.struct is not None:
            self.resize(2 * self.capacity)
        return super().append(trans)

    def append_batch(self, trans):
        batch_size = len(trans[0])
        target = self.capacity
        while batch_size + self.size > target:
            target *= 2
        if target != self.capacity:
            if self.struct is None:
                self._capacity = target
            else:
                self.resize(target)
        return super().append_batch(trans)


class PrioritizedBuffer:
    """prioritized_buffer.py:8-74 over an HBM replay shard (sum-tree kernels).

    Semantics kept: append(data, weight) stores `weight` (default 1) as given;
    append_batch(data, weights) stores ones, or (weights + 1e-6) ** alpha; sample() steps
    alpha and beta BEFORE the IS weights (p / min) ** -beta; update_priorities normalises."""

    def __init__(self, capacity=50000, alpha=0.6, beta=0.4, struct=None, device=None, seed=0):
        self._capacity = int(capacity)
        self._alpha_str, self._beta_str = alpha, beta
        self.device = _device(device)
        self.seed = int(seed)
        self._struct = None
        self.replay = None
        if struct is not None:
            self._create(struct)

    def _create(self, struct):
        self._struct = [(dt, tuple(shape)) for dt, shape in struct]
        cols = [Column(shape, _torch_dtype(dt)) for dt, shape in self._struct]
        self.replay = HbmReplay(self._capacity, cols, self._alpha_str, self._beta_str, self.device, self.seed)

    def _ensure(self, rows):
        if self.replay is None:
            self._create(NumpyBuffer(1)._detect_struct(rows))

    @property
    def alpha(self):
        return self.replay.alpha if self.replay is not None else None

    @property
    def beta(self):
        return self.replay.beta if self.replay is not None else None

    def _cols(self, data, n):
        return [_as_col(c, col.dtype, self.device).reshape(n, *col.shape).contiguous()
                for c, col in zip(data, self.replay.columns)]

    def append(self, data, weight=None):
        self._ensure(data)
        w = torch.tensor([1.0 if weight is None else float(weight)], dtype=torch.float64, device=self.device)
        self.replay.append(self._cols(data, 1), w, raw=True)

    def append_batch(self, data, weights=None):
        self._ensure([c[0] for c in data])
        n = len(data[0])
        if weights is None:
            self.replay.append(self._cols(data, n), torch.ones(n, dtype=torch.float64, device=self.device), raw=True)
        else:
            assert len(weights) == n
            self.replay.append(self._cols(data, n), weights)

    def sample(self, batch_size, uniforms=None):
        assert batch_size <= self.size
        empty = torch.empty(0, dtype=torch.int64, device=self.device)
        self.replay.update_priorities(empty, torch.empty(0, device=self.device), step=True)  # alpha/beta.step()
        data, indices, weights = self.replay.sample(batch_size, uniforms)
        return data, indices, weights

    def update_priorities(self, indices, weights):
        self.replay.update_priorities(indices, weights)

    def clear(self):
        if self.replay is not None:
            struct = self._struct
            self.replay = None
            self._create(struct)

    @property
    def capacity(self):
        return self._capacity

    @property
    def size(self):
        return 0 if self.replay is None else self.replay.size

    @property
    def struct(self):
        return self._struct
