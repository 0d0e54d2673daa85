"""reth.buffer.NumpyBuffer on the host: the uniform replay of BASELINE configs[0]
(CartPole, CPU torch) and the apex worker's 64-row staging batch (test/apex-dqn/worker.py:34,
53-60), which never touch a GPU.  `reth_amd.buffer.NumpyBuffer(..., device="cpu")` builds
this class; every other device gets the HBM buffer.

Same surface and index semantics as reth/reth/buffer/buffer.py:4-113: columns detected from
the first row (dtype name, row shape), a ring of `capacity` rows (or a non-circular batch
that asserts on overflow), append_batch returning the slots it wrote, sample = a uniform
draw of `batch_size` slots with replacement (np.random.choice over the stored rows), data =
the stored prefix of every column.
"""
import numpy as np


class HostNumpyBuffer:
    def __init__(self, capacity, struct=None, circular=True, device="cpu", seed=None):
        self._capacity = int(capacity)
        self._struct = list(struct) if struct is not None else None
        self.circular = circular
        self._cols = None
        self._n = 0      # rows stored
        self._last = -1  # slot of the newest row
        if self._struct is not None:
            self._alloc()

    # ---------------------------------------------------------------- layout
    def _alloc(self):
        self._cols = [np.empty((self._capacity, *shape), dtype=dt) for dt, shape in self._struct]

    def _learn(self, row):
        self._struct = [(np.asarray(x).dtype.name, np.asarray(x).shape) for x in row]
        self._alloc()

    def resize(self, new_capacity):
        assert new_capacity > self._n
        old = self._cols
        self._capacity = int(new_capacity)
        if self._struct is not None:
            self._alloc()
            for new, prev in zip(self._cols, old):
                new[:self._n] = prev[:self._n]

    # ---------------------------------------------------------------- writes
    def append(self, trans):
        if self._cols is None:
            self._learn(trans)
        if not self.circular:
            assert self._n < self._capacity
        slot = (self._last + 1) % self._capacity
        for col, x in zip(self._cols, trans):
            col[slot] = x
        self._last = slot
        self._n = min(self._n + 1, self._capacity)
        return slot

    def append_batch(self, trans):
        if self._cols is None:
            self._learn([c[0] for c in trans])
        n = len(trans[0])
        assert (self._n + n <= self._capacity) if not self.circular else (n <= self._capacity)
        first = (self._last + 1) % self._capacity
        slots = (first + np.arange(n)) % self._capacity
        head = min(n, self._capacity - first)  # rows before the wrap
        for col, x in zip(self._cols, trans):
            x = np.asarray(x)
            col[first:first + head] = x[:head]
            col[:n - head] = x[head:]
        self._last = int(slots[-1]) if n else self._last
        self._n = min(self._n + n, self._capacity)
        return slots

    # ---------------------------------------------------------------- reads
    def sample(self, batch_size):
        return self.select(np.random.choice(self._n, batch_size))

    def select(self, indices):
        return [col[indices] for col in self._cols]

    def clear(self):
        self._n, self._last = 0, -1

    @property
    def data(self):
        return [col[:self._n] for col in self._cols]

    @property
    def capacity(self):
        return self._capacity

    @property
    def struct(self):
        return self._struct

    @property
    def size(self):
        return self._n
