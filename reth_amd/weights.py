"""On-device weights broadcast: a latest-wins slot with a device version counter.

Replaces the perwez PUB/SUB with CONFLATE used for learner -> actor weights
(perwez/perwez/client/socket.py:19-122, 302-328; test/apex-dqn/trainer.py:38-41 sends every
`send_weights_interval` updates, worker.py:37-41 loads when more than
`recv_weights_interval` steps passed and a message is waiting).  Learner and actors of a
GPU share its HBM, so the message is the parameters themselves, in the C-ABI slot
(rth_weights_publish / rth_weights_acquire, csrc/weights.hip): publishing is one gather of
the parameter tensors into the slot plus a device version bump; acquiring takes the
reference's load decision on the device (newer version, and with a device step counter the
interval gate) and copies out only then -- conflation falls out of overwriting the slot.
`version` mirrors the device counter on the host for the publisher's process.
The torch.save stream format stays available through DQNSolver.save_weights/load_weights
and the perwez facade (reth_amd.perwez) for byte messages.
"""
import ctypes

import torch

from . import _lib
from ._lib import c_vp, call, stream_ptr


def _dense(t):
    """the bytes of t are one dense run (contiguous or channels_last): the slot copies raw bytes"""
    return t.is_contiguous() or (t.dim() == 4 and t.is_contiguous(memory_format=torch.channels_last))


def _segments(tensors):
    n = len(tensors)
    ptrs = (c_vp * n)(*[t.data_ptr() for t in tensors])
    nbytes = (ctypes.c_int64 * n)(*[t.numel() * t.element_size() for t in tensors])
    return n, ptrs, nbytes


class WeightsSlot:
    """the channel: one slot per published module layout (parameter order of the module)"""

    def __init__(self, module):
        params = [p for p in module.parameters()]
        if not params or any(not p.is_cuda or not _dense(p) for p in params):
            raise ValueError("WeightsSlot needs dense (contiguous or channels_last) device parameters")
        # the slot holds raw bytes: publishers and consumers must share this layout
        self.layout = [(tuple(p.shape), p.stride()) for p in params]
        self.device = params[0].device
        nbytes = sum(p.numel() * p.element_size() for p in params)
        h = c_vp()
        call("rth_weights_create", nbytes, self.device.index or 0, ctypes.byref(h))
        self._h = h
        self.nbytes = nbytes
        self.version = 0  # host mirror of the device counter (publishes of this process)
        # the construction snapshot fills the slot without a message (device version 0, like the
        # mirror): subscribers see nothing newer until the first publish (a SUB socket
        # receives nothing before the trainer's first send)
        params = [p.detach() for p in module.parameters()]
        self._check(params)
        n, ptrs, nbytes = _segments(params)
        call("rth_weights_fill", self._h, n, ptrs, nbytes, stream_ptr())
        self._seen = torch.zeros((), dtype=torch.int64, device=self.device)  # acquire() consumers

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and _lib._lib is not None:
            _lib._lib.rth_weights_destroy(h)
            self._h = None

    @torch.no_grad()
    def publish(self, module):
        """SendSocket.send: the module's parameters into the slot, version += 1"""
        params = [p.detach() for p in module.parameters()]
        self._check(params)
        n, ptrs, nbytes = _segments(params)
        call("rth_weights_publish", self._h, n, ptrs, nbytes, stream_ptr())
        self.version += 1

    @torch.no_grad()
    def acquire(self, module, seen=None, step=None, prev=None, interval=0, loaded=None):
        """RecvSocket.recv into `module`'s parameters when the device decides to (newer
        version than `seen`; with `step`/`prev` device counters also step - prev > interval).
        seen/step/prev: int64 device scalars (default: this slot's own seen counter), loaded:
        optional int32 device scalar set to 1 / 0.  Returns the host version mirror."""
        params = [p for p in module.parameters()]
        self._check(params)
        n, ptrs, nbytes = _segments(params)
        call("rth_weights_acquire", self._h, n, ptrs, nbytes, (seen if seen is not None else self._seen).data_ptr(),
             None if step is None else step.data_ptr(), None if prev is None else prev.data_ptr(), int(interval),
             None if loaded is None else loaded.data_ptr(), stream_ptr())
        if getattr(module, "dueling", False) and hasattr(module, "freeze_heads"):
            module.freeze_heads()  # the actor's cached merged heads follow its parameters
        return self.version

    @torch.no_grad()
    def copy_out(self, module):
        """the slot's current contents into `module` unconditionally (no version gate): the
        actors' starting weights = the learner's initial ones, before any message"""
        force = torch.full((), -1, dtype=torch.int64, device=self.device)
        self.acquire(module, seen=force)

    def _check(self, params):
        if [(tuple(p.shape), p.stride()) for p in params] != self.layout:
            raise ValueError("module parameters do not match the slot's layout (shapes / memory format)")

    def device_version(self):
        """the device counter (synchronous read)"""
        v = ctypes.c_int64()
        call("rth_weights_version", self._h, ctypes.byref(v))
        return v.value


class WeightsSubscriber:
    """the actor side: reload when `interval` actor steps passed and something newer exists
    (worker.py:37-41).  The decision is taken on the host from the publisher's version mirror
    (same process); the device then finds the slot newer than this subscriber's seen counter
    and copies."""

    def __init__(self, slot, interval):
        self.slot, self.interval = slot, int(interval)
        self.loaded_version = 0
        self.prev_load = 0
        self._seen = torch.zeros((), dtype=torch.int64, device=slot.device)

    def maybe_load(self, module, cur_step):
        if cur_step - self.prev_load > self.interval and self.slot.version > self.loaded_version:
            self.loaded_version = self.slot.acquire(module, seen=self._seen)
            self.prev_load = cur_step
            return True
        return False
