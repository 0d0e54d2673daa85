"""`reth.buffer` (reth/reth/buffer/__init__.py).  The reference's NumpyBuffer is a host numpy
buffer, so it stays on the host unless a device is named (the apex worker's staging batch,
test/apex-dqn/worker.py:35); PrioritizedBuffer keeps reth_amd's HBM default."""
from reth_amd.buffer import DynamicSizeBuffer, PrioritizedBuffer  # noqa: F401
from reth_amd.buffer import NumpyBuffer as _NumpyBuffer


def NumpyBuffer(capacity, struct=None, circular=True, device="cpu", **kwargs):
    return _NumpyBuffer(capacity, struct=struct, circular=circular, device=device, **kwargs)
