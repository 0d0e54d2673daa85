"""`reth_buffer` -> reth_amd.reth_buffer (reth_buffer/reth_buffer/__init__.py:1-49)"""
from reth_amd.reth_buffer import Client, NumpyLoader, TorchCudaLoader, start_per, start_server  # noqa: F401
