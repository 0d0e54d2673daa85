"""rth_fc_x9 alone (for kernel-trace / PMC passes): FC1's [FC_M, 3136] x [512, 3136]^T + bias + ReLU,
20 launches (FC_M default 512: the target pass's rows; 256 = the actors', 1024 = the learner's)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from reth_amd import _lib  # noqa: E402

dev = torch.device("cuda")
N, K = 512, 3136
for M in [int(v) for v in os.environ.get("FC_M", "512").split(",")]:
    x = torch.rand((M, K), device=dev) * 3
    w = (torch.rand((N, K), device=dev) * 2 - 1) / 56
    b = torch.rand(N, device=dev) * 0.1
    y = torch.empty((M, N), device=dev)
    ws = torch.empty(max(_lib.lib().rth_fc_x9_workspace(M, N, K), 16) // 4, device=dev)
    for _ in range(20):
        _lib.call("rth_fc_x9", x.data_ptr(), K, M, w.data_ptr(), N, K, b.data_ptr(), 1, y.data_ptr(), ws.data_ptr(),
                  _lib.stream_ptr())
    torch.cuda.synchronize()
