"""Microbench (development aid): FC1 (x [M, 3136] -> [M, 512], bias + ReLU) on hipBLASLt
(torch._addmm_activation, the committed TunableOp picks) vs rth_fc_x9, alone, HIP events."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from reth_amd import _lib, gemm_tuning  # noqa: E402

dev = torch.device("cuda")
gemm_tuning.enable()
N, K = 512, 3136
for M in (512, 1024, 2048):
    x = torch.rand((M, K), device=dev)
    w = torch.randn((N, K), device=dev) / 56
    b = torch.randn(N, device=dev) * 0.1
    y = torch.empty((M, N), device=dev)
    ws = torch.empty(max(_lib.lib().rth_fc_x9_workspace(M, N, K), 16) // 4, device=dev)

    def lib():
        torch._addmm_activation(b, x, w.t(), out=y)

    def ours():
        _lib.call("rth_fc_x9", x.data_ptr(), K, M, w.data_ptr(), N, K, b.data_ptr(), 1, y.data_ptr(), ws.data_ptr(),
                  _lib.stream_ptr())

    res = {}
    for name, fn in (("hipblaslt", lib), ("rth_fc_x9", ours)):
        for _ in range(5):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(50):
            fn()
        e1.record()
        torch.cuda.synchronize()
        res[name] = e0.elapsed_time(e1) * 1e3 / 50
    fl = 2.0 * M * N * K
    print(f"M={M}: " + "  ".join(f"{k} {v:6.1f} us ({fl / v / 1e6:6.1f} TF/s)" for k, v in res.items()), flush=True)
