"""Microbench (development aid): FC1 (x [M, 3136] -> [M, 512], bias + ReLU) on hipBLASLt
(torch._addmm_activation, the committed TunableOp picks) vs rth_fc_x9 and rth_fc_f32, alone,
HIP events.  FC_MS=512,1024 picks the row counts."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from reth_amd import _lib, gemm_tuning  # noqa: E402

dev = torch.device("cuda")
gemm_tuning.enable()
N, K = 512, 3136
for M in [int(v) for v in os.environ.get("FC_MS", "256,512,1024,2048").split(",")]:
    x = torch.rand((M, K), device=dev)
    w = torch.randn((N, K), device=dev) / 56
    b = torch.randn(N, device=dev) * 0.1
    y = torch.empty((M, N), device=dev)
    fns = {"hipblaslt": lambda: torch._addmm_activation(b, x, w.t(), out=y)}
    for kind in ("x9", "f32"):
        name = "rth_fc_" + kind
        if not getattr(_lib.lib(), name + "_supported")(M, N, K):
            continue
        ws = torch.empty(max(getattr(_lib.lib(), name + "_workspace")(M, N, K), 16) // 4, device=dev)
        fns[name] = (lambda nm=name, wsp=ws: _lib.call(nm, x.data_ptr(), K, M, w.data_ptr(), N, K, b.data_ptr(), 1,
                                                        y.data_ptr(), wsp.data_ptr(), _lib.stream_ptr()))
    ref = torch.relu(x.double() @ w.double().t() + b.double())
    res = {}
    for name, fn in fns.items():
        for _ in range(5):
            fn()
        torch.cuda.synchronize()
        err = float((y.double() - ref).abs().max())
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(50):
            fn()
        e1.record()
        torch.cuda.synchronize()
        res[name] = (e0.elapsed_time(e1) * 1e3 / 50, err)
    fl = 2.0 * M * N * K
    print(f"M={M}: " + "  ".join(f"{k} {v:6.1f} us ({fl / v / 1e6:6.1f} TF/s, err {e:.1e})" for k, (v, e) in res.items()),
          flush=True)
