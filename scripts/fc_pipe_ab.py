"""Development aid (r06): rth_fc_x9's 128 x 128 forms, k_fc_x9p (RTH_FC_PIPE=1) vs k_fc_x9t
(RTH_FC_PIPE=0, read once per process): time each FC1 shape alone (HIP events) and save the
outputs, so two runs can be compared bit for bit.  usage: fc_pipe_ab.py OUT.pt"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from reth_amd import _lib  # noqa: E402

dev = torch.device("cuda")
N, K = 512, 3136
g = torch.Generator(device=dev).manual_seed(1)
res = {}
for M in (256, 512, 1024, 2048):
    x = torch.rand((M, K), device=dev, generator=g)
    w = torch.randn((N, K), device=dev, generator=g) / 56
    b = torch.randn(N, device=dev, generator=g) * 0.1
    y = torch.empty((M, N), device=dev)
    ws = torch.empty(max(_lib.lib().rth_fc_x9_workspace(M, N, K), 16) // 4, device=dev)
    fn = lambda: _lib.call("rth_fc_x9", x.data_ptr(), K, M, w.data_ptr(), N, K, b.data_ptr(), 1, y.data_ptr(),
                           ws.data_ptr(), _lib.stream_ptr())
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    ev = []
    for _ in range(40):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        ev.append((e0, e1))
    torch.cuda.synchronize()
    us = sorted(a.elapsed_time(c) * 1e3 for a, c in ev)[len(ev) // 2]
    ref = torch.relu(x.double() @ w.double().t() + b.double())
    err = float((y.double() - ref).abs().max())
    res[M] = y.cpu()
    print(f"pipe={os.environ.get('RTH_FC_PIPE', '1')} M={M}: {us:6.1f} us median "
          f"({2.0 * M * N * K / us / 1e6:6.1f} TF/s fp32-equivalent), err vs fp64 {err:.2e}", flush=True)
torch.save(res, sys.argv[1])
