"""Development aid: the FC1 forward GEMMs through the committed TunableOp results (the
solutions the loop uses): run-to-run bit equality and the error against an fp64 reference;
run under rocprofv3 --kernel-trace to see which kernels they are."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from reth_amd import gemm_tuning  # noqa: E402

print("results file:", gemm_tuning.enable(tune_missing=False), flush=True)
dev = torch.device("cuda:0")
g = torch.Generator(device=dev).manual_seed(0)
w = torch.randn(512, 3136, device=dev, generator=g) * 0.02
b = torch.randn(512, device=dev, generator=g) * 0.02
for rows in (512, 1024):
    x = torch.rand(rows, 3136, device=dev, generator=g)
    ys = [F.linear(x, w, b) for _ in range(5)]
    torch.cuda.synchronize()
    same = all(torch.equal(ys[0], y) for y in ys[1:])
    ref = (x.double() @ w.double().t() + b.double())
    err = ((ys[0].double() - ref).abs() / (ref.abs() + 1e-3)).max().item()
    print(f"rows {rows}: bit-identical over 5 runs: {same}; max rel err vs fp64 {err:.2e}", flush=True)
