"""Development aid: list TunableOp's candidate solutions and their isolated times for the FC1
forward shapes (actor / target pass: 512 rows, learner: 1,024 rows), so alternatives to the
isolated winner can be A/B-tested in the loop (RTH_TUNABLEOP_IN points the loop at a
variant results file).  Output: PyTorch's verbose tuning log on stderr."""
import os
import sys

os.environ.setdefault("PYTORCH_TUNABLEOP_ENABLED", "1")
os.environ.setdefault("PYTORCH_TUNABLEOP_TUNING", "1")
os.environ.setdefault("PYTORCH_TUNABLEOP_VERBOSE", "3")
os.environ.setdefault("PYTORCH_TUNABLEOP_FILENAME", os.path.join(os.getcwd(), "gpurun_out", "gemm_cand.csv"))

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

dev = torch.device("cuda:0")
w = torch.randn(512, 3136, device=dev) * 0.02
b = torch.randn(512, device=dev) * 0.02
for arg in (sys.argv[1:] or ["512", "1024"]):
    rows, bwd = int(arg.rstrip("b")), arg.endswith("b")  # "512b": also the backward (NN / NT GEMMs)
    x = torch.rand(rows, 3136, device=dev, requires_grad=bwd)
    wq = w.clone().requires_grad_(bwd)
    y = F.linear(x, wq, b)
    if bwd:
        y.backward(torch.randn_like(y))
    torch.cuda.synchronize()
    print(f"rows {rows}{' + backward' if bwd else ''}: done {tuple(y.shape)}", flush=True)
