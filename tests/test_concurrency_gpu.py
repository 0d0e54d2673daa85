"""Kernels sharing the CUs with another stream's launches (r06).  The Ape-X loop runs the actor
block and the learner block concurrently on two streams; a launch must give the same bits
whatever runs beside it.  r06 found the actors' counted FC1 tail rows (k_linear_relu_rows'
scheme) returning wrong sums -- single outputs off by one float4's worth of products, in 6-60 %
of the launches -- while k_fc_x9t's bf16-MFMA waves of the learner's FC1 shared the CUs, and
exact results from the same source compiled without the packed-FP32 VALU ops; the library is
built without them since (reth_amd._lib.HIPCC_FLAGS).  This repeats the actors' counted FC1 and
second layer on fixed inputs on one stream while the learner-shaped x9 FC1 runs on another, and
asserts every repetition equal to the first, and the first equal to fp64 within fp32 rounding."""
import pytest
import torch

from reth_amd._lib import c_vp, call, lib, ptr

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("form", ["x9_rows_upto", "rows_upto"])
def test_counted_fc1_rows_exact_beside_concurrent_x9(form):
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev)
    g.manual_seed(1)
    N, F, O, A, reps = 256, 3136, 512, 6, 200
    h = torch.rand((2 * N, F), device=dev, generator=g)
    w1 = (torch.rand((O, F), device=dev, generator=g) - 0.5) * 0.05
    b1 = (torch.rand(O, device=dev, generator=g) - 0.5) * 0.1
    fc2 = [(torch.rand((A, O // 2), device=dev, generator=g) - 0.5) * 0.1,
           (torch.rand((1, O // 2), device=dev, generator=g) - 0.5) * 0.1, torch.zeros(A, device=dev),
           torch.zeros(1, device=dev)]
    arr = (c_vp * 4)(*[p.data_ptr() for p in fc2])
    n_dev = torch.tensor([N + 3], dtype=torch.int64, device=dev)  # three counted rows behind the fixed ones
    h1 = torch.zeros((2 * N, O), device=dev)
    out = torch.zeros((2 * N, A + 1), device=dev)
    ws = torch.empty(max(lib().rth_fc_x9_workspace(N, O, F), 16) // 4, device=dev)
    hist = torch.zeros((reps, 3, O), device=dev)
    hq = torch.zeros((reps, 3, A + 1), device=dev)
    xl = torch.rand((4 * N, F), device=dev, generator=g)  # the learner's FC1 on the other stream
    wl = w1.clone()
    yl = torch.empty((4 * N, O), device=dev)
    wsl = torch.empty(max(lib().rth_fc_x9_workspace(4 * N, O, F), 16) // 4, device=dev)
    torch.cuda.synchronize()
    sa, sb = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
    for i in range(reps):
        with torch.cuda.stream(sa):
            h1[N:].fill_(float("nan"))
            if form == "x9_rows_upto":
                call("rth_fc_x9_rows_upto", ptr(h), F, N, 2 * N, ptr(n_dev), ptr(w1), O, F, ptr(b1), ptr(h1), ptr(ws),
                     sa.cuda_stream)
            else:
                call("rth_linear_relu_rows_upto", ptr(h), F, N, 2 * N, ptr(n_dev), ptr(w1), ptr(b1), F, O, ptr(h1), O,
                     sa.cuda_stream)
            call("rth_heads_fc2_upto", ptr(h1), O, 2 * N, ptr(n_dev), O // 2, A, arr, ptr(out), None, None,
                 sa.cuda_stream)
            hist[i].copy_(h1[N:N + 3])
            hq[i].copy_(out[N:N + 3])
        with torch.cuda.stream(sb):
            for _ in range(2):
                call("rth_fc_x9", ptr(xl), F, 4 * N, ptr(wl), O, F, ptr(b1), 1, ptr(yl), ptr(wsl), sb.cuda_stream)
    torch.cuda.synchronize()
    bad = [i for i in range(reps) if not (torch.equal(hist[i], hist[0]) and torch.equal(hq[i], hq[0]))]
    assert not bad, f"{len(bad)} of {reps} repetitions differ (first {bad[:8]})"
    ref = torch.relu(h[N:N + 3].double() @ w1.double().t() + b1.double())
    assert float((hist[0].double() - ref).abs().max()) < 1e-5
