"""rth_fc_x9 / rth_fc_f32: FC1 of the dueling heads (dqn_model.py:38-47, both branches' first
Linear as one [512, 3136] weight) on the exact-split bf16 MFMA and on the fp32 MFMA (r05),
against a float64 CPU reference of relu(x w^T + b): within fp32 summation error (the products
are exact; only the order of the fp32 sums differs from an fp32 GEMM), run-to-run
bit-identical, every output written, the split-K and single-split paths, a strided x, no bias /
no ReLU, and (rth_fc_f32) ragged row counts -- the actors' N + k live rows."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _run(dev, x, w, b, relu, ldx=None, kind="x9"):
    from reth_amd import _lib

    M, K = x.shape[0], w.shape[1]
    N = w.shape[0]
    fn = "rth_fc_" + kind
    ws = torch.empty(max(getattr(_lib.lib(), fn + "_workspace")(M, N, K), 16) // 4, device=dev)
    y = torch.full((M, N), float("nan"), device=dev)
    _lib.call(fn, x.data_ptr(), ldx or K, M, w.data_ptr(), N, K, b.data_ptr() if b is not None else None,
              int(relu), y.data_ptr(), ws.data_ptr(), _lib.stream_ptr())
    return y


def _check_vs_fp64(dev, M, kind):
    from reth_amd import _lib

    N, K = 512, 3136
    assert getattr(_lib.lib(), f"rth_fc_{kind}_supported")(M, N, K) == 1
    g = torch.Generator(device=dev).manual_seed(M)
    x = torch.rand((M, K), device=dev, generator=g) * 3  # post-ReLU features: non-negative, O(1)
    w = (torch.rand((N, K), device=dev, generator=g) * 2 - 1) / np.sqrt(K)
    b = (torch.rand(N, device=dev, generator=g) * 2 - 1) * 0.1
    y = _run(dev, x, w, b, True, kind=kind)
    y2 = _run(dev, x, w, b, True, kind=kind)
    assert torch.equal(y, y2)
    assert not torch.isnan(y).any()
    want = torch.relu(x.double().cpu() @ w.double().cpu().t() + b.double().cpu())
    err = (y.double().cpu() - want).abs().max().item()
    # fp32 sums of 3,136 products of magnitude ~ 3 / sqrt(K): the error of an fp32 GEMM
    ref32 = torch.relu(x.cpu() @ w.cpu().t() + b.cpu()).double()
    err32 = (ref32 - want).abs().max().item()
    assert err <= max(4 * err32, 2e-6), (err, err32)


@pytest.mark.parametrize("M", [64, 128, 192, 256, 320, 512, 1024, 2048])
def test_fc_x9_vs_fp64(dev, M):
    """every row count the loop runs (256 actors, 512 target rows, the learner's 1,024, Breakout's
    2,048 actors: the 128 x 128 tile at 16 / 16 / 8 / 4 k splits) and the 64 x 128 tile's (rows
    not a multiple of 128: 64, 192, 320)"""
    _check_vs_fp64(dev, M, "x9")


@pytest.mark.parametrize("M", [1, 64, 256, 259, 512, 1024, 2048])
def test_fc_f32_vs_fp64(dev, M):
    _check_vs_fp64(dev, M, "f32")


@pytest.mark.parametrize("kind", ["x9", "f32"])
def test_fc_strided_no_bias_no_relu(dev, kind):
    M, N, K = 128, 256, 96
    g = torch.Generator(device=dev).manual_seed(3)
    big = torch.randn((M, K + 32), device=dev, generator=g)
    x = big[:, :K]
    w = torch.randn((N, K), device=dev, generator=g)
    y = _run(dev, x, w, None, False, ldx=K + 32, kind=kind)
    want = x.double().cpu() @ w.double().cpu().t()
    assert (y.double().cpu() - want).abs().max().item() <= 1e-4


@pytest.mark.parametrize("kind", ["x9", "f32"])
def test_fc_strided_big_tile(dev, kind):
    """a strided x through the 128 x 128 x9 tile (M and N multiples of 128) and split-K"""
    M, N, K = 256, 256, 320
    g = torch.Generator(device=dev).manual_seed(5)
    big = torch.randn((M, K + 64), device=dev, generator=g)
    x = big[:, :K]
    w = torch.randn((N, K), device=dev, generator=g)
    b = torch.randn(N, device=dev, generator=g)
    y = _run(dev, x, w, b, True, ldx=K + 64, kind=kind)
    want = torch.relu(x.double().cpu() @ w.double().cpu().t() + b.double().cpu())
    assert (y.double().cpu() - want).abs().max().item() <= 1e-4


@pytest.mark.parametrize("kind", ["x9", "f32"])
def test_fc_unsupported(dev, kind):
    from reth_amd import _lib

    fn = "rth_fc_" + kind
    assert getattr(_lib.lib(), fn + "_supported")(100, 500, 3136) == 0
    t = torch.zeros(16, device=dev)
    with pytest.raises(_lib.RethHipError, match="not built"):
        _lib.call(fn, t.data_ptr(), 3136, 100, t.data_ptr(), 500, 3136, None, 1, t.data_ptr(), None,
                  _lib.stream_ptr())


@pytest.mark.parametrize("count", [256, 259, 300, 512])
def test_fc_x9_rows_upto_matches_two_launches(dev, count):
    """rth_fc_x9_rows_upto (the actors' counted FC1: the x9 GEMM over the 256 fixed rows, then
    its split-K reduce and the device-counted rows behind them in one launch) == rth_fc_x9 +
    rth_linear_relu_rows_upto, bit for bit; rows past the count untouched"""
    from reth_amd import _lib

    M, n_max, N, K = 256, 512, 512, 3136
    g = torch.Generator(device=dev).manual_seed(count)
    x = torch.rand((n_max, K), device=dev, generator=g) * 3
    w = (torch.rand((N, K), device=dev, generator=g) * 2 - 1) / 56
    b = (torch.rand(N, device=dev, generator=g) * 2 - 1) * 0.1
    n_dev = torch.tensor([count], dtype=torch.int64, device=dev)
    ws = torch.empty(_lib.lib().rth_fc_x9_workspace(M, N, K) // 4, device=dev)
    ys = []
    for fused in (True, False):
        y = torch.full((n_max, N), float("nan"), device=dev)
        if fused:
            _lib.call("rth_fc_x9_rows_upto", x.data_ptr(), K, M, n_max, n_dev.data_ptr(), w.data_ptr(), N, K,
                      b.data_ptr(), y.data_ptr(), ws.data_ptr(), _lib.stream_ptr())
        else:
            _lib.call("rth_fc_x9", x.data_ptr(), K, M, w.data_ptr(), N, K, b.data_ptr(), 1, y.data_ptr(), ws.data_ptr(),
                      _lib.stream_ptr())
            _lib.call("rth_linear_relu_rows_upto", x.data_ptr(), K, M, n_max, n_dev.data_ptr(), w.data_ptr(),
                      b.data_ptr(), K, N, y.data_ptr(), N, _lib.stream_ptr())
        ys.append(y)
    live = min(count, n_max)
    assert torch.equal(ys[0][:live], ys[1][:live])
    assert not torch.isnan(ys[0][:live]).any() and torch.isnan(ys[0][live:]).all()
    want = torch.relu(x[:live].double() @ w.double().t() + b.double())
    assert (ys[0][:live].double() - want).abs().max().item() < 1e-4


@pytest.mark.parametrize("M,A", [(512, 6), (1024, 6), (256, 4), (2048, 7), (512, 1)])
def test_fc1_heads_matches_two_launches(dev, M, A):
    """r06 rth_fc1_heads (the x9 GEMM, then its split-K reduce + bias + ReLU and the second layer
    of both dueling branches in one launch): heads and h1 bit-identical to rth_fc_x9 +
    rth_heads_fc2; run-to-run identical; shapes it does not build are refused"""
    from reth_amd import _lib

    N, K, H = 512, 3136, 256
    g = torch.Generator(device=dev).manual_seed(M + A)
    x = torch.randn((M, K), device=dev, generator=g)
    w1 = torch.randn((N, K), device=dev, generator=g) * 0.02
    b1 = torch.randn(N, device=dev, generator=g) * 0.1
    ps = [torch.randn((A, H), device=dev, generator=g) * 0.05, torch.randn((1, H), device=dev, generator=g) * 0.05,
          torch.randn(A, device=dev, generator=g) * 0.1, torch.randn(1, device=dev, generator=g) * 0.1]
    arr = (_lib.c_vp * 4)(*[p.data_ptr() for p in ps])
    assert _lib.lib().rth_fc1_heads_supported(M, N, K, A) == 1
    h1 = _run(dev, x, w1, b1, True)
    want = torch.full((M, A + 1), float("nan"), device=dev)
    _lib.call("rth_heads_fc2", h1.data_ptr(), N, M, H, A, arr, want.data_ptr(), _lib.stream_ptr())
    ws = torch.empty(max(_lib.lib().rth_fc_x9_workspace(M, N, K), 16) // 4, device=dev)
    outs = []
    for keep_h1 in (True, False, True):
        heads = torch.full((M, A + 1), float("nan"), device=dev)
        h1o = torch.full((M, N), float("nan"), device=dev) if keep_h1 else None
        _lib.call("rth_fc1_heads", x.data_ptr(), K, M, w1.data_ptr(), N, K, b1.data_ptr(), A, arr, heads.data_ptr(),
                  h1o.data_ptr() if keep_h1 else None, ws.data_ptr(), _lib.stream_ptr())
        assert torch.equal(heads, want)
        if keep_h1:
            assert torch.equal(h1o, h1)
        outs.append(heads)
    assert _lib.lib().rth_fc1_heads_supported(M, N, K, 8) == 0  # A + 1 > 8
    assert _lib.lib().rth_fc1_heads_supported(M, 1024, K, A) == 0  # N > 512
