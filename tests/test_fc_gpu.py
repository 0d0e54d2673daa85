"""rth_fc_x9: FC1 of the dueling heads (dqn_model.py:38-47, both branches' first Linear as one
[512, 3136] weight) on the exact-split bf16 MFMA, against a float64 CPU reference of
relu(x w^T + b): within fp32 summation error (the products are exact; only the order of the
fp32 sums differs from an fp32 GEMM), run-to-run bit-identical, every output written, the
split-K and single-split paths, a strided x and no bias / no ReLU."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _run(dev, x, w, b, relu, ldx=None):
    from reth_amd import _lib

    M, K = x.shape[0], w.shape[1]
    N = w.shape[0]
    ws = torch.empty(max(_lib.lib().rth_fc_x9_workspace(M, N, K), 16) // 4, device=dev)
    y = torch.full((M, N), float("nan"), device=dev)
    _lib.call("rth_fc_x9", x.data_ptr(), ldx or K, M, w.data_ptr(), N, K, b.data_ptr() if b is not None else None,
              int(relu), y.data_ptr(), ws.data_ptr(), _lib.stream_ptr())
    return y


@pytest.mark.parametrize("M", [64, 512, 1024, 2048])
def test_fc_x9_vs_fp64(dev, M):
    from reth_amd import _lib

    N, K = 512, 3136
    assert _lib.lib().rth_fc_x9_supported(M, N, K) == 1
    g = torch.Generator(device=dev).manual_seed(M)
    x = torch.rand((M, K), device=dev, generator=g) * 3  # post-ReLU features: non-negative, O(1)
    w = (torch.rand((N, K), device=dev, generator=g) * 2 - 1) / np.sqrt(K)
    b = (torch.rand(N, device=dev, generator=g) * 2 - 1) * 0.1
    y = _run(dev, x, w, b, True)
    y2 = _run(dev, x, w, b, True)
    assert torch.equal(y, y2)
    assert not torch.isnan(y).any()
    want = torch.relu(x.double().cpu() @ w.double().cpu().t() + b.double().cpu())
    err = (y.double().cpu() - want).abs().max().item()
    # fp32 sums of 3,136 products of magnitude ~ 3 / sqrt(K): the error of an fp32 GEMM
    ref32 = torch.relu(x.cpu() @ w.cpu().t() + b.cpu()).double()
    err32 = (ref32 - want).abs().max().item()
    assert err <= max(4 * err32, 2e-6), (err, err32)


def test_fc_x9_strided_no_bias_no_relu(dev):
    M, N, K = 128, 256, 96
    g = torch.Generator(device=dev).manual_seed(3)
    big = torch.randn((M, K + 32), device=dev, generator=g)
    x = big[:, :K]
    w = torch.randn((N, K), device=dev, generator=g)
    y = _run(dev, x, w, None, False, ldx=K + 32)
    want = x.double().cpu() @ w.double().cpu().t()
    assert (y.double().cpu() - want).abs().max().item() <= 1e-4


def test_fc_x9_unsupported(dev):
    from reth_amd import _lib

    assert _lib.lib().rth_fc_x9_supported(100, 512, 3136) == 0
    t = torch.zeros(16, device=dev)
    with pytest.raises(_lib.RethHipError, match="not built"):
        _lib.call("rth_fc_x9", t.data_ptr(), 3136, 100, t.data_ptr(), 512, 3136, None, 1, t.data_ptr(), None,
                  _lib.stream_ptr())
