"""rth_clip_adam (ClipAdam) against torch's clip_grad_norm_ + Adam on the same gradients
(the reference's dqn_solver.py:118-121 sequence): fp32 agreement over several steps, with
the clip active and inactive, on NCHW and channels-last (NHWC) conv weights -- through the
one-launch form (aligned tensors that fit its resident grid: the Q-net's) and the two-launch
form (an unaligned tensor, or more elements than the one-launch grid holds)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _params(dev, seed):
    g = torch.Generator(device=dev).manual_seed(seed)
    shapes = [(32, 4, 8, 8), (32,), (64, 32, 4, 4), (512, 3136), (7, 512), (3,)]
    ps = [torch.randn(s, device=dev, generator=g) * 0.05 for s in shapes]
    ps[2] = ps[2].contiguous(memory_format=torch.channels_last)
    return ps


def _unaligned(dev, seed):
    """the Q-net shapes with one parameter 4 bytes past a 16-byte boundary: the two-launch form"""
    ps = _params(dev, seed)
    buf = torch.empty(ps[4].numel() + 1, device=dev)
    buf[1:].copy_(ps[4].flatten())
    ps[4] = buf[1:].view(ps[4].shape)
    return ps


def _large(dev, seed):
    g = torch.Generator(device=dev).manual_seed(seed)
    return [torch.randn(s, device=dev, generator=g) * 0.05 for s in [(4096, 1100), (7,)]]  # > 256 x 8 x 2048


@pytest.mark.parametrize("max_norm", [None, 40.0, 0.5])
@pytest.mark.parametrize("kind", ["qnet", "unaligned", "large"])
def test_clip_adam_matches_torch(dev, max_norm, kind):
    from reth_amd import _lib
    from reth_amd.optim import ClipAdam

    make = {"qnet": _params, "unaligned": _unaligned, "large": _large}[kind]
    if kind != "qnet" and max_norm == 0.5:
        pytest.skip("the clip is covered by the other max_norm")
    ref = [torch.nn.Parameter(p.clone()) for p in make(dev, 1)]
    ours = [torch.nn.Parameter(p) for p in make(dev, 1)]  # (the unaligned view kept as it is)
    if kind == "unaligned":
        assert ours[4].data_ptr() % 16 == 4
    topt = torch.optim.Adam(ref, lr=1e-4, eps=1.5e-4, foreach=False)
    oopt = ClipAdam(ours, lr=1e-4, eps=1.5e-4, max_norm=max_norm)
    g = torch.Generator(device=dev).manual_seed(2)
    for step in range(5):
        grads = [torch.randn(p.shape, device=dev, generator=g) * (3.0 if step % 2 else 0.01) for p in ref]
        for p, q, gr in zip(ref, ours, grads):
            p.grad = gr.clone().contiguous(memory_format=torch.channels_last) if p.dim() == 4 else gr.clone()
            q.grad = p.grad.clone()
        if max_norm is not None:
            tn = torch.nn.utils.clip_grad_norm_(ref, max_norm, foreach=False)
        topt.step()
        oopt.step()
        if max_norm is not None:
            torch.testing.assert_close(oopt.total_norm[0], tn, rtol=1e-6, atol=0)
        # torch's CUDA kernels may fuse multiply-adds; agreement to a few f32 ulps of each
        # tensor's scale
        for p, q in zip(ref, ours):
            for x, y in ((q, p), (oopt.state[q]["exp_avg"], topt.state[p]["exp_avg"]),
                         (oopt.state[q]["exp_avg_sq"], topt.state[p]["exp_avg_sq"])):
                err = ((x - y).abs().max() / y.abs().max()).item()
                assert err < 1e-6, err
    assert int(oopt._step.item()) == 5
    if kind == "qnet":
        assert ours[2].is_contiguous(memory_format=torch.channels_last)


def test_clip_adam_many_steps_and_reset(dev):
    """60 steps, then a reset of Adam's state and step count alone, then of the workspace too --
    every step equal to the reference computed by torch"""
    from reth_amd import _lib
    from reth_amd.optim import ClipAdam

    ref = [torch.nn.Parameter(p.clone()) for p in _params(dev, 3)]
    ours = [torch.nn.Parameter(p.clone()) for p in _params(dev, 3)]
    topt = torch.optim.Adam(ref, lr=1e-4, eps=1.5e-4, foreach=False)
    oopt = ClipAdam(ours, lr=1e-4, eps=1.5e-4, max_norm=10.0)
    g = torch.Generator(device=dev).manual_seed(4)
    for step in range(90):
        if step in (60, 75):  # fresh Adam state; at 75 the workspace (call counter) zeroed as well
            for p, q in zip(ref, ours):
                topt.state[p]["exp_avg"].zero_()
                topt.state[p]["exp_avg_sq"].zero_()
                topt.state[p]["step"].zero_()
                oopt.state[q]["exp_avg"].zero_()
                oopt.state[q]["exp_avg_sq"].zero_()
            oopt._step.zero_()
            if step == 75:
                oopt._ws.zero_()
        grads = [torch.randn(p.shape, device=dev, generator=g) * 0.5 for p in ref]
        for p, q, gr in zip(ref, ours, grads):
            p.grad = gr.clone().contiguous(memory_format=torch.channels_last) if p.dim() == 4 else gr.clone()
            q.grad = p.grad.clone()
        tn = torch.nn.utils.clip_grad_norm_(ref, 10.0, foreach=False)
        topt.step()
        oopt.step()
        torch.testing.assert_close(oopt.total_norm[0], tn, rtol=1e-6, atol=0)
    for p, q in zip(ref, ours):
        err = ((q - p).abs().max() / p.abs().max()).item()
        assert err < 1e-5, err
    assert int(oopt._step.item()) == 15


def test_clip_adam_skips_gradless_and_validates(dev):
    from reth_amd.optim import ClipAdam

    a, b = torch.nn.Parameter(torch.ones(10, device=dev)), torch.nn.Parameter(torch.ones(10, device=dev))
    opt = ClipAdam([a, b], lr=0.1)
    a.grad = torch.ones(10, device=dev)
    opt.step()
    assert torch.all(a < 1) and torch.equal(b, torch.ones(10, device=dev))
    with pytest.raises(ValueError):
        ClipAdam([torch.nn.Parameter(torch.ones(4, 4, device=dev).t())])
