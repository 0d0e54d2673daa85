"""The explicit learner gradient pass (reth_amd/fused_learner.py) against torch.autograd over
the same network: rth_heads_backward against the addmm -> relu autograd chain, and the whole
pass (one 2B forward, TD, backward) against DQNSolver's autograd path and the reference's
update (golden vectors, dqn_solver.py:104-124) on uint8 stacks."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("B,H2,A1", [(512, 512, 7), (37, 64, 5), (8, 512, 19)])
def test_heads_backward_matches_autograd(dev, B, H2, A1):
    from reth_amd._lib import call, ptr, stream_ptr

    g = torch.Generator(device=dev).manual_seed(B + A1)
    h = torch.relu(torch.randn(B, H2, device=dev, generator=g))
    w2 = torch.randn(A1, H2, device=dev, generator=g) * 0.05
    dq = torch.randn(B, A1, device=dev, generator=g) * 1e-3
    td = torch.rand(B, device=dev, generator=g)
    acc = torch.full((), 0.25, device=dev)
    gh, gw2 = torch.empty(B, H2, device=dev), torch.empty(A1, H2, device=dev)
    gb2, gb1 = torch.empty(A1, device=dev), torch.empty(H2, device=dev)
    call("rth_heads_backward", ptr(dq), ptr(h), H2, ptr(w2), B, H2, A1, ptr(gh), ptr(gw2), ptr(gb2), ptr(gb1),
         ptr(td), ptr(acc), stream_ptr())
    # autograd of heads = addmm(b2, h, w2^T), h = relu(pre)
    hh = h.clone().requires_grad_(True)
    ww = w2.clone().requires_grad_(True)
    bb = torch.zeros(A1, device=dev, requires_grad=True)
    torch.addmm(bb, hh, ww.t()).backward(dq)
    want_gh = torch.ops.aten.threshold_backward(hh.grad, h, 0)
    torch.testing.assert_close(gh, want_gh, rtol=1e-5, atol=1e-9)
    torch.testing.assert_close(gw2, ww.grad, rtol=1e-5, atol=1e-8)
    torch.testing.assert_close(gb2, bb.grad, rtol=1e-5, atol=1e-9)
    torch.testing.assert_close(gb1, want_gh.sum(0), rtol=1e-5, atol=1e-8)
    torch.testing.assert_close(acc, 0.25 + td.mean(), rtol=1e-6, atol=0)
    # deterministic
    gh2 = torch.empty_like(gh)
    call("rth_heads_backward", ptr(dq), ptr(h), H2, ptr(w2), B, H2, A1, ptr(gh2), ptr(gw2), ptr(gb2), ptr(gb1),
         None, None, stream_ptr())
    assert torch.equal(gh, gh2)


def _solver(dev, seed):
    from reth_amd.solver import Box, DQNSolver, Discrete

    torch.manual_seed(seed)
    return DQNSolver(Box(0, 255, (4, 84, 84)), Discrete(6), gamma=0.99, clip_value=40, double_q=True, dueling=True,
                     learning_rate=1e-4, adam_epsilon=1.5e-4, update_target_interval=100, device=dev, n_step=3,
                     channels_last=True)


@pytest.mark.parametrize("u8,adjacent,hip_dgrad,hip_wgrad", [(True, True, {1}, None), (True, False, {1}, None),
                                                             (False, False, {1}, None), (True, True, set(), None),
                                                             (True, True, {1, 2}, None), (True, True, {1}, "f32"),
                                                             (True, True, {1}, "x9")])
def test_fused_grads_match_autograd(dev, u8, adjacent, hip_dgrad, hip_wgrad, monkeypatch):
    from reth_amd import fused_learner

    monkeypatch.setattr(fused_learner, "HIP_DGRAD", hip_dgrad)  # layers whose data gradient is rth_conv_dgrad's
    monkeypatch.setattr(fused_learner, "HIP_WGRAD", hip_wgrad)  # conv2/conv3 weight gradients: MIOpen / f32 / x9

    B = 64
    g = torch.Generator(device=dev).manual_seed(5)
    frames = torch.randint(0, 256, (2 * B, 4, 84, 84), dtype=torch.uint8, device=dev, generator=g)
    s0, s1 = frames[:B], frames[B:]
    if not adjacent:
        s1 = s1.clone()  # separate allocation -> the pass concatenates
    if not u8:
        s0 = s0.float().contiguous(memory_format=torch.channels_last)
        s1 = s1.float().contiguous(memory_format=torch.channels_last)
    a = torch.randint(0, 6, (B,), device=dev, generator=g)
    r = (torch.rand(B, device=dev, generator=g) < 0.3).float()
    done = (torch.rand(B, device=dev, generator=g) < 0.1).float()
    isw = torch.rand(B, device=dev, generator=g, dtype=torch.float64) + 0.5
    solver = _solver(dev, 7)
    for p in solver.target_q_network.parameters():  # target != online
        p.data.add_(torch.randn_like(p) * 1e-3)
    solver.target_q_network.freeze_heads()
    assert fused_learner.eligible(solver.q_network, s0, s1)
    res = {}
    for fused in (True, False):
        solver.fused_grads = fused
        td = solver.compute_grads([s0, a, r, s1, done], weights=isw)
        res[fused] = (td.clone(), float(solver.last_loss), [p.grad.clone() for p in solver.q_network.parameters()])
    torch.testing.assert_close(res[True][0], res[False][0], rtol=1e-5, atol=1e-6)
    assert abs(res[True][1] - res[False][1]) <= 1e-5 * max(1.0, abs(res[False][1]))
    for (name, _), x, y in zip(solver.q_network.named_parameters(), res[True][2], res[False][2]):
        err = ((x - y).abs().max() / y.abs().max().clamp_min(1e-30)).item()
        assert err < 1e-4, (name, err)


@pytest.mark.parametrize("name", ["dqn_pong_b8.npz", "dqn_pong_b32.npz"])
def test_fused_update_u8_vs_reference(golden, dev, name):
    """DQNSolver.update on uint8 stacks (the apex learner's input) through the fused pass
    vs the reference's torch-CPU update on the same frames as float32"""
    gd = golden(name)
    solver = _solver(dev, int(gd["seed"]))
    assert np.array_equal(gd["s0"], gd["s0"].astype(np.uint8)) and np.array_equal(gd["s1"], gd["s1"].astype(np.uint8))
    B = gd["s0"].shape[0]
    frames = torch.as_tensor(np.concatenate([gd["s0"], gd["s1"]]).astype(np.uint8), device=dev)
    batch = [frames[:B], gd["a"], gd["r"], frames[B:], gd["done"]]
    for k in range(2):
        td = solver.update(batch, weights=gd["isw"]).numpy()
        np.testing.assert_allclose(td, gd[f"upd{k}_abs_td"], rtol=1e-5, atol=1e-5)
        sd = solver.q_network.state_dict()
        head = np.stack([np.pad(v.flatten()[:16].float().cpu().numpy(), (0, max(0, 16 - v.numel())),
                                constant_values=np.nan) for v in sd.values()])
        np.testing.assert_allclose(head, gd[f"upd{k}_head"], rtol=1e-4, atol=2e-6)


def test_batch_slots_keep_s1_behind_s0(dev):
    from reth_amd.actors import apex_columns
    from reth_amd.fused_learner import _pair
    from reth_amd.replay import HbmReplay

    rep = HbmReplay(1024, apex_columns(True, frames_u8=True), 0.5, "0.4,1,100", dev)
    cols, idx, isw = rep.new_batch(32)
    s0, s1 = cols[0], cols[3]
    assert s1.data_ptr() == s0.data_ptr() + s0.numel()
    x = _pair(s0, s1)
    assert x.data_ptr() == s0.data_ptr() and x.shape[0] == 64


@pytest.mark.parametrize("B,A,double_q", [(512, 6, 1), (37, 4, 1), (64, 18, 0)])
def test_td_heads_backward_equals_two_launches(dev, B, A, double_q):
    """rth_td_heads_backward (TD rows recomputed per workgroup in LDS) gives exactly the |td|
    and gradients of rth_td_huber + rth_heads_backward; the loss within fp32 rounding"""
    from reth_amd._lib import call, ptr, stream_ptr

    g = torch.Generator(device=dev).manual_seed(B + A)
    A1, H2 = A + 1, 512
    q0, q1o, q1t = (torch.randn(B, A1, device=dev, generator=g) for _ in range(3))
    a = torch.randint(0, A, (B,), device=dev, generator=g)
    r = torch.randn(B, device=dev, generator=g)
    done = (torch.rand(B, device=dev, generator=g) < 0.2).float()
    isw = torch.rand(B, device=dev, generator=g, dtype=torch.float64) + 0.5
    h = torch.relu(torch.randn(B, H2, device=dev, generator=g))
    w2 = torch.randn(A1, H2, device=dev, generator=g) * 0.05
    gn = float(np.float32(0.99 ** 3))
    outs = []
    for fused in (True, False):
        td = torch.empty(B, device=dev)
        loss = torch.empty(1, device=dev)
        gh, gw2 = torch.empty(B, H2, device=dev), torch.empty(A1, H2, device=dev)
        gb2, gb1 = torch.empty(A1, device=dev), torch.empty(H2, device=dev)
        acc = torch.zeros((), device=dev)
        if fused:
            call("rth_td_heads_backward", ptr(q0), ptr(q1o), ptr(q1t), ptr(a), ptr(r), ptr(done), ptr(isw), B, A, gn,
                 double_q, ptr(h), H2, ptr(w2), H2, ptr(td), ptr(loss), ptr(gh), ptr(gw2), ptr(gb2), ptr(gb1),
                 ptr(acc), stream_ptr())
        else:
            dq = torch.empty(B, A1, device=dev)
            call("rth_td_huber", ptr(q0), ptr(q1o), ptr(q1t), ptr(a), ptr(r), ptr(done), ptr(isw), B, A, gn, double_q,
                 1, None, ptr(td), None, ptr(loss), ptr(dq), stream_ptr())
            call("rth_heads_backward", ptr(dq), ptr(h), H2, ptr(w2), B, H2, A1, ptr(gh), ptr(gw2), ptr(gb2), ptr(gb1),
                 ptr(td), ptr(acc), stream_ptr())
        outs.append((td, gh, gw2, gb2, gb1, acc, loss))
    for x, y in zip(outs[0][:6], outs[1][:6]):
        assert torch.equal(x, y)
    torch.testing.assert_close(outs[0][6], outs[1][6], rtol=1e-6, atol=0)


@pytest.mark.parametrize("B,A,fused", [(512, 6, True), (37, 4, True), (64, 18, False), (300, 6, False)])
def test_heads_backward_branch_form_equals_merged(dev, B, A, fused):
    """rth_(td_)heads_backward_branches (the second layer read and its gradients written in the
    reference's four tensors) == the merged block-diagonal form on the diagonal blocks, bit for
    bit (the off-diagonal weights are exact zeros in both); gh, gb1, |td| identical"""
    from reth_amd import _lib
    from reth_amd._lib import call, ptr, stream_ptr

    g = torch.Generator(device=dev).manual_seed(3 * B + A)
    H, A1 = 256, A + 1
    H2 = 2 * H
    q0, q1o, q1t = (torch.randn(B, A1, device=dev, generator=g) for _ in range(3))
    a = torch.randint(0, A, (B,), device=dev, generator=g)
    r = torch.randn(B, device=dev, generator=g)
    done = (torch.rand(B, device=dev, generator=g) < 0.2).float()
    isw = torch.rand(B, device=dev, generator=g, dtype=torch.float64) + 0.5
    h = torch.relu(torch.randn(B, H2, device=dev, generator=g))
    wa2, wv2 = torch.randn(A, H, device=dev, generator=g) * 0.05, torch.randn(1, H, device=dev, generator=g) * 0.05
    w2 = torch.zeros(A1, H2, device=dev)
    w2[:A, :H], w2[A:, H:] = wa2, wv2
    gn = float(np.float32(0.99 ** 3))
    dq = torch.empty(B, A1, device=dev)
    td0 = torch.empty(B, device=dev)
    call("rth_td_huber", ptr(q0), ptr(q1o), ptr(q1t), ptr(a), ptr(r), ptr(done), ptr(isw), B, A, gn, 1, 1, None,
         ptr(td0), None, ptr(torch.empty(1, device=dev)), ptr(dq), stream_ptr())
    outs = []
    for branches in (False, True):
        td, loss, acc = torch.empty(B, device=dev), torch.empty(1, device=dev), torch.zeros((), device=dev)
        gh, gb1 = torch.empty(B, H2, device=dev), torch.empty(H2, device=dev)
        gw2, gb2 = torch.full((A1, H2), float("nan"), device=dev), torch.empty(A1, device=dev)
        g2 = [torch.empty(A, H, device=dev), torch.empty(1, H, device=dev), torch.empty(A, device=dev),
              torch.empty(1, device=dev)]
        pa = (_lib.c_vp * 4)(wa2.data_ptr(), wv2.data_ptr(), None, None)
        ga = (_lib.c_vp * 4)(*[t.data_ptr() for t in g2])
        if fused and branches:
            call("rth_td_heads_backward_branches", ptr(q0), ptr(q1o), ptr(q1t), ptr(a), ptr(r), ptr(done), ptr(isw), B,
                 A, gn, 1, ptr(h), H2, pa, H, ptr(td), ptr(loss), ptr(gh), ga, ptr(gb1), ptr(acc), stream_ptr())
        elif fused:
            call("rth_td_heads_backward", ptr(q0), ptr(q1o), ptr(q1t), ptr(a), ptr(r), ptr(done), ptr(isw), B, A, gn,
                 1, ptr(h), H2, ptr(w2), H2, ptr(td), ptr(loss), ptr(gh), ptr(gw2), ptr(gb2), ptr(gb1), ptr(acc),
                 stream_ptr())
        elif branches:
            call("rth_heads_backward_branches", ptr(dq), ptr(h), H2, pa, H, B, A, ptr(gh), ga, ptr(gb1), ptr(td0),
                 ptr(acc), stream_ptr())
        else:
            call("rth_heads_backward", ptr(dq), ptr(h), H2, ptr(w2), B, H2, A1, ptr(gh), ptr(gw2), ptr(gb2), ptr(gb1),
                 ptr(td0), ptr(acc), stream_ptr())
        if not branches:
            g2 = [gw2[:A, :H], gw2[A:, H:], gb2[:A], gb2[A:]]
        outs.append((gh, gb1, acc, *g2) + ((td,) if fused else ()))
    for x, y in zip(*outs):
        assert torch.equal(x, y)


@pytest.mark.parametrize("n,A", [(1, 6), (260, 6), (1024, 4), (33, 7), (64, 9), (300, 18), (17, 32)])
def test_heads_fc2_forward(dev, n, A):
    """rth_heads_fc2 (the second layer from the branch parameters) == the block-diagonal
    addmm within fp32 summation error, against an fp64 reference, for every action count up
    to kMaxActions = 32 (BeamRider's 9, the full Atari set's 18); more are refused"""
    from reth_amd import _lib
    from reth_amd._lib import call, ptr, stream_ptr

    g = torch.Generator(device=dev).manual_seed(n + A)
    H = 256
    h = torch.relu(torch.randn(n, 2 * H, device=dev, generator=g))
    ps = [torch.randn(A, H, device=dev, generator=g) * 0.05, torch.randn(1, H, device=dev, generator=g) * 0.05,
          torch.randn(A, device=dev, generator=g), torch.randn(1, device=dev, generator=g)]
    out = torch.full((n, A + 1), float("nan"), device=dev)
    call("rth_heads_fc2", ptr(h), 2 * H, n, H, A, (_lib.c_vp * 4)(*[p.data_ptr() for p in ps]), ptr(out),
         stream_ptr())
    hd = h.double()
    want = torch.cat([hd[:, :H] @ ps[0].double().t() + ps[2].double(), hd[:, H:] @ ps[1].double().t() + ps[3].double()],
                     1)
    torch.testing.assert_close(out.double(), want, rtol=1e-5, atol=1e-5)
    big = [torch.zeros(33, H, device=dev), ps[1], torch.zeros(33, device=dev), ps[3]]
    with pytest.raises(_lib.RethHipError):
        call("rth_heads_fc2", ptr(h), 2 * H, n, H, 33, (_lib.c_vp * 4)(*[p.data_ptr() for p in big]), ptr(out),
             stream_ptr())


@pytest.mark.parametrize("n,A,counts", [(512, 6, [0, 255, 256, 257, 300, 512, 600]), (40, 9, [0, 1, 17, 40]),
                                        (33, 32, [5, 33])])
def test_heads_fc2_upto_and_cache(dev, n, A, counts):
    """rth_heads_fc2_upto == rth_heads_fc2 bit for bit on the counted rows (the same launch
    arithmetic), rows past the count untouched; the cache rows receive the same heads and no
    other cache row is written"""
    from reth_amd import _lib
    from reth_amd._lib import call, ptr, stream_ptr

    g = torch.Generator(device=dev).manual_seed(n * A)
    H = 512
    h = torch.relu(torch.randn(n, 2 * H, device=dev, generator=g))
    ps = [torch.randn(A, H, device=dev, generator=g) * 0.05, torch.randn(1, H, device=dev, generator=g) * 0.05,
          torch.randn(A, device=dev, generator=g), torch.randn(1, device=dev, generator=g)]
    arr = (_lib.c_vp * 4)(*[p.data_ptr() for p in ps])
    want = torch.empty((n, A + 1), device=dev)
    call("rth_heads_fc2", ptr(h), 2 * H, n, H, A, arr, ptr(want), stream_ptr())
    stacks = 3 * n + 1
    rows = torch.randperm(stacks, device=dev, generator=g)[:n]
    for c in counts:
        cnt = torch.tensor([c], dtype=torch.int64, device=dev)
        out = torch.full((n, A + 1), float("nan"), device=dev)
        cache = torch.full((stacks, A + 1), -3.0, device=dev)
        call("rth_heads_fc2_upto", ptr(h), 2 * H, n, ptr(cnt), H, A, arr, ptr(out), ptr(cache), ptr(rows), stream_ptr())
        k = min(c, n)
        assert torch.equal(out[:k], want[:k]) and bool(out[k:].isnan().all())
        assert torch.equal(cache[rows[:k]], want[:k])
        untouched = torch.ones(stacks, dtype=torch.bool, device=dev)
        untouched[rows[:k]] = False
        assert bool((cache[untouched] == -3.0).all())
        out2 = torch.full_like(out, float("nan"))  # without the cache
        call("rth_heads_fc2_upto", ptr(h), 2 * H, n, ptr(cnt), H, A, arr, ptr(out2), None, None, stream_ptr())
        assert torch.equal(out2[:k], want[:k])
    with pytest.raises(_lib.RethHipError):  # a cache without its rows
        call("rth_heads_fc2_upto", ptr(h), 2 * H, n, ptr(cnt), H, A, arr, ptr(out), ptr(cache), None, stream_ptr())


@pytest.mark.parametrize("n_max,r0,F,O", [(512, 256, 3136, 1024), (80, 40, 3136, 1024), (64, 0, 12, 6),
                                          (300, 100, 256, 130)])
def test_linear_relu_rows_upto(dev, n_max, r0, F, O):
    """rows r0 <= r < min(*n_dev, n_max) of relu(x w^T + b) within fp32 summation error of an
    fp64 reference; every other row untouched; deterministic (run twice, equal)"""
    from reth_amd._lib import call, ptr, stream_ptr

    g = torch.Generator(device=dev).manual_seed(F + O)
    x = torch.relu(torch.randn(n_max, F, device=dev, generator=g))
    w = torch.randn(O, F, device=dev, generator=g) * F ** -0.5
    b = torch.randn(O, device=dev, generator=g) * 0.1
    want = torch.relu(x.double() @ w.double().t() + b.double())
    for c in sorted({r0, r0 + 1, r0 + 7, r0 + 8, r0 + 9, (r0 + n_max) // 2, n_max, n_max + 5, 0}):
        cnt = torch.tensor([c], dtype=torch.int64, device=dev)
        y = torch.full((n_max, O), -1.0, device=dev)
        call("rth_linear_relu_rows_upto", ptr(x), F, r0, n_max, ptr(cnt), ptr(w), ptr(b), F, O, ptr(y), O, stream_ptr())
        hi = max(r0, min(c, n_max))
        torch.testing.assert_close(y[r0:hi].double(), want[r0:hi], rtol=1e-5, atol=1e-5)
        assert bool((y[:r0] == -1.0).all()) and bool((y[hi:] == -1.0).all())
        y2 = torch.full_like(y, -1.0)
        call("rth_linear_relu_rows_upto", ptr(x), F, r0, n_max, ptr(cnt), ptr(w), ptr(b), F, O, ptr(y2), O,
             stream_ptr())
        assert torch.equal(y, y2)


def test_forward_heads_counted_matches_full(dev):
    """forward_heads over a device-counted batch with n_fixed (FC1 GEMM over the fixed rows,
    rth_linear_relu_rows_upto behind them, the counted second layer + cache scatter) gives the
    uncounted forward's heads on every counted row, within fp32 GEMM blocking error; without
    n_fixed (one GEMM over all rows, the counted second layer + cache scatter) bit for bit"""
    from reth_amd.model import DQNNetwork

    torch.manual_seed(3)
    net = DQNNetwork((4, 84, 84), 6).to(dev, memory_format=torch.channels_last)
    net.hwc_features = True
    net.requires_grad_(False)
    net.freeze_heads()
    g = torch.Generator(device=dev).manual_seed(5)
    stacks = torch.randint(0, 256, (90, 4, 84, 84), dtype=torch.uint8, device=dev, generator=g)
    N = 32
    rows = torch.randint(0, 90, (2 * N,), device=dev, generator=g)
    with torch.no_grad():
        full = net.forward_heads(stacks, rows=rows)
        for k in (0, 1, 5, N):
            cnt = torch.tensor([N + k], dtype=torch.int64, device=dev)
            cache = torch.zeros((100, 7), device=dev)
            crow = torch.arange(2 * N, device=dev) + 30
            for nf in (N, None):
                cache.zero_()
                q = net.forward_heads(stacks, rows=rows, n_dev=cnt, n_fixed=nf, cache=(cache, crow))
                torch.testing.assert_close(q[:N + k], full[:N + k], rtol=1e-5, atol=1e-5)
                if nf is None:  # the same 2N-row GEMM: the same heads bit for bit
                    assert torch.equal(q[:N + k], full[:N + k])
                assert torch.equal(cache[crow[:N + k]], q[:N + k])
                assert bool((cache[:30] == 0).all()) and bool((cache[30 + N + k:] == 0).all())


def test_norm_in_backward_matches_clip_adam(dev, monkeypatch):
    """r06: clip_grad_norm_'s partials written by conv1's weight-gradient reduce launch
    (rth_conv1_relu_wgrad_norm) + rth_adam_prenormed against rth_clip_adam's two launches: the
    same gradients, the same step count, the norm and every updated tensor equal up to the
    norm's summation order (a fixed one: run to run bit-identical)"""
    from reth_amd import fused_learner

    # run-to-run determinism needs fixed-order conv2 / conv3 weight gradients: the default
    # rth_conv_wgrad_f32 (MIOpen's solvers differ in the last bits run to run)
    assert fused_learner.HIP_WGRAD == "f32"
    B = 64
    g = torch.Generator(device=dev).manual_seed(11)
    frames = torch.randint(0, 256, (2 * B, 4, 84, 84), dtype=torch.uint8, device=dev, generator=g)
    batch = [frames[:B], torch.randint(0, 6, (B,), device=dev, generator=g),
             (torch.rand(B, device=dev, generator=g) < 0.3).float(), frames[B:],
             (torch.rand(B, device=dev, generator=g) < 0.1).float()]
    isw = torch.rand(B, device=dev, generator=g, dtype=torch.float64) + 0.5
    res = {}
    for on in (True, False, True):
        monkeypatch.setattr(fused_learner, "NORM_IN_BACKWARD", on)
        solver = _solver(dev, 3)
        solver.clip_value = solver.optimizer.max_norm = 1.0  # the clip active (the gradient norm is ~10-100)
        tds, norms = [], []
        for _ in range(3):
            tds.append(solver.update_device(batch, weights=isw).clone())
            norms.append(float(solver.optimizer.total_norm))
        assert solver.optimizer._prenormed is None
        state = [p.detach().clone() for p in solver.q_network.parameters()]
        state += [solver.optimizer.state[p][k].clone() for p in solver.q_network.parameters()
                  for k in ("exp_avg", "exp_avg_sq")]
        res.setdefault(on, []).append((tds, norms, state, int(solver.optimizer._step)))
    (a,), (b, c) = res[False], res[True]
    assert b[3] == a[3] == 3
    for x, y in zip(b[2], c[2]):  # deterministic
        assert torch.equal(x, y)
    for k in range(3):
        assert abs(b[1][k] - a[1][k]) <= 1e-6 * a[1][k], (k, b[1][k], a[1][k])
        assert a[1][k] > 1.0  # clipped
    for x, y in zip(b[2], a[2]):
        torch.testing.assert_close(x, y, rtol=1e-5, atol=1e-7)
