"""Learner parity: the fused TD/Huber kernel is bit-exact against the oracle given the same
Q values; the full DQNSolver.update on the GPU matches the reference's torch-CPU update
(golden vectors) within north_star's fp32 tolerance (conv summation order differs)."""
import io

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

GAMMA_N = float(np.float32(0.99 ** 3))


@pytest.mark.parametrize("B,A", [(1, 2), (8, 6), (512, 6), (512, 18), (700, 4), (2048, 6)])
def test_td_huber_kernel_bit_exact(dev, orc, B, A):
    from reth_amd.solver import td_huber_forward

    rng = np.random.default_rng(B + A)
    q0, q1o, q1t = (rng.standard_normal((B, A)).astype(np.float32) * 3 for _ in range(3))
    q1o[: B // 4] = np.round(q1o[: B // 4])  # argmax ties
    a = rng.integers(0, A, B)
    r = rng.choice(np.array([-1, 0, 1], np.float32), B)
    done = (rng.random(B) < 0.3).astype(np.float32)
    isw = rng.random(B) + 0.1
    T = lambda x: torch.as_tensor(x, device=dev)
    for double_q in (True, False):
        loss, td_abs, dq = td_huber_forward(T(q0), T(q1o), T(q1t), T(a), T(r), T(done), T(isw), GAMMA_N, double_q, True)
        td = orc.td_error(q0, q1o if double_q else None, q1t, a, r, done, GAMMA_N, double_q)
        assert np.array_equal(td_abs.cpu().numpy(), np.abs(td))
        ol, _, odq = orc.td_huber(td, isw.astype(np.float32), a, A)
        assert np.array_equal(dq.cpu().numpy(), odq)
        assert abs(loss.item() - float(ol)) <= 1e-6 * max(1.0, abs(float(ol)))
    # no IS weights
    loss, td_abs, dq = td_huber_forward(T(q0), T(q1o), T(q1t), T(a), T(r), T(done), None, GAMMA_N, True, True)
    _, _, odq = orc.td_huber(orc.td_error(q0, q1o, q1t, a, r, done, GAMMA_N), None, a, A)
    assert np.array_equal(dq.cpu().numpy(), odq)


def test_td_huber_autograd_matches_torch_reference(dev):
    """the custom autograd op == the reference's op chain (dqn_solver.py:77-115) on device"""
    import torch.nn.functional as F

    from reth_amd.solver import td_huber_loss

    B, A = 512, 6
    g = torch.Generator(device=dev).manual_seed(0)
    q0 = torch.randn(B, A, device=dev, generator=g, requires_grad=True)
    q1o, q1t = torch.randn(B, A, device=dev, generator=g), torch.randn(B, A, device=dev, generator=g)
    a = torch.randint(0, A, (B,), device=dev, generator=g)
    r = torch.randn(B, device=dev, generator=g)
    done = (torch.rand(B, device=dev, generator=g) < 0.2).float()
    w = torch.rand(B, device=dev, generator=g, dtype=torch.float64)
    loss, td_abs = td_huber_loss(q0, q1o, q1t, a, r, done, w, GAMMA_N, True)
    loss.backward()
    ours = q0.grad.clone()
    q0.grad = None
    qv = torch.sum(q0 * F.one_hot(a, A).float(), 1)
    nqb = torch.sum(q1t * F.one_hot(torch.argmax(q1o, 1), A).float(), 1)
    td = qv - (r + (0.99 ** 3) * nqb * (1 - done)).detach()
    ref = (F.smooth_l1_loss(td, torch.zeros_like(td), reduction="none") * w.float()).mean()
    ref.backward()
    torch.testing.assert_close(td_abs, td.detach().abs(), rtol=0, atol=0)
    torch.testing.assert_close(ours, q0.grad, rtol=0, atol=0)
    torch.testing.assert_close(loss, ref, rtol=1e-6, atol=1e-7)


@pytest.mark.parametrize("B,A", [(8, 6), (512, 6), (512, 18)])
def test_td_huber_dueling_heads(dev, orc, B, A):
    """dueling mode: the kernel forms Q from raw heads [B, A+1]; td bit-exact against the
    oracle on the f32 restatement of the combine, d(loss)/d(heads) to 1e-6 against torch
    autograd through the reference's combine (dqn_model.py:192-193)"""
    from test_actor_gpu import dueling_q

    from reth_amd.solver import td_huber_forward, td_huber_loss

    rng = np.random.default_rng(100 + B + A)
    h0, h1o, h1t = ((rng.standard_normal((B, A + 1)) * 3).astype(np.float32) for _ in range(3))
    a = rng.integers(0, A, B)
    r = rng.choice(np.array([-1, 0, 1], np.float32), B)
    done = (rng.random(B) < 0.3).astype(np.float32)
    isw = rng.random(B) + 0.1
    T = lambda x: torch.as_tensor(x, device=dev)
    loss, td_abs, dq = td_huber_forward(T(h0), T(h1o), T(h1t), T(a), T(r), T(done), T(isw), GAMMA_N, True, True,
                                        dueling=True)
    q0, q1o, q1t = dueling_q(h0), dueling_q(h1o), dueling_q(h1t)
    td = orc.td_error(q0, q1o, q1t, a, r, done, GAMMA_N, True)
    assert np.array_equal(td_abs.cpu().numpy(), np.abs(td))
    ol, _, odq = orc.td_huber(td, isw.astype(np.float32), a, A)
    assert abs(loss.item() - float(ol)) <= 1e-6 * max(1.0, abs(float(ol)))
    # gradient through the combine, torch autograd on the same dq
    hh = torch.as_tensor(h0, device=dev).requires_grad_(True)
    adv, val = hh[:, :A], hh[:, A:]
    (val + adv - adv.mean(dim=1, keepdim=True)).backward(T(odq))
    # the kernel divides by A as CPU torch does (mean_backward); CUDA torch multiplies by 1/A
    torch.testing.assert_close(dq, hh.grad, rtol=1e-6, atol=0)
    # the autograd op routes the heads gradient
    hh2 = torch.as_tensor(h0, device=dev).requires_grad_(True)
    l2, _ = td_huber_loss(hh2, T(h1o), T(h1t), T(a), T(r), T(done), T(isw), GAMMA_N, True, True)
    l2.backward()
    assert torch.equal(hh2.grad, dq)


def test_dueling_heads_forward_matches_module(dev):
    """merged-heads forward (one FC1 GEMM + block-diagonal FC2) == the module's forward"""
    from reth_amd.model import DQNNetwork

    torch.manual_seed(5)
    net = DQNNetwork((4, 84, 84), 6).to(dev)
    x = torch.rand(64, 4, 84, 84, device=dev) * 255
    with torch.no_grad():
        ref = net(x)
        h = net.forward_heads(x)
        adv, val = h[:, :6], h[:, 6:]
        torch.testing.assert_close(val + adv - adv.mean(1, keepdim=True), ref, rtol=1e-5, atol=1e-5)
        net.freeze_heads()
        torch.testing.assert_close(net.forward_heads(x), h, rtol=1e-6, atol=1e-6)


@pytest.mark.parametrize("C,hw", [(32, 20), (64, 9), (64, 7), (4, 3)])
def test_conv_epilogue_kernels(dev, C, hw):
    """rth_bias_relu == relu(conv + b) bit for bit; rth_relu_bias_grad: the mask bit for bit,
    the channel sums deterministic and within fp32 summation error of torch's"""
    from reth_amd import _lib

    g0 = torch.Generator(device=dev).manual_seed(C + hw)
    n = 37
    y = torch.randn(n, C, hw, hw, device=dev, generator=g0).contiguous(memory_format=torch.channels_last)
    b = torch.randn(C, device=dev, generator=g0)
    ref = torch.relu(y + b.view(1, C, 1, 1))
    out = y.clone()
    _lib.call("rth_bias_relu", out.data_ptr(), b.data_ptr(), n * hw * hw, C, _lib.stream_ptr())
    assert torch.equal(out, ref)
    g = torch.randn(n, C, hw, hw, device=dev, generator=g0).contiguous(memory_format=torch.channels_last)
    ws = torch.zeros(_lib.lib().rth_relu_bias_grad_workspace(C), dtype=torch.uint8, device=dev)
    dbs = []
    for _ in range(3):  # the workspace re-arms itself
        gy = torch.empty_like(out)
        db = torch.empty(C, device=dev)
        _lib.call("rth_relu_bias_grad", g.data_ptr(), out.data_ptr(), gy.data_ptr(), db.data_ptr(), ws.data_ptr(),
                  n * hw * hw, C, _lib.stream_ptr())
        dbs.append(db)
    assert torch.equal(gy, torch.ops.aten.threshold_backward(g, out, 0))
    assert torch.equal(dbs[0], dbs[1]) and torch.equal(dbs[0], dbs[2])
    torch.testing.assert_close(dbs[0], gy.sum((0, 2, 3)), rtol=1e-5, atol=1e-4)  # ~2k-term fp32 sums


def test_nhwc_features_forward_backward_match_module(dev):
    """the HIP-epilogue channels-last torso (the last conv written NCHW, FC1 on the tied
    storage) == the reference module (values and every parameter gradient, fp32 tolerance)"""
    from reth_amd.model import DQNNetwork

    torch.manual_seed(11)
    net = DQNNetwork((4, 84, 84), 6).to(dev, memory_format=torch.channels_last)
    x = (torch.rand(48, 4, 84, 84, device=dev) * 255).floor().contiguous(memory_format=torch.channels_last)
    ref = net(x)
    ref.square().sum().backward()
    gref = [p.grad.clone() for p in net.parameters()]
    net.zero_grad()
    net.hwc_features = True
    h = net.forward_heads(x)
    adv, val = h[:, :6], h[:, 6:]
    q = val + adv - adv.mean(1, keepdim=True)
    torch.testing.assert_close(q, ref, rtol=1e-5, atol=1e-5)
    q.square().sum().backward()
    for (name, p), gr in zip(net.named_parameters(), gref):
        err = ((p.grad - gr).abs().max() / gr.abs().max()).item()  # relative to the tensor's scale
        assert err < 1e-5, (name, err)


def _make_solver(dev, seed, **kw):
    from reth_amd.solver import Box, DQNSolver, Discrete

    torch.manual_seed(seed)
    args = dict(gamma=0.99, clip_value=40, double_q=True, dueling=True, learning_rate=1e-4, adam_epsilon=1.5e-4,
                update_target_interval=100, device=dev, n_step=3)
    args.update(kw)
    return DQNSolver(Box(0, 255, (4, 84, 84)), Discrete(6), **args)


@pytest.mark.parametrize("name", ["dqn_pong_b8.npz", "dqn_pong_b32.npz"])
@pytest.mark.parametrize("fused,channels_last", [(True, False), (False, False), (True, True)])
def test_dqn_update_vs_reference(golden, dev, name, fused, channels_last):
    g = golden(name)
    solver = _make_solver(dev, int(g["seed"]), fused_adam=fused, channels_last=channels_last)
    batch = [g["s0"].astype(np.float32), g["a"], g["r"], g["s1"].astype(np.float32), g["done"]]
    with torch.no_grad():
        q0 = solver.q_network(torch.as_tensor(batch[0], device=dev)).cpu().numpy()
    np.testing.assert_allclose(q0, g["q_s0"], rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(solver.calc_loss(batch).numpy(), g["calc_loss"], rtol=1e-5, atol=1e-5)
    assert solver.act(batch[0][0]) == int(g["act0"])
    for k in range(2):
        td = solver.update(batch, weights=g["isw"]).numpy()
        np.testing.assert_allclose(td, g[f"upd{k}_abs_td"], rtol=1e-5, atol=1e-5)
        sd = solver.q_network.state_dict()
        s1 = np.array([float(v.double().sum()) for v in sd.values()])
        head = np.stack([np.pad(v.flatten()[:16].float().cpu().numpy(), (0, max(0, 16 - v.numel())),
                                constant_values=np.nan) for v in sd.values()])
        # one Adam step moves each weight by ~lr = 1e-4: fp32 agreement to ~1e-6 abs
        np.testing.assert_allclose(head, g[f"upd{k}_head"], rtol=1e-4, atol=2e-6)
        np.testing.assert_allclose(s1, g[f"upd{k}_sum"], rtol=1e-4, atol=1e-3)


def test_cartpole_mlp_three_updates(golden, dev):
    from reth_amd.solver import Box, DQNSolver, Discrete

    g = golden("dqn_cartpole_b64.npz")
    torch.manual_seed(int(g["seed"]))
    solver = DQNSolver(Box(-1, 1, (4,)), Discrete(2), gamma=0.99, clip_value=40, double_q=True, dueling=True,
                       learning_rate=1e-4, update_target_interval=200, device=dev)
    batch = [g["s0"], g["a"], g["r"], g["s1"], g["done"]]
    for k in range(3):
        td = solver.update(batch).numpy()
        np.testing.assert_allclose(td, g[f"upd{k}_abs_td"], rtol=1e-5, atol=1e-6)
    for k, v in solver.q_network.state_dict().items():
        np.testing.assert_allclose(v.cpu().numpy(), g[f"final/{k}"], rtol=1e-5, atol=1e-6)


def test_target_interval_and_weights_stream(dev):
    s = _make_solver(dev, 0, update_target_interval=2)
    batch = [np.random.rand(16, 4, 84, 84).astype(np.float32) * 255, np.random.randint(0, 6, 16),
             np.random.rand(16).astype(np.float32), np.random.rand(16, 4, 84, 84).astype(np.float32) * 255,
             np.zeros(16, np.float32)]
    s.update(batch)
    differs = any(not torch.equal(p, q) for p, q in zip(s.q_network.parameters(), s.target_q_network.parameters()))
    assert differs
    s.update(batch)  # interval 2 -> target synced
    assert all(torch.equal(p, q) for p, q in zip(s.q_network.parameters(), s.target_q_network.parameters()))
    buf = s.save_weights()
    s2 = _make_solver(dev, 1)
    s2.load_weights(io.BytesIO(buf.getvalue()))
    assert all(torch.equal(p, q) for p, q in zip(s.q_network.parameters(), s2.q_network.parameters()))
    assert all(torch.equal(p, q) for p, q in zip(s2.q_network.parameters(), s2.target_q_network.parameters()))


@pytest.mark.parametrize("hwc", [False, True])
def test_merged_heads_kernels_match_torch(dev, hwc):
    """rth_heads_merge / rth_heads_split_grad == the torch cat/permute construction of the
    merged dueling heads and its autograd, element for element"""
    from reth_amd.model import DQNNetwork

    torch.manual_seed(3)
    net = DQNNetwork((4, 84, 84), 6).to(dev)
    net.hwc_features = hwc
    ours = net._merged_head_weights()
    cpu = DQNNetwork((4, 84, 84), 6)
    cpu.load_state_dict({k: v.cpu() for k, v in net.state_dict().items()})
    cpu.hwc_features = hwc
    ref = cpu._merged_head_weights()  # the torch construction (CPU tensors)
    for a, b in zip(ours, ref):
        assert torch.equal(a.cpu(), b)
    g = [torch.randn(t.shape) for t in ref]
    torch.autograd.backward(ours, [x.to(dev) for x in g])
    torch.autograd.backward(ref, g)
    for (name, p), q in zip(net.named_parameters(), cpu.parameters()):
        if name.startswith("fc_"):
            assert torch.equal(p.grad.cpu(), q.grad), name


def test_heads_merge_split_kernels_nhwc_permutation(dev):
    """rth_heads_merge / rth_heads_split_grad with a C x P column permutation (C > 0: one LDS
    row transpose per FC1 row) against the torch construction, and split(merge) == identity"""
    from reth_amd import _lib
    from reth_amd.model import DQNNetwork

    torch.manual_seed(11)
    net = DQNNetwork((4, 84, 84), 6).to(dev)
    ps = [p.detach() for p in net._head_params()]
    H, F, A = ps[0].shape[0], ps[0].shape[1], ps[4].shape[0]
    o = dict(device=dev)
    w1, b1, w2, b2 = torch.empty(2 * H, F, **o), torch.empty(2 * H, **o), torch.empty(A + 1, 2 * H, **o), \
        torch.empty(A + 1, **o)
    arr = (_lib.c_vp * 8)(*[p.data_ptr() for p in ps])
    _lib.call("rth_heads_merge", arr, H, F, A, 64, 49, w1.data_ptr(), b1.data_ptr(), w2.data_ptr(), b2.data_ptr(),
              _lib.stream_ptr())
    hwc = lambda wt: wt.view(wt.shape[0], 64, 7, 7).permute(0, 2, 3, 1).reshape(wt.shape[0], -1)
    assert torch.equal(w1, torch.cat([hwc(ps[0]), hwc(ps[1])])) and torch.equal(b1, torch.cat([ps[2], ps[3]]))
    grads = [torch.empty_like(p) for p in ps]
    arr = (_lib.c_vp * 8)(*[g.data_ptr() for g in grads])
    _lib.call("rth_heads_split_grad", w1.data_ptr(), b1.data_ptr(), w2.data_ptr(), b2.data_ptr(), H, F, A, 64, 49,
              arr, _lib.stream_ptr())
    assert all(torch.equal(g, p) for g, p in zip(grads, ps))  # the inverse permutation


def test_tied_heads_storage(dev):
    """the two FC1 branches are row slices of one storage (model._tie_heads) on every device
    and after .to(memory_format=...); state_dict / load_state_dict / parameters() keep the
    reference's eight tensors; the no-grad merged FC1 IS that storage"""
    from reth_amd.model import DQNNetwork

    torch.manual_seed(2)
    cpu = DQNNetwork((4, 84, 84), 6)
    ref = {k: v.clone() for k, v in cpu.state_dict().items()}
    net = DQNNetwork((4, 84, 84), 6)
    net.load_state_dict(ref)
    net = net.to(dev, memory_format=torch.channels_last)
    a0, v0 = net.fc_adv[0], net.fc_value[0]
    for m in (cpu, net):
        w, b = m._w1s, m._b1s
        H = m.fc_adv[0].weight.shape[0]
        assert m.fc_adv[0].weight.data_ptr() == w.data_ptr()
        assert m.fc_value[0].weight.data_ptr() == w.data_ptr() + H * w.shape[1] * 4
        assert m.fc_adv[0].bias.data_ptr() == b.data_ptr() and m.fc_value[0].bias.data_ptr() == b.data_ptr() + H * 4
    assert list(net.state_dict()) == list(ref) and len(list(net.parameters())) == 14
    assert all(torch.equal(v.cpu(), ref[k]) for k, v in net.state_dict().items())
    with torch.no_grad():
        w1, b1, w2, b2 = net._merged_head_weights()
        assert w1.data_ptr() == net._w1s.data_ptr() and b1.data_ptr() == net._b1s.data_ptr()
        assert w2 is None and b2 is None  # the second layer is read from its parameters in place
    sd = {k: v + 1.0 for k, v in ref.items()}
    net.load_state_dict(sd)  # copies into the shared storage
    assert torch.equal(net._w1s[: a0.weight.shape[0]].cpu(), sd["fc_adv.0.weight"])
    assert torch.equal(net._w1s[a0.weight.shape[0]:].cpu(), sd["fc_value.0.weight"])
    assert torch.equal(v0.bias.cpu(), sd["fc_value.0.bias"])


def test_fc2_only_merge_split(dev):
    """RTH_HEADS_FC2_ONLY: the block-diagonal second layer built / split without FC1"""
    from reth_amd import _lib
    from reth_amd.model import DQNNetwork

    torch.manual_seed(4)
    net = DQNNetwork((4, 84, 84), 6).to(dev)
    ps = [p.detach() for p in net._head_params()]
    H, F, A = ps[0].shape[0], ps[0].shape[1], ps[4].shape[0]
    w2, b2 = torch.full((A + 1, 2 * H), 7.0, device=dev), torch.empty(A + 1, device=dev)
    arr = (_lib.c_vp * 8)(*[None] * 4, *[p.data_ptr() for p in ps[4:]])
    _lib.call("rth_heads_merge", arr, H, F, A, _lib.HEADS_FC2_ONLY, 1, None, None, w2.data_ptr(), b2.data_ptr(),
              _lib.stream_ptr())
    want = torch.zeros(A + 1, 2 * H, device=dev)
    want[:A, :H], want[A:, H:] = ps[4], ps[5]
    assert torch.equal(w2, want) and torch.equal(b2, torch.cat([ps[6], ps[7]]))
    gw2, gb2 = torch.randn(A + 1, 2 * H, device=dev), torch.randn(A + 1, device=dev)
    grads = [torch.empty_like(p) for p in ps[4:]]
    arr = (_lib.c_vp * 8)(*[None] * 4, *[g.data_ptr() for g in grads])
    _lib.call("rth_heads_split_grad", None, None, gw2.data_ptr(), gb2.data_ptr(), H, F, A, _lib.HEADS_FC2_ONLY, 1,
              arr, _lib.stream_ptr())
    assert torch.equal(grads[0], gw2[:A, :H]) and torch.equal(grads[1], gw2[A:, H:])
    assert torch.equal(grads[2], gb2[:A]) and torch.equal(grads[3], gb2[A:])


@pytest.mark.parametrize("n", [1, 37, 512])
def test_relu_bias_grad_nchw(dev, n):
    """rth_relu_bias_grad_nchw: the mask bit for bit, gy written channels-last, bias sums
    deterministic and within fp32 summation error; a deferred job (rows = n * P) finishes the
    same slabs"""
    from reth_amd import _lib

    gen = torch.Generator(device=dev).manual_seed(n)
    C, P = 64, 49
    y = torch.relu(torch.randn(n, C, 7, 7, device=dev, generator=gen))
    g = torch.randn(n, C, 7, 7, device=dev, generator=gen)
    ws = torch.zeros(_lib.lib().rth_relu_bias_grad_workspace(C), dtype=torch.uint8, device=dev)
    gy = torch.empty(n, C, 7, 7, device=dev, memory_format=torch.channels_last)
    db = torch.empty(C, device=dev)
    _lib.call("rth_relu_bias_grad_nchw", g.data_ptr(), y.data_ptr(), gy.data_ptr(), db.data_ptr(), ws.data_ptr(), n,
              C, P, _lib.stream_ptr())
    want = torch.ops.aten.threshold_backward(g, y, 0)
    assert gy.is_contiguous(memory_format=torch.channels_last) and torch.equal(gy, want)
    torch.testing.assert_close(db, want.sum((0, 2, 3)), rtol=1e-5, atol=1e-4)
    db2 = torch.empty(C, device=dev)
    _lib.call("rth_relu_bias_grad_nchw", g.data_ptr(), y.data_ptr(), gy.data_ptr(), db2.data_ptr(), ws.data_ptr(), n,
              C, P, _lib.stream_ptr())
    assert torch.equal(db, db2)
