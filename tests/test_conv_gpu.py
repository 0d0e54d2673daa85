"""rth_conv_bias_relu (conv.hip) against a float64 CPU convolution: the three Nature-DQN
torso geometries (dqn_model.py:14-20) on channels-last fp32 input, conv1 on uint8 CHW
stacks addressed through a row index, ragged tails and the unsupported-shape error."""
import os

import numpy as np
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

GEOMS = [(4, 84, 84, 32, 8, 4), (32, 20, 20, 64, 4, 2), (64, 9, 9, 64, 3, 1)]


def _shape(inp, cin, h, w, cout, k, s):
    from reth_amd import _lib

    return _lib.ConvShape(inp, cin, h, w, cout, k, k, s)


def _run(shape, x, rows, n, w, b, dev):
    from reth_amd import _lib

    ho = (shape.hin - shape.kh) // shape.stride + 1
    wo = (shape.win - shape.kw) // shape.stride + 1
    y = torch.full((n, ho, wo, shape.cout), float("nan"), device=dev)
    wt = w.to(dev).contiguous(memory_format=torch.channels_last)
    pk = torch.full((_lib.lib().rth_conv_packed_bytes(_lib.ctypes.byref(shape)) // 4,), float("nan"), device=dev)
    _lib.call("rth_conv_pack", _lib.ctypes.byref(shape), wt.data_ptr(), pk.data_ptr(), _lib.stream_ptr())
    assert not torch.isnan(pk).any()  # every fragment slot written
    _lib.call("rth_conv_bias_relu", _lib.ctypes.byref(shape), x.data_ptr(), None if rows is None else rows.data_ptr(),
              n, pk.data_ptr(), b.to(dev).data_ptr(), y.data_ptr(), _lib.stream_ptr())
    return y.permute(0, 3, 1, 2).cpu()


def _ref(x_nchw, w, b, s):
    return F.relu(F.conv2d(x_nchw.double(), w.double(), b.double(), stride=s))


@pytest.mark.parametrize("geom", GEOMS)
@pytest.mark.parametrize("n", [1, 3, 37])
def test_conv_f32_nhwc(dev, geom, n):
    from reth_amd import _lib

    cin, h, wd, cout, k, s = geom
    g = torch.Generator().manual_seed(hash((geom, n)) % 2**31)
    x = torch.rand((n, cin, h, wd), generator=g) * 2 - 1
    w = (torch.rand((cout, cin, k, k), generator=g) * 2 - 1) / np.sqrt(cin * k * k)
    b = (torch.rand(cout, generator=g) * 2 - 1) * 0.1
    xd = x.to(dev).contiguous(memory_format=torch.channels_last)
    got = _run(_shape(_lib.CONV_F32_NHWC, *geom), xd, None, n, w, b, dev)
    want = _ref(x, w, b, s)
    assert not torch.isnan(got).any()
    torch.testing.assert_close(got.double(), want, rtol=1e-5, atol=1e-5)
    assert (got == 0).any() and (got > 0).any()  # ReLU active on both sides


# the learner / target / actor batch sizes, and sizes whose tiles (16 output pixels) leave a
# short partial last round on 256 CUs (several tiles per wave, the last round ragged)
@pytest.mark.parametrize("gi,n", [(0, 41), (0, 72), (1, 204), (1, 1024), (2, 340), (2, 1024), (2, 512), (1, 513),
                                  (1, 768), (1, 769), (2, 1023), (2, 1025), (2, 259)])
def test_conv_partial_rounds(dev, gi, n):
    from reth_amd import _lib

    geom = GEOMS[gi]
    cin, h, wd, cout, k, s = geom
    g = torch.Generator().manual_seed(1000 * gi + n)
    x = torch.rand((n, cin, h, wd), generator=g) * 2 - 1
    w = (torch.rand((cout, cin, k, k), generator=g) * 2 - 1) / np.sqrt(cin * k * k)
    b = (torch.rand(cout, generator=g) * 2 - 1) * 0.1
    xd = x.to(dev).contiguous(memory_format=torch.channels_last)
    got = _run(_shape(_lib.CONV_F32_NHWC, *geom), xd, None, n, w, b, dev)
    assert not torch.isnan(got).any()  # every output written
    torch.testing.assert_close(got.double(), _ref(x, w, b, s), rtol=1e-5, atol=1e-5)
    if gi == 0:  # the uint8 form of conv1
        st = torch.randint(0, 256, (n, 4, 84, 84), dtype=torch.uint8, generator=g)
        got = _run(_shape(_lib.CONV_U8_CHW, *geom), st.to(dev), None, n, w, b, dev)
        torch.testing.assert_close(got.double(), _ref(st.double(), w, b, 4), rtol=1e-5, atol=5e-4)


@pytest.mark.parametrize("n", [1, 5, 64])
def test_conv1_u8_rows(dev, n):
    from reth_amd import _lib

    g = torch.Generator().manual_seed(7 + n)
    stacks = torch.randint(0, 256, (80, 4, 84, 84), dtype=torch.uint8, generator=g)
    rows = torch.randint(0, 80, (n,), generator=g)
    rows[0] = 79
    w = (torch.rand((32, 4, 8, 8), generator=g) * 2 - 1) / 16
    b = (torch.rand(32, generator=g) * 2 - 1) * 0.1
    shape = _shape(_lib.CONV_U8_CHW, *GEOMS[0])
    got = _run(shape, stacks.to(dev), rows.to(dev), n, w, b, dev)
    want = _ref(stacks[rows].double(), w, b, 4)
    torch.testing.assert_close(got.double(), want, rtol=1e-5, atol=5e-4)  # |x| <= 255: sums ~ 1e2
    # without a row index: stacks 0..n-1; the f32 NHWC form of the same data agrees
    got2 = _run(shape, stacks.to(dev), None, n, w, b, dev)
    torch.testing.assert_close(got2.double(), _ref(stacks[:n].double(), w, b, 4), rtol=1e-5, atol=5e-4)
    xf = stacks[:n].float().to(dev).contiguous(memory_format=torch.channels_last)
    got3 = _run(_shape(_lib.CONV_F32_NHWC, *GEOMS[0]), xf, None, n, w, b, dev)
    torch.testing.assert_close(got3, got2, rtol=1e-5, atol=5e-4)


def test_conv_empty_and_unsupported(dev):
    from reth_amd import _lib

    shape = _shape(_lib.CONV_F32_NHWC, *GEOMS[1])
    assert _lib.lib().rth_conv_supported(_lib.ctypes.byref(shape)) == 1
    x = torch.zeros(16, device=dev)
    y = torch.zeros(16, device=dev)
    w = torch.zeros(64 * 32 * 16, device=dev)
    _lib.call("rth_conv_bias_relu", _lib.ctypes.byref(shape), x.data_ptr(), None, 0, w.data_ptr(), w.data_ptr(),
              y.data_ptr(), _lib.stream_ptr())
    bad = _shape(_lib.CONV_F32_NHWC, 3, 84, 84, 32, 8, 4)
    assert _lib.lib().rth_conv_supported(_lib.ctypes.byref(bad)) == 0
    assert _lib.lib().rth_conv_packed_bytes(_lib.ctypes.byref(bad)) == 0
    # conv2's packed weights: one fp32 copy (the fp32-MFMA kernel)
    assert _lib.lib().rth_conv_packed_bytes(_lib.ctypes.byref(shape)) == 64 * 32 * 16 * 4
    with pytest.raises(_lib.RethHipError, match="not built"):
        _lib.call("rth_conv_bias_relu", _lib.ctypes.byref(bad), x.data_ptr(), None, 1, w.data_ptr(), w.data_ptr(),
                  y.data_ptr(), _lib.stream_ptr())


def _torso_net(dev, seed=0):
    from reth_amd.model import DQNNetwork

    torch.manual_seed(seed)
    net = DQNNetwork((4, 84, 84), 6).to(dev, memory_format=torch.channels_last)
    net.hwc_features = True
    return net


def test_frozen_packed_weights_follow_refresh(dev):
    """a frozen copy's packed conv weights are rebuilt by freeze_heads (target sync / actor
    reload) and used by default; stale until then (the conv biases and the heads -- FC1's
    tied storage, FC2's parameters -- are read live)"""
    net = _torso_net(dev, seed=2)
    x = torch.randint(0, 256, (8, 4, 84, 84), dtype=torch.uint8, device=dev)
    with torch.no_grad():
        net.freeze_heads()
        q0 = net.forward_heads(x)
        for name, p in net.named_parameters():
            if name.startswith("features") and name.endswith("weight"):  # the convs
                p.mul_(1.01)
        q_stale = net.forward_heads(x)
        net.freeze_heads()
        q1 = net.forward_heads(x)
        q_fresh = net.forward_heads(x, net._merged_head_weights(), packed=net.pack_convs())
        net.fc_adv[0].weight.mul_(1.01)  # FC1: live
        net.fc_value[2].weight.mul_(1.01)  # FC2: live
        q_fc1 = net.forward_heads(x)
        q_fc1_fresh = net.forward_heads(x, net._merged_head_weights(), packed=net.pack_convs())
    assert torch.equal(q0, q_stale)
    assert not torch.equal(q0, q1)
    torch.testing.assert_close(q1, q_fresh, rtol=0, atol=0)
    assert not torch.equal(q_fc1, q1) and torch.equal(q_fc1, q_fc1_fresh)


def test_forward_heads_u8_rows_matches_miopen(dev):
    """the HIP torso on uint8 stacks through a row index == MIOpen on the gathered f32 batch"""
    net = _torso_net(dev)
    g = torch.Generator(device=dev).manual_seed(3)
    frames = torch.randint(0, 256, (40, 4, 84, 84), dtype=torch.uint8, device=dev, generator=g)
    rows = torch.randint(0, 40, (33,), device=dev, generator=g)
    with torch.no_grad():
        q = net.forward_heads(frames, rows=rows)
        net.hip_conv = False
        want = net.forward_heads(frames[rows].float().contiguous(memory_format=torch.channels_last))
        net.hip_conv = True
        q_gathered = net.forward_heads(frames[rows].contiguous())
        q_all = net.forward_heads(frames)
    torch.testing.assert_close(q, want, rtol=1e-5, atol=1e-4)
    # the row index only changes where the torso reads: same kernels, same shapes, same bits
    torch.testing.assert_close(q_gathered, q, rtol=0, atol=0)
    # the 40-row batch runs FC1 at another M, where the library GEMM may pick another
    # solution (another summation order), so only close
    torch.testing.assert_close(q_all[rows], q, rtol=1e-5, atol=1e-5)


def test_hip_torso_gradients_match_miopen(dev):
    """grad path: rth_conv_bias_relu forward + MIOpen backward == MIOpen forward + backward"""
    net = _torso_net(dev, seed=1)
    g = torch.Generator(device=dev).manual_seed(4)
    x = torch.randint(0, 256, (24, 4, 84, 84), device=dev, generator=g).float()
    x = x.contiguous(memory_format=torch.channels_last)
    grads = []
    for hip in (True, False):
        net.hip_conv = hip
        net.zero_grad(set_to_none=True)
        h = net.forward_heads(x, net._merged_head_weights())
        (h.square().sum() * 1e-3).backward()
        grads.append([p.grad.clone() for p in net.parameters()])
    for a, b in zip(*grads):
        scale = b.abs().max().clamp_min(1e-12)
        assert ((a - b).abs().max() / scale) < 1e-4


def test_pack_many_matches_single_packs(dev):
    from reth_amd import _lib

    shapes = [_shape(_lib.CONV_F32_NHWC, *GEOMS[0]), _shape(_lib.CONV_F32_NHWC, *GEOMS[1]),
              _shape(_lib.CONV_F32_NHWC, *GEOMS[2]), _shape(_lib.CONV_U8_CHW, *GEOMS[0])]
    ws, singles, many = [], [], []
    for shp in shapes:
        cin, cout, k = shp.cin, shp.cout, shp.kh
        w = torch.randn((cout, cin, k, k), device=dev).contiguous(memory_format=torch.channels_last)
        nb = _lib.lib().rth_conv_packed_bytes(_lib.ctypes.byref(shp)) // 4
        a, b = torch.zeros(nb, device=dev), torch.zeros(nb, device=dev)
        _lib.call("rth_conv_pack", _lib.ctypes.byref(shp), w.data_ptr(), a.data_ptr(), _lib.stream_ptr())
        ws.append(w), singles.append(a), many.append(b)
    n = len(shapes)
    _lib.call("rth_conv_pack_many", n, (_lib.ConvShape * n)(*shapes), (_lib.c_vp * n)(*[w.data_ptr() for w in ws]),
              (_lib.c_vp * n)(*[b.data_ptr() for b in many]), _lib.stream_ptr())
    for a, b in zip(singles, many):
        assert torch.equal(a, b)


@pytest.mark.parametrize("n", [1, 7, 40, 512, 1024])
def test_conv1_relu_wgrad_u8(dev, n):
    """rth_conv_relu_wgrad against a float64 CPU autograd of relu(conv2d(x, w) + b); n = 512
    is the learner's batch (the bench's launch: split partials over every workgroup + the
    reduce), 1024 the [s0; s1] size"""
    from reth_amd import _lib

    g = torch.Generator().manual_seed(100 + n)
    stacks = torch.randint(0, 256, (60, 4, 84, 84), dtype=torch.uint8, generator=g)
    rows = torch.randint(0, 60, (n,), generator=g)
    w = ((torch.rand((32, 4, 8, 8), generator=g) * 2 - 1) / 16).double().requires_grad_(True)
    b = ((torch.rand(32, generator=g) * 2 - 1) * 0.5).double().requires_grad_(True)
    x = stacks[rows].double()
    y = F.relu(F.conv2d(x, w, b, stride=4))
    up = torch.randn(y.shape, generator=g, dtype=torch.float64)
    (y * up).sum().backward()
    shape = _shape(_lib.CONV_U8_CHW, *GEOMS[0])
    yd = y.detach().float().permute(0, 2, 3, 1).contiguous().to(dev)   # NHWC
    gd = up.float().permute(0, 2, 3, 1).contiguous().to(dev)
    gw = torch.full((32, 8, 8, 4), float("nan"), device=dev)           # OHWI
    gb = torch.full((32,), float("nan"), device=dev)
    ws = torch.empty(_lib.lib().rth_conv_wgrad_workspace(_lib.ctypes.byref(shape)) // 4, device=dev)
    _lib.call("rth_conv_relu_wgrad", _lib.ctypes.byref(shape), stacks.to(dev).data_ptr(), rows.to(dev).data_ptr(), n,
              gd.data_ptr(), yd.data_ptr(), gw.data_ptr(), gb.data_ptr(), ws.data_ptr(), _lib.stream_ptr())
    want_w = w.grad.permute(0, 2, 3, 1)
    scale = want_w.abs().max()
    assert ((gw.cpu().double() - want_w).abs().max() / scale) < 2e-6
    torch.testing.assert_close(gb.cpu().double(), b.grad, rtol=1e-5, atol=1e-4)
    # deterministic: a second call gives the same bits
    gw2 = torch.empty_like(gw)
    _lib.call("rth_conv_relu_wgrad", _lib.ctypes.byref(shape), stacks.to(dev).data_ptr(), rows.to(dev).data_ptr(), n,
              gd.data_ptr(), yd.data_ptr(), gw2.data_ptr(), gb.data_ptr(), ws.data_ptr(), _lib.stream_ptr())
    assert torch.equal(gw, gw2)


def test_hip_torso_gradients_u8_input(dev):
    """grad path on uint8 stacks (forward + rth_conv_relu_wgrad for conv1) == MIOpen on the
    float32 batch"""
    net = _torso_net(dev, seed=3)
    g = torch.Generator(device=dev).manual_seed(5)
    xu = torch.randint(0, 256, (24, 4, 84, 84), dtype=torch.uint8, device=dev, generator=g)
    grads = []
    for hip in (True, False):
        net.hip_conv = hip
        net.zero_grad(set_to_none=True)
        x = xu if hip else xu.float().contiguous(memory_format=torch.channels_last)
        h = net.forward_heads(x, net._merged_head_weights())
        (h.square().sum() * 1e-3).backward()
        grads.append([p.grad.clone() for p in net.parameters()])
    for a, b in zip(*grads):
        scale = b.abs().max().clamp_min(1e-12)
        assert ((a - b).abs().max() / scale) < 1e-4


@pytest.mark.parametrize("count", [0, 5, 37, 64])
def test_conv_upto_device_count(dev, count):
    """rth_conv_bias_relu_upto computes the first *n_dev samples exactly as the plain launch
    and leaves the rest of the output untouched"""
    from reth_amd import _lib

    n = 64
    g = torch.Generator().manual_seed(31 + count)
    stacks = torch.randint(0, 256, (n, 4, 84, 84), dtype=torch.uint8, generator=g).to(dev)
    rows = torch.randperm(n, generator=g).to(dev)
    w = ((torch.rand((32, 4, 8, 8), generator=g) * 2 - 1) / 16).to(dev).contiguous(memory_format=torch.channels_last)
    b = ((torch.rand(32, generator=g) * 2 - 1) * 0.1).to(dev)
    shape = _shape(_lib.CONV_U8_CHW, *GEOMS[0])
    pk = torch.empty(_lib.lib().rth_conv_packed_bytes(_lib.ctypes.byref(shape)) // 4, device=dev)
    _lib.call("rth_conv_pack", _lib.ctypes.byref(shape), w.data_ptr(), pk.data_ptr(), _lib.stream_ptr())
    full = torch.empty((n, 20, 20, 32), device=dev)
    _lib.call("rth_conv_bias_relu", _lib.ctypes.byref(shape), stacks.data_ptr(), rows.data_ptr(), n, pk.data_ptr(),
              b.data_ptr(), full.data_ptr(), _lib.stream_ptr())
    part = torch.full((n, 20, 20, 32), float("nan"), device=dev)
    cnt = torch.tensor([count], dtype=torch.int64, device=dev)
    _lib.call("rth_conv_bias_relu_upto", _lib.ctypes.byref(shape), stacks.data_ptr(), rows.data_ptr(), n,
              cnt.data_ptr(), pk.data_ptr(), b.data_ptr(), part.data_ptr(), _lib.stream_ptr())
    assert torch.equal(part[:count], full[:count])
    assert bool(torch.isnan(part[count:]).all())


@pytest.mark.parametrize("gi", [1, 2])
@pytest.mark.parametrize("n", [1, 3, 37, 512])
def test_conv_dgrad(dev, gi, n):
    """rth_conv_dgrad (per stride-parity class implicit GEMM) against the float64 CPU data
    gradient of conv2d; every element of gx written (no fill: NaN-initialised output)"""
    from reth_amd import _lib

    cin, h, wd, cout, k, s = GEOMS[gi]
    shape = _shape(_lib.CONV_F32_NHWC, *GEOMS[gi])
    assert _lib.lib().rth_conv_dgrad_supported(_lib.ctypes.byref(shape)) == 1
    g = torch.Generator().manual_seed(31 * gi + n)
    ho, wo = (h - k) // s + 1, (wd - k) // s + 1
    gy = torch.rand((n, cout, ho, wo), generator=g) * 2 - 1
    gy[gy < -0.3] = 0  # ReLU-masked, like the learner's
    w = (torch.rand((cout, cin, k, k), generator=g) * 2 - 1) / np.sqrt(cin * k * k)
    gyd = gy.to(dev).contiguous(memory_format=torch.channels_last)
    wd_ = w.to(dev).contiguous(memory_format=torch.channels_last)
    gx = torch.full((n, cin, h, wd), float("nan"), device=dev).contiguous(memory_format=torch.channels_last)
    _lib.call("rth_conv_dgrad", _lib.ctypes.byref(shape), gyd.data_ptr(), n, wd_.data_ptr(), gx.data_ptr(),
              _lib.stream_ptr())
    want = torch.nn.grad.conv2d_input((n, cin, h, wd), w.double(), gy.double(), stride=s)
    got = gx.cpu()
    assert not torch.isnan(got).any()
    torch.testing.assert_close(got.double(), want, rtol=1e-5, atol=1e-5)
    # the exact-split bf16 MFMA (k_conv_x9: every product exact, fp32 sums): within a few fp32
    # roundings of the 256- / 576-term sums
    err = (got.double() - want).abs().max().item()
    assert err <= 2e-6 * max(1.0, want.abs().max().item()), err


@pytest.mark.parametrize("gi", [1, 2])
def test_conv_dgrad_ws_two_streams(dev, gi):
    """rth_conv_dgrad_ws: two data gradients with different weights, each with its own
    workspace, issued on two streams repeatedly -- each bit-identical to its single-stream
    result (the internal per-device workspace of rth_conv_dgrad would be shared by them)"""
    from reth_amd import _lib

    cin, h, wd, cout, k, s = GEOMS[gi]
    shape = _shape(_lib.CONV_F32_NHWC, *GEOMS[gi])
    n, ho = 256, (h - k) // s + 1
    g = torch.Generator(device=dev).manual_seed(5 + gi)
    gys = [torch.randn((n, cout, ho, ho), device=dev, generator=g).contiguous(memory_format=torch.channels_last)
           for _ in range(2)]
    ws_ = [(torch.randn((cout, cin, k, k), device=dev, generator=g) * 0.05).contiguous(
        memory_format=torch.channels_last) for _ in range(2)]
    nbytes = _lib.lib().rth_conv_dgrad_workspace(_lib.ctypes.byref(shape))
    work = [torch.empty(max(nbytes, 16) // 4, device=dev) for _ in range(2)]
    want = []
    for j in range(2):
        gx = torch.empty((n, cin, h, wd), device=dev).contiguous(memory_format=torch.channels_last)
        _lib.call("rth_conv_dgrad_ws", _lib.ctypes.byref(shape), gys[j].data_ptr(), n, ws_[j].data_ptr(),
                  gx.data_ptr(), work[j].data_ptr(), _lib.stream_ptr())
        want.append(gx)
    torch.cuda.synchronize()
    streams = [torch.cuda.Stream(dev) for _ in range(2)]
    outs = [[torch.empty_like(want[j]) for _ in range(8)] for j in range(2)]
    for it in range(8):
        for j in range(2):
            with torch.cuda.stream(streams[j]):
                _lib.call("rth_conv_dgrad_ws", _lib.ctypes.byref(shape), gys[j].data_ptr(), n, ws_[j].data_ptr(),
                          outs[j][it].data_ptr(), work[j].data_ptr(), _lib.stream_ptr())
    torch.cuda.synchronize()
    for j in range(2):
        for o in outs[j]:
            assert torch.equal(o, want[j])


@pytest.mark.parametrize("gi", [1, 2])
def test_conv_dgrad_prepacked(dev, gi):
    """rth_conv_dgrad_prepacked from a kernel packed by rth_conv_pack_many's CONV_PACK_DGRAD job
    (in the same launch as the forward packs, as the learner issues it): bit-identical to
    rth_conv_dgrad_ws (pack + convolution) on the same weights; the forward packs of the same
    launch equal rth_conv_pack's"""
    from reth_amd import _lib

    cin, h, wd, cout, k, s = GEOMS[gi]
    shape = _shape(_lib.CONV_F32_NHWC, *GEOMS[gi])
    nbytes = _lib.lib().rth_conv_dgrad_workspace(_lib.ctypes.byref(shape))
    assert nbytes > 0
    n, ho = 300, (h - k) // s + 1
    g = torch.Generator(device=dev).manual_seed(11 + gi)
    gy = torch.randn((n, cout, ho, ho), device=dev, generator=g).contiguous(memory_format=torch.channels_last)
    w = (torch.randn((cout, cin, k, k), device=dev, generator=g) * 0.05).contiguous(memory_format=torch.channels_last)
    work = torch.empty(nbytes // 4, device=dev)
    want = torch.empty((n, cin, h, wd), device=dev).contiguous(memory_format=torch.channels_last)
    _lib.call("rth_conv_dgrad_ws", _lib.ctypes.byref(shape), gy.data_ptr(), n, w.data_ptr(), want.data_ptr(),
              work.data_ptr(), _lib.stream_ptr())
    # one pack launch: the forward image and the data-gradient kernel of the same weights
    fwd_bytes = _lib.lib().rth_conv_packed_bytes(_lib.ctypes.byref(shape))
    fwd = torch.empty(fwd_bytes // 4, device=dev)
    fwd_want = torch.empty_like(fwd)
    _lib.call("rth_conv_pack", _lib.ctypes.byref(shape), w.data_ptr(), fwd_want.data_ptr(), _lib.stream_ptr())
    pk = torch.full((nbytes // 4,), float("nan"), device=dev)
    flagged = _lib.ConvShape(shape.input | _lib.CONV_PACK_DGRAD, shape.cin, shape.hin, shape.win, shape.cout,
                             shape.kh, shape.kw, shape.stride)
    shapes = (_lib.ConvShape * 2)(shape, flagged)
    ws = (_lib.c_vp * 2)(w.data_ptr(), w.data_ptr())
    pks = (_lib.c_vp * 2)(fwd.data_ptr(), pk.data_ptr())
    _lib.call("rth_conv_pack_many", 2, shapes, ws, pks, _lib.stream_ptr())
    got = torch.full_like(want, float("nan"))
    _lib.call("rth_conv_dgrad_prepacked", _lib.ctypes.byref(shape), gy.data_ptr(), n, pk.data_ptr(), got.data_ptr(),
              _lib.stream_ptr())
    torch.cuda.synchronize()
    assert torch.equal(pk, work)
    assert torch.equal(fwd, fwd_want)
    assert torch.equal(got, want)


@pytest.mark.parametrize("n", [1, 5, 300, 512])
def test_conv_dgrad_relu_prepacked(dev, n):
    """conv3's data gradient with conv2's ReLU mask and bias slabs in its epilogue
    (rth_conv_dgrad_relu_prepacked, r05): the masked gradient bit-identical to
    rth_conv_dgrad_prepacked + rth_relu_bias_grad, and conv2's bias gradient -- the slabs finished
    by the deferred job of conv1's reduce launch -- within fp32 summation error of the fp64 sum,
    run-to-run bit-identical; refused for other geometries"""
    from reth_amd import _lib

    cin, h, wd, cout, k, s = GEOMS[2]
    shape = _shape(_lib.CONV_F32_NHWC, *GEOMS[2])
    assert _lib.lib().rth_conv_dgrad_relu_supported(_lib.ctypes.byref(shape))
    ho = (h - k) // s + 1
    g = torch.Generator(device=dev).manual_seed(500 + n)
    gy = torch.randn((n, cout, ho, ho), device=dev, generator=g).contiguous(memory_format=torch.channels_last)
    w = (torch.randn((cout, cin, k, k), device=dev, generator=g) * 0.05).contiguous(memory_format=torch.channels_last)
    y2 = torch.randn((n, cin, h, wd), device=dev, generator=g).contiguous(memory_format=torch.channels_last)
    work = torch.empty(_lib.lib().rth_conv_dgrad_workspace(_lib.ctypes.byref(shape)) // 4, device=dev)
    plain = torch.empty((n, cin, h, wd), device=dev).contiguous(memory_format=torch.channels_last)
    _lib.call("rth_conv_dgrad_ws", _lib.ctypes.byref(shape), gy.data_ptr(), n, w.data_ptr(), plain.data_ptr(),
              work.data_ptr(), _lib.stream_ptr())  # packs the flipped kernel into work, as the learner's pack launch
    rows = n * h * wd
    want = torch.empty_like(plain)
    ws_ref = torch.empty(_lib.lib().rth_relu_bias_grad_workspace(cin), dtype=torch.uint8, device=dev)
    db_ref = torch.empty(cin, device=dev)
    _lib.call("rth_relu_bias_grad", plain.data_ptr(), y2.data_ptr(), want.data_ptr(), db_ref.data_ptr(),
              ws_ref.data_ptr(), rows, cin, _lib.stream_ptr())
    # conv1's reduce launch finishes the deferred job (a small conv1 problem beside it)
    c1 = _shape(_lib.CONV_U8_CHW, *GEOMS[0])
    st = torch.randint(0, 256, (3, 4, 84, 84), dtype=torch.uint8, device=dev, generator=g)
    gc = torch.randn((3, 20, 20, 32), device=dev, generator=g)
    yc = torch.randn((3, 20, 20, 32), device=dev, generator=g)
    wsc = torch.empty(_lib.lib().rth_conv_wgrad_workspace(_lib.ctypes.byref(c1)), dtype=torch.uint8, device=dev)
    dbs = []
    for _ in range(2):
        got = torch.full_like(plain, float("nan"))
        ws = torch.empty(_lib.lib().rth_relu_bias_grad_workspace(cin), dtype=torch.uint8, device=dev)
        slabs = _lib.ctypes.c_int64(-1)
        _lib.call("rth_conv_dgrad_relu_prepacked", _lib.ctypes.byref(shape), gy.data_ptr(), n, work.data_ptr(),
                  y2.data_ptr(), got.data_ptr(), ws.data_ptr(), _lib.ctypes.byref(slabs), _lib.stream_ptr())
        assert 1 <= slabs.value <= n
        db = torch.full((cin,), float("nan"), device=dev)
        jobs = (_lib.BiasDeferred * 1)(_lib.BiasDeferred(ws.data_ptr(), db.data_ptr(), rows, cin, slabs.value))
        gw, gb = torch.empty((32, 8, 8, 4), device=dev), torch.empty(32, device=dev)
        _lib.call("rth_conv_relu_wgrad_ex", _lib.ctypes.byref(c1), st.data_ptr(), None, 3, gc.data_ptr(),
                  yc.data_ptr(), gw.data_ptr(), gb.data_ptr(), wsc.data_ptr(), jobs, 1, None, 0, _lib.stream_ptr())
        torch.cuda.synchronize()
        assert torch.equal(got, want)
        dbs.append(db.clone())
    assert torch.equal(dbs[0], dbs[1])
    m = want.permute(0, 2, 3, 1).reshape(-1, cin).double().cpu()
    exact, scale = m.sum(0), m.abs().sum(0)
    assert ((dbs[0].double().cpu() - exact).abs() <= 1e-6 * scale + 1e-12).all()
    assert ((db_ref.double().cpu() - exact).abs() <= 1e-6 * scale + 1e-12).all()
    conv2 = _shape(_lib.CONV_F32_NHWC, *GEOMS[1])
    assert _lib.lib().rth_conv_dgrad_relu_supported(_lib.ctypes.byref(conv2)) == 0
    with pytest.raises(_lib.RethHipError, match="only conv3"):
        _lib.call("rth_conv_dgrad_relu_prepacked", _lib.ctypes.byref(conv2), gy.data_ptr(), n, work.data_ptr(),
                  y2.data_ptr(), got.data_ptr(), ws.data_ptr(), _lib.ctypes.byref(slabs), _lib.stream_ptr())


def test_conv_dgrad_unsupported(dev):
    from reth_amd import _lib

    conv1 = _shape(_lib.CONV_F32_NHWC, *GEOMS[0])
    assert _lib.lib().rth_conv_dgrad_supported(_lib.ctypes.byref(conv1)) == 0
    t = torch.zeros(16, device=dev)
    with pytest.raises(_lib.RethHipError, match="not built"):
        _lib.call("rth_conv_dgrad", _lib.ctypes.byref(conv1), t.data_ptr(), 1, t.data_ptr(), t.data_ptr(),
                  _lib.stream_ptr())


def test_deferred_bias_grads_finished_by_conv1_reduce(dev):
    """rth_relu_bias_grad with db = NULL leaves its slabs; rth_conv_relu_wgrad_ex finishes
    them in conv1's reduce launch: bit-identical bias gradients to the two-launch form (the
    same 1024-lane summation order), conv1's own gradients unchanged"""
    from reth_amd import _lib

    g = torch.Generator(device=dev).manual_seed(11)
    jobs, want, outs, keep = [], [], [], []
    for rows, C in [(512 * 49, 64), (512 * 81, 64), (37, 64)]:
        gg = torch.randn((rows, C), device=dev, generator=g)
        yy = torch.randn((rows, C), device=dev, generator=g)
        ws = torch.empty(_lib.lib().rth_relu_bias_grad_workspace(C), dtype=torch.uint8, device=dev)
        gy, db = torch.empty_like(gg), torch.empty(C, device=dev)
        _lib.call("rth_relu_bias_grad", gg.data_ptr(), yy.data_ptr(), gy.data_ptr(), db.data_ptr(), ws.data_ptr(),
                  rows, C, _lib.stream_ptr())
        want.append(db.clone())
        gy2, db2 = torch.empty_like(gg), torch.full((C,), float("nan"), device=dev)
        _lib.call("rth_relu_bias_grad", gg.data_ptr(), yy.data_ptr(), gy2.data_ptr(), None, ws.data_ptr(), rows, C,
                  _lib.stream_ptr())
        assert torch.equal(gy, gy2)
        jobs.append(_lib.BiasDeferred(ws.data_ptr(), db2.data_ptr(), rows, C))
        outs.append(db2)
        keep += [gg, yy, ws, gy, gy2]
    n = 5
    shape = _shape(_lib.CONV_U8_CHW, *GEOMS[0])
    st = torch.randint(0, 256, (n, 4, 84, 84), dtype=torch.uint8, device=dev, generator=g)
    gc = torch.randn((n, 20, 20, 32), device=dev, generator=g)
    yc = torch.randn((n, 20, 20, 32), device=dev, generator=g)
    wsc = torch.empty(_lib.lib().rth_conv_wgrad_workspace(_lib.ctypes.byref(shape)), dtype=torch.uint8, device=dev)
    res = []
    for deferred in (False, True):
        gw, gb = torch.empty((32, 8, 8, 4), device=dev), torch.empty(32, device=dev)
        arr = (_lib.BiasDeferred * len(jobs))(*jobs)
        _lib.call("rth_conv_relu_wgrad_ex", _lib.ctypes.byref(shape), st.data_ptr(), None, n, gc.data_ptr(),
                  yc.data_ptr(), gw.data_ptr(), gb.data_ptr(), wsc.data_ptr(), arr if deferred else None,
                  len(jobs) if deferred else 0, None, 0, _lib.stream_ptr())
        res.append((gw.clone(), gb.clone()))
    assert torch.equal(res[0][0], res[1][0]) and torch.equal(res[0][1], res[1][1])
    for got, ref in zip(outs, want):
        assert torch.equal(got, ref)


@pytest.mark.parametrize("n", [0, 1, 37, 512])
def test_deferred_wgrads_finished_by_conv1_reduce(dev, n):
    """r06: rth_conv_wgrad_f32_partials leaves conv2's and conv3's split partials;
    conv1's reduce launch (rth_conv_relu_wgrad_ex's wdeferred jobs) finishes them beside a
    deferred bias gradient: weight gradients bit-identical to rth_conv_wgrad_f32's (the same
    per-element split order), conv1's own gradients and the bias unchanged"""
    from reth_amd import _lib

    g = torch.Generator(device=dev).manual_seed(17 + n)
    want, jobs, outs, keep = [], [], [], []
    for gi in (1, 2):
        cin, h, wd, cout, k, s = GEOMS[gi]
        ho = (h - k) // s + 1
        x = torch.randn((n, cin, h, wd), device=dev, generator=g).contiguous(memory_format=torch.channels_last)
        gy = torch.randn((n, cout, ho, ho), device=dev, generator=g).contiguous(memory_format=torch.channels_last)
        shape = _shape(_lib.CONV_F32_NHWC, *GEOMS[gi])
        ws = torch.empty(_lib.lib().rth_conv_wgrad_f32_workspace(_lib.ctypes.byref(shape)) // 4, device=dev)
        gw = torch.full((cout, cin, k, k), float("nan"), device=dev).contiguous(memory_format=torch.channels_last)
        _lib.call("rth_conv_wgrad_f32", _lib.ctypes.byref(shape), x.data_ptr(), n, gy.data_ptr(), gw.data_ptr(),
                  ws.data_ptr(), _lib.stream_ptr())
        want.append(gw)
        gw2 = torch.full_like(gw, float("nan"))
        job = _lib.WgradDeferred()
        _lib.call("rth_conv_wgrad_f32_partials", _lib.ctypes.byref(shape), x.data_ptr(), n, gy.data_ptr(),
                  gw2.data_ptr(), ws.data_ptr(), _lib.ctypes.byref(job), _lib.stream_ptr())
        jobs.append(job)
        outs.append(gw2)
        keep += [x, gy, ws]
    rows, C = 3 * 81, 64
    gg, yy = torch.randn((rows, C), device=dev, generator=g), torch.randn((rows, C), device=dev, generator=g)
    wsb = torch.empty(_lib.lib().rth_relu_bias_grad_workspace(C), dtype=torch.uint8, device=dev)
    gyb, db = torch.empty_like(gg), torch.full((C,), float("nan"), device=dev)
    _lib.call("rth_relu_bias_grad", gg.data_ptr(), yy.data_ptr(), gyb.data_ptr(), None, wsb.data_ptr(), rows, C,
              _lib.stream_ptr())
    shape1 = _shape(_lib.CONV_U8_CHW, *GEOMS[0])
    m = max(n, 1)
    st = torch.randint(0, 256, (m, 4, 84, 84), dtype=torch.uint8, device=dev, generator=g)
    gc = torch.randn((m, 20, 20, 32), device=dev, generator=g)
    yc = torch.randn((m, 20, 20, 32), device=dev, generator=g)
    wsc = torch.empty(_lib.lib().rth_conv_wgrad_workspace(_lib.ctypes.byref(shape1)), dtype=torch.uint8, device=dev)
    res = []
    for deferred in (False, True):
        gw1, gb1 = torch.empty((32, 8, 8, 4), device=dev), torch.empty(32, device=dev)
        barr = (_lib.BiasDeferred * 1)(_lib.BiasDeferred(wsb.data_ptr(), db.data_ptr(), rows, C))
        warr = (_lib.WgradDeferred * 2)(*jobs)
        _lib.call("rth_conv_relu_wgrad_ex", _lib.ctypes.byref(shape1), st.data_ptr(), None, m, gc.data_ptr(),
                  yc.data_ptr(), gw1.data_ptr(), gb1.data_ptr(), wsc.data_ptr(), barr, 1, warr if deferred else None,
                  2 if deferred else 0, _lib.stream_ptr())
        res.append((gw1.clone(), gb1.clone(), db.clone()))
    assert all(torch.equal(a, b) for a, b in zip(res[0], res[1]))
    for got, ref in zip(outs, want):
        assert not torch.isnan(got).any()
        assert torch.equal(got, ref)
        if n == 0:
            assert not got.any()


@pytest.mark.parametrize("gi,n", [(1, 3), (2, 1), (2, 37), (2, 1024)])
def test_conv_nchw_output(dev, gi, n):
    """RTH_CONV_OUT_NCHW: the same values as the NHWC output, written [n, cout, hout, wout]
    (the last conv feeding FC1 in the (C, H, W) flatten order); refused for the uint8 conv1"""
    from reth_amd import _lib

    geom = GEOMS[gi]
    cin, h, wd, cout, k, s = geom
    g = torch.Generator().manual_seed(77 + n)
    x = (torch.rand((n, cin, h, wd), generator=g) * 2 - 1).to(dev).contiguous(memory_format=torch.channels_last)
    w = ((torch.rand((cout, cin, k, k), generator=g) * 2 - 1) / np.sqrt(cin * k * k)).to(dev)
    b = ((torch.rand(cout, generator=g) * 2 - 1) * 0.1).to(dev)
    shape = _shape(_lib.CONV_F32_NHWC, *geom)
    flagged = _shape(_lib.CONV_F32_NHWC | _lib.CONV_OUT_NCHW, *geom)
    assert _lib.lib().rth_conv_supported(_lib.ctypes.byref(flagged)) == 1
    wt = w.contiguous(memory_format=torch.channels_last)
    pk = torch.empty(_lib.lib().rth_conv_packed_bytes(_lib.ctypes.byref(shape)) // 4, device=dev)
    _lib.call("rth_conv_pack", _lib.ctypes.byref(shape), wt.data_ptr(), pk.data_ptr(), _lib.stream_ptr())
    ho = (h - k) // s + 1
    y_hwc = torch.empty((n, cout, ho, ho), device=dev, memory_format=torch.channels_last)
    y_chw = torch.full((n, cout, ho, ho), float("nan"), device=dev)
    for shp, y in ((shape, y_hwc), (flagged, y_chw)):
        _lib.call("rth_conv_bias_relu", _lib.ctypes.byref(shp), x.data_ptr(), None, n, pk.data_ptr(), b.data_ptr(),
                  y.data_ptr(), _lib.stream_ptr())
    assert y_chw.is_contiguous() and torch.equal(y_chw, y_hwc)
    u8 = _shape(_lib.CONV_U8_CHW | _lib.CONV_OUT_NCHW, *GEOMS[0])
    assert _lib.lib().rth_conv_supported(_lib.ctypes.byref(u8)) == 0


@pytest.mark.parametrize("kind", ["f32", "x9"])
@pytest.mark.parametrize("gi,n", [(1, 1), (1, 37), (1, 512), (2, 1), (2, 3), (2, 512), (2, 1024)])
def test_conv_wgrad_f32(dev, gi, n, kind):
    """rth_conv_wgrad_f32 (conv2 / conv3 weight gradient on the fp32 MFMA) and rth_conv_wgrad_x9
    (the bf16 MFMA, both operands split into three exact bf16 terms) against an fp64 CPU
    convolution backward, within fp32 summation error; deterministic (a second call is bit
    identical) and odd pixel counts (the last pair / 32-pixel chunk partly empty) included"""
    from reth_amd import _lib

    geom = GEOMS[gi]
    cin, h, wd, cout, k, s = geom
    g = torch.Generator().manual_seed(31 * n + gi)
    x = torch.rand((n, cin, h, wd), generator=g) * 2 - 1
    ho = (h - k) // s + 1
    gy = torch.randn((n, cout, ho, ho), generator=g)
    w = torch.zeros((cout, cin, k, k), dtype=torch.float64)
    _, want, _ = torch.ops.aten.convolution_backward(gy.double(), x.double(), w, None, [s, s], [0, 0], [1, 1], False,
                                                     [0, 0], 1, [False, True, False])
    shape = _shape(_lib.CONV_F32_NHWC, *geom)
    assert getattr(_lib.lib(), f"rth_conv_wgrad_{kind}_supported")(_lib.ctypes.byref(shape)) == 1
    ws = torch.empty(getattr(_lib.lib(), f"rth_conv_wgrad_{kind}_workspace")(_lib.ctypes.byref(shape)) // 4, device=dev)
    xd = x.to(dev).contiguous(memory_format=torch.channels_last)
    gyd = gy.to(dev).contiguous(memory_format=torch.channels_last)
    outs = []
    for _ in range(2):
        gw = torch.full((cout, cin, k, k), float("nan"), device=dev).contiguous(memory_format=torch.channels_last)
        _lib.call(f"rth_conv_wgrad_{kind}", _lib.ctypes.byref(shape), xd.data_ptr(), n, gyd.data_ptr(), gw.data_ptr(),
                  ws.data_ptr(), _lib.stream_ptr())
        outs.append(gw)
    assert torch.equal(outs[0], outs[1])
    scale = want.abs().max().item()
    err = (outs[0].double().cpu() - want).abs().max().item()
    assert err <= 2e-6 * max(scale, 1.0) * max(1.0, (n * ho * ho) ** 0.5 / 8), (err, scale)


@pytest.mark.parametrize("gi,n", [(1, 64), (1, 512), (2, 64), (2, 512), (1, 1024)])
def test_conv_fp32_grade_accuracy(dev, gi, n):
    """the exact-split bf16 kernels (k_conv_x9) and the fp32-MFMA kernels are as accurate as an
    fp32 convolution: the worst error against float64 stays within a small multiple of what
    torch's own fp32 CPU convolution makes on the same data (the learner's Adam step, eps
    1.5e-4, turns coarser forward rounding into weight drift: test_learner_full_gpu)"""
    from reth_amd import _lib

    cin, h, wd, cout, k, s = GEOMS[gi]
    g = torch.Generator().manual_seed(1000 + gi * 7 + n)
    x = torch.relu(torch.randn((n, cin, h, wd), generator=g))
    w = torch.randn((cout, cin, k, k), generator=g) / np.sqrt(cin * k * k)
    b = torch.randn(cout, generator=g) * 0.1
    xd = x.to(dev).contiguous(memory_format=torch.channels_last)
    got = _run(_shape(_lib.CONV_F32_NHWC, *GEOMS[gi]), xd, None, n, w, b, dev).double()
    want = _ref(x, w, b, s)
    t32 = F.relu(F.conv2d(x, w, b, stride=s)).double()
    e_ours, e_t32 = (got - want).abs().max().item(), (t32 - want).abs().max().item()
    print(f"conv{gi + 1} n={n}: ours {e_ours:.3e} torch-fp32 {e_t32:.3e}")
    assert e_ours <= 4 * e_t32 + 1e-7, (e_ours, e_t32)


def test_conv_impl_selection(dev):
    """rth_conv_impl names the kernel a launch runs: conv1 on uint8 stacks the bf16x3 kernel,
    conv2 the fp32-MFMA kernel, conv3 the x9 kernel with the
    samples per workgroup of the cost model (one round of at most 4-sample workgroups on 256
    CUs when the batch allows)"""
    import ctypes
    import os

    from reth_amd import _lib

    ns = ctypes.c_int32(-1)
    impl = lambda sh, n: (_lib.lib().rth_conv_impl(ctypes.byref(sh), n, ctypes.byref(ns)), ns.value)
    u8 = _shape(_lib.CONV_U8_CHW, *GEOMS[0])
    assert impl(u8, 1024) == (_lib.CONV_IMPL_BF16X3, 0)
    assert impl(_shape(_lib.CONV_F32_NHWC, *GEOMS[1]), 256) == (_lib.CONV_IMPL_F32, 0)
    c3 = _shape(_lib.CONV_F32_NHWC | _lib.CONV_OUT_NCHW, *GEOMS[2])
    cus = torch.cuda.get_device_properties(dev).multi_processor_count
    slots = cus  # workgroups per round (the model's: one x9 workgroup per CU)
    for n in (1, cus // 2, cus, 2 * cus, 3 * cus, 4 * cus, 6 * cus):
        kind, s = impl(c3, n)
        assert kind == _lib.CONV_IMPL_X9 and 1 <= s <= 4, (n, kind, s)
        rounds = lambda q: -(-(-(-n // q)) // slots)
        # the chosen instantiation's estimated time is the least of the built ones
        assert all(rounds(s) * (s + 0.5) <= rounds(q) * (q + 0.5) for q in (1, 2, 3, 4)), (n, s)
    assert impl(c3, 0)[0] == 0 and impl(_shape(_lib.CONV_F32_NHWC, 3, 84, 84, 32, 8, 4), 8)[0] == 0


@pytest.mark.parametrize("n", [1, 7, 512, 1024])
def test_conv1_frames_in_place_bit_identical(dev, n):
    """frames in place (rth_conv1_frames_bias_relu / rth_conv1_frames_relu_wgrad_ex): conv1
    reading each sample's 4 frames from a frame store by int32 [n][4] frame ids gives the same
    bits as rth_conv_bias_relu / rth_conv_relu_wgrad_ex on the stacks the gather would have
    assembled from those ids (repeated and out-of-order ids, the store's last frame included)"""
    from reth_amd import _lib

    g = torch.Generator().manual_seed(300 + n)
    F_ = 97
    store = torch.randint(0, 256, (F_, 84, 84), dtype=torch.uint8, generator=g).to(dev)
    ids = torch.randint(0, F_, (n, 4), dtype=torch.int32, generator=g)
    ids[0] = torch.tensor([F_ - 1, 0, F_ - 1, 5], dtype=torch.int32)
    ids = ids.to(dev)
    stacks = store[ids.long()].contiguous()  # [n, 4, 84, 84]: the gather's output
    w = (torch.rand((32, 4, 8, 8), generator=g) * 2 - 1) / 16
    b = ((torch.rand(32, generator=g) * 2 - 1) * 0.1).to(dev)
    shape = _shape(_lib.CONV_U8_CHW, *GEOMS[0])
    pk = torch.empty(_lib.lib().rth_conv_packed_bytes(_lib.ctypes.byref(shape)) // 4, device=dev)
    _lib.call("rth_conv_pack", _lib.ctypes.byref(shape), w.to(dev).contiguous(memory_format=torch.channels_last)
              .data_ptr(), pk.data_ptr(), _lib.stream_ptr())
    y_st = torch.full((n, 20, 20, 32), float("nan"), device=dev)
    y_fr = torch.full((n, 20, 20, 32), float("nan"), device=dev)
    _lib.call("rth_conv_bias_relu", _lib.ctypes.byref(shape), stacks.data_ptr(), None, n, pk.data_ptr(), b.data_ptr(),
              y_st.data_ptr(), _lib.stream_ptr())
    _lib.call("rth_conv1_frames_bias_relu", _lib.ctypes.byref(shape), store.data_ptr(), ids.data_ptr(), n,
              pk.data_ptr(), b.data_ptr(), y_fr.data_ptr(), _lib.stream_ptr())
    assert not torch.isnan(y_fr).any()
    assert torch.equal(y_st, y_fr)
    torch.testing.assert_close(y_fr.permute(0, 3, 1, 2).cpu().double(), _ref(stacks.cpu().double(), w, b.cpu(), 4),
                               rtol=1e-5, atol=5e-4)
    # the weight / bias gradients (ReLU mask from y) from the frames == from the stacks
    up = torch.randn((n, 20, 20, 32), generator=g).to(dev)
    ws = torch.empty(_lib.lib().rth_conv_wgrad_workspace(_lib.ctypes.byref(shape)) // 4, device=dev)
    out = []
    for fn, x, ix in (("rth_conv_relu_wgrad_ex", stacks, None), ("rth_conv1_frames_relu_wgrad_ex", store, ids)):
        gw = torch.full((32, 8, 8, 4), float("nan"), device=dev)
        gb = torch.full((32,), float("nan"), device=dev)
        args = [x.data_ptr(), None] if ix is None else [x.data_ptr(), ix.data_ptr()]
        _lib.call(fn, _lib.ctypes.byref(shape), *args, n, up.data_ptr(), y_st.data_ptr(), gw.data_ptr(), gb.data_ptr(),
                  ws.data_ptr(), None, 0, None, 0, _lib.stream_ptr())
        out.append((gw, gb))
    assert not torch.isnan(out[1][0]).any()
    assert torch.equal(out[0][0], out[1][0]) and torch.equal(out[0][1], out[1][1])
    # misaligned ids are refused
    with pytest.raises(RuntimeError):
        _lib.call("rth_conv1_frames_bias_relu", _lib.ctypes.byref(shape), store.data_ptr(), ids.data_ptr() + 4, 1,
                  pk.data_ptr(), b.data_ptr(), y_fr.data_ptr(), _lib.stream_ptr())
