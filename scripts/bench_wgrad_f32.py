"""Development aid: rth_conv_wgrad_f32 (conv2 / conv3 weight gradient, fp32 MFMA) and
rth_conv_wgrad_x9 (bf16 MFMA, exact 3 x 3-term split) against MIOpen's weight-gradient solver
(+ its zero fill) at the learner's batch, alone, HIP events."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from reth_amd import _lib

dev = torch.device("cuda:0")
torch.backends.cudnn.benchmark = True
for (cin, h, cout, k, s) in [(32, 20, 64, 4, 2), (64, 9, 64, 3, 1)]:
    n = 512
    ho = (h - k) // s + 1
    x = torch.rand((n, cin, h, h), device=dev).contiguous(memory_format=torch.channels_last)
    gy = torch.randn((n, cout, ho, ho), device=dev).contiguous(memory_format=torch.channels_last)
    w = torch.randn((cout, cin, k, k), device=dev).contiguous(memory_format=torch.channels_last)
    shape = _lib.ConvShape(_lib.CONV_F32_NHWC, cin, h, h, cout, k, k, s)
    ws = torch.empty(_lib.lib().rth_conv_wgrad_f32_workspace(_lib.ctypes.byref(shape)) // 4, device=dev)
    wsx = torch.empty(_lib.lib().rth_conv_wgrad_x9_workspace(_lib.ctypes.byref(shape)) // 4, device=dev)
    gw = torch.empty_like(w)

    def ours():
        _lib.call("rth_conv_wgrad_f32", _lib.ctypes.byref(shape), x.data_ptr(), n, gy.data_ptr(), gw.data_ptr(),
                  ws.data_ptr(), _lib.stream_ptr())

    def ours_x9():
        _lib.call("rth_conv_wgrad_x9", _lib.ctypes.byref(shape), x.data_ptr(), n, gy.data_ptr(), gw.data_ptr(),
                  wsx.data_ptr(), _lib.stream_ptr())

    def miopen():
        torch.ops.aten.convolution_backward(gy, x, w, None, [s, s], [0, 0], [1, 1], False, [0, 0], 1,
                                            [False, True, False])

    ours()
    torch.cuda.synchronize()
    got = gw.clone()
    want = torch.ops.aten.convolution_backward(gy.double(), x.double(), w.double(), None, [s, s], [0, 0], [1, 1],
                                               False, [0, 0], 1, [False, True, False])[1]
    print(f"conv {cin}x{h}: rth_conv_wgrad_f32 max |err| / max |gw| = "
          f"{((got.double() - want).abs().max() / want.abs().max()).item():.2e}", flush=True)
    fns = [("rth_conv_wgrad_f32", ours)]
    if not os.environ.get("WGF_ONLY"):
        fns += [("rth_conv_wgrad_x9", ours_x9), ("miopen", miopen)]
    for name, fn in fns:
        for _ in range(5):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(50):
            fn()
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / 50
        flops = 2.0 * n * ho * ho * cout * cin * k * k
        print(f"conv {cin}x{h}x{h}->{cout} k{k} s{s} n={n}: {name:>20} {us:7.1f} us  {flops / us / 1e6:6.1f} TF/s",
              flush=True)
