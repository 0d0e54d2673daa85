"""Microbench: conv2 / conv3 data gradient, MIOpen (aten.convolution_backward, data only) vs
rth_conv_dgrad, at the learner's B = 512 (development aid)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from reth_amd import _lib  # noqa: E402

torch.backends.cudnn.benchmark = True
dev = torch.device("cuda")
GEOMS = [(32, 20, 20, 64, 4, 2), (64, 9, 9, 64, 3, 1)]


def timeit(fn, iters=50):
    for _ in range(5):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1000.0


n = int(os.environ.get("DGRAD_N", "512"))
for cin, h, w, cout, k, s in GEOMS:
    ho, wo = (h - k) // s + 1, (w - k) // s + 1
    x = torch.randn((n, cin, h, w), device=dev).contiguous(memory_format=torch.channels_last)
    gy = torch.randn((n, cout, ho, wo), device=dev).contiguous(memory_format=torch.channels_last)
    wt = (torch.randn((cout, cin, k, k), device=dev) * 0.05).contiguous(memory_format=torch.channels_last)
    gx = torch.empty_like(x)
    shape = _lib.ConvShape(_lib.CONV_F32_NHWC, cin, h, w, cout, k, k, s)
    flops = 2.0 * n * ho * wo * cout * cin * k * k

    def miopen():
        torch.ops.aten.convolution_backward(gy, x, wt, None, [s, s], [0, 0], [1, 1], False, [0, 0], 1,
                                            [True, False, False])

    def ours():
        _lib.call("rth_conv_dgrad", _lib.ctypes.byref(shape), gy.data_ptr(), n, wt.data_ptr(), gx.data_ptr(),
                  _lib.stream_ptr())

    ref = miopen_out = torch.ops.aten.convolution_backward(gy, x, wt, None, [s, s], [0, 0], [1, 1], False, [0, 0], 1,
                                                           [True, False, False])[0]
    ours()
    torch.cuda.synchronize()
    err = (gx - ref).abs().max().item()
    tm, to = timeit(miopen), timeit(ours)
    print(f"n={n} dgrad {cin}x{h}x{w}<-{cout} k{k} s{s}: miopen {tm:7.1f} us ({flops / tm / 1e6:6.1f} TF)  "
          f"ours {to:7.1f} us ({flops / to / 1e6:6.1f} TF)  max|diff| {err:.2e}", flush=True)
