"""Microbench: MIOpen conv (+ rth_bias_relu) vs rth_conv_bias_relu per torso layer."""
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from reth_amd import _lib  # noqa: E402

torch.backends.cudnn.benchmark = True
dev = torch.device("cuda")
GEOMS = [(4, 84, 84, 32, 8, 4), (32, 20, 20, 64, 4, 2), (64, 9, 9, 64, 3, 1)]


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


for n in [int(v) for v in os.environ.get("CONV_NS", "512,768,1536").split(",")]:
    for li, (cin, h, w, cout, k, s) in enumerate(GEOMS):
        x = torch.randn((n, cin, h, w), device=dev).contiguous(memory_format=torch.channels_last)
        wt = (torch.randn((cout, cin, k, k), device=dev) * 0.05).contiguous(memory_format=torch.channels_last)
        b = torch.randn(cout, device=dev) * 0.1
        ho, wo = (h - k) // s + 1, (w - k) // s + 1
        y = torch.empty((n, ho, wo, cout), device=dev)
        flops = 2.0 * n * ho * wo * cout * cin * k * k

        def miopen():
            yy = torch.ops.aten.convolution(x, wt, None, [s, s], [0, 0], [1, 1], False, [0, 0], 1)
            _lib.call("rth_bias_relu", yy.data_ptr(), b.data_ptr(), n * ho * wo, cout, _lib.stream_ptr())

        shp = _lib.ConvShape(_lib.CONV_F32_NHWC, cin, h, w, cout, k, k, s)

        def packed(shape):
            pk = torch.empty(_lib.lib().rth_conv_packed_bytes(_lib.ctypes.byref(shape)) // 4, device=dev)
            _lib.call("rth_conv_pack", _lib.ctypes.byref(shape), wt.data_ptr(), pk.data_ptr(), _lib.stream_ptr())
            return pk

        pk = packed(shp)

        def ours():
            _lib.call("rth_conv_bias_relu", _lib.ctypes.byref(shp), x.data_ptr(), None, n, pk.data_ptr(), b.data_ptr(),
                      y.data_ptr(), _lib.stream_ptr())

        tm, to = timeit(miopen), timeit(ours)
        line = f"n={n} conv{li + 1}: miopen+epi {tm:7.1f} us ({flops / tm / 1e6:6.1f} TF)  ours {to:7.1f} us ({flops / to / 1e6:6.1f} TF)"
        if li == 0:
            st = torch.randint(0, 256, (n, 4, 84, 84), dtype=torch.uint8, device=dev)
            rows = torch.randperm(n, device=dev)
            shu = _lib.ConvShape(_lib.CONV_U8_CHW, cin, h, w, cout, k, k, s)
            pku = packed(shu)

            def ours_u8():
                _lib.call("rth_conv_bias_relu", _lib.ctypes.byref(shu), st.data_ptr(), rows.data_ptr(), n,
                          pku.data_ptr(), b.data_ptr(), y.data_ptr(), _lib.stream_ptr())

            tu = timeit(ours_u8)
            line += f"  ours-u8 {tu:7.1f} us ({flops / tu / 1e6:6.1f} TF)"
        print(line, flush=True)
