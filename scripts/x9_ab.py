"""Development aid (r06): the x9 kernels (conv3 forward at the loop's 256 / 512 / 1,024
samples, conv3's and conv2's data gradients at B = 512) alone, HIP events, median of 40; the
outputs saved so two libraries (RTH_LIB_PATH) can be compared bit for bit.
usage: x9_ab.py OUT.pt"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from reth_amd import _lib  # noqa: E402

dev = torch.device("cuda")
g = torch.Generator(device=dev).manual_seed(3)
out, line = {}, []


def timed(fn):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    ev = []
    for _ in range(40):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        ev.append((a, b))
    torch.cuda.synchronize()
    return sorted(a.elapsed_time(b) * 1e3 for a, b in ev)[len(ev) // 2]


c3 = _lib.ConvShape(_lib.CONV_F32_NHWC | _lib.CONV_OUT_NCHW, 64, 9, 9, 64, 3, 3, 1)
w3 = (torch.randn((64, 64, 3, 3), device=dev, generator=g) * 0.05).contiguous(memory_format=torch.channels_last)
b3 = torch.randn(64, device=dev, generator=g) * 0.1
pk = torch.empty(_lib.lib().rth_conv_packed_bytes(_lib.ctypes.byref(c3)) // 4, device=dev)
_lib.call("rth_conv_pack", _lib.ctypes.byref(c3), w3.data_ptr(), pk.data_ptr(), _lib.stream_ptr())
for n in (256, 512, 1024, 1027):
    x = torch.rand((n, 64, 9, 9), device=dev, generator=g).contiguous(memory_format=torch.channels_last)
    y = torch.full((n, 64, 7, 7), float("nan"), device=dev)
    f = lambda: _lib.call("rth_conv_bias_relu", _lib.ctypes.byref(c3), x.data_ptr(), None, n, pk.data_ptr(),
                          b3.data_ptr(), y.data_ptr(), _lib.stream_ptr())
    us = timed(f)
    out[f"conv3_{n}"] = y.cpu()
    line.append(f"conv3 fwd n={n} {us:.1f} us ({2 * n * 49 * 64 * 576 / us / 1e6:.1f} TF/s fp32-eq)")
for name, geo in (("dgrad3", (64, 9, 9, 64, 3, 1)), ("dgrad2", (32, 20, 20, 64, 4, 2))):
    cin, h, wd, cout, k, s = geo
    sh = _lib.ConvShape(_lib.CONV_F32_NHWC, cin, h, wd, cout, k, k, s)
    ho = (h - k) // s + 1
    w = (torch.randn((cout, cin, k, k), device=dev, generator=g) * 0.05).contiguous(memory_format=torch.channels_last)
    ws = torch.empty(max(_lib.lib().rth_conv_dgrad_workspace(_lib.ctypes.byref(sh)), 16) // 4, device=dev)
    for n in (512, 515):
        gy = torch.randn((n, cout, ho, ho), device=dev, generator=g).contiguous(memory_format=torch.channels_last)
        gx = torch.full((n, cin, h, wd), float("nan"), device=dev).contiguous(memory_format=torch.channels_last)
        f = lambda: _lib.call("rth_conv_dgrad_ws", _lib.ctypes.byref(sh), gy.data_ptr(), n, w.data_ptr(), gx.data_ptr(),
                              ws.data_ptr(), _lib.stream_ptr())
        us = timed(f)
        out[f"{name}_{n}"] = gx.cpu()
        line.append(f"{name} n={n} {us:.1f} us ({2 * n * ho * ho * cout * cin * k * k / us / 1e6:.1f} TF/s fp32-eq)")
for l in line:
    print(os.environ.get("RTH_LIB_PATH", "default"), l, flush=True)
bad = [k for k, v in out.items() if torch.isnan(v).any()]
print("NaN in", bad if bad else "none")
torch.save(out, sys.argv[1])  # (write it outside gpurun_out: ~100 MB)
