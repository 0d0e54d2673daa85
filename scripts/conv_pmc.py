"""rth_conv_bias_relu / rth_conv_dgrad alone (for PMC passes), 20 launches each.

CONV_N (default 1024 = the learner's [s0; s1]) samples; CONV_LAYERS (default "1,2,3,d2")
picks the launches: 1-3 = the torso forward layers (conv3 writes NCHW as in the learner),
d2 / d3 = conv2's / conv3's data gradient (rth_conv_dgrad), w2 / w3 = their weight gradients
on rth_conv_wgrad_x9, at CONV_N / 2 samples (the learner's B)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from reth_amd import _lib  # noqa: E402
from reth_amd.model import nchw_out  # noqa: E402

dev = torch.device("cuda")
n = int(os.environ.get("CONV_N", "1024"))
layers = os.environ.get("CONV_LAYERS", "1,2,3,d2").split(",")
GEOMS = [(1, 4, 84, 84, 32, 8, 4), (0, 32, 20, 20, 64, 4, 2), (0, 64, 9, 9, 64, 3, 1)]
for li, (mode, cin, h, w, cout, k, s) in enumerate(GEOMS):
    if str(li + 1) not in layers:
        continue
    x = (torch.randint(0, 256, (n, cin, h, w), dtype=torch.uint8, device=dev) if mode else
         torch.rand((n, h, w, cin), device=dev))
    wt = (torch.randn((cout, cin, k, k), device=dev) * 0.05).contiguous(memory_format=torch.channels_last)
    b = torch.randn(cout, device=dev) * 0.1
    ho, wo = (h - k) // s + 1, (w - k) // s + 1
    y = torch.empty((n, ho, wo, cout), device=dev)
    shp = _lib.ConvShape(mode, cin, h, w, cout, k, k, s)
    pk = torch.empty(_lib.lib().rth_conv_packed_bytes(_lib.ctypes.byref(shp)) // 4, device=dev)
    _lib.call("rth_conv_pack", _lib.ctypes.byref(shp), wt.data_ptr(), pk.data_ptr(), _lib.stream_ptr())
    run = nchw_out(shp) if li == 2 else shp
    for _ in range(20):
        _lib.call("rth_conv_bias_relu", _lib.ctypes.byref(run), x.data_ptr(), None, n, pk.data_ptr(), b.data_ptr(),
                  y.data_ptr(), _lib.stream_ptr())
    torch.cuda.synchronize()
if "d2" in layers:
    B = n // 2
    shp = _lib.ConvShape(0, 32, 20, 20, 64, 4, 4, 2)
    gy = torch.randn((B, 64, 9, 9), device=dev).contiguous(memory_format=torch.channels_last)
    wt = (torch.randn((64, 32, 4, 4), device=dev) * 0.05).contiguous(memory_format=torch.channels_last)
    gx = torch.empty((B, 32, 20, 20), device=dev).contiguous(memory_format=torch.channels_last)
    for _ in range(20):
        _lib.call("rth_conv_dgrad", _lib.ctypes.byref(shp), gy.data_ptr(), B, wt.data_ptr(), gx.data_ptr(),
                  _lib.stream_ptr())
    torch.cuda.synchronize()
if "d3" in layers:
    B = n // 2
    shp = _lib.ConvShape(0, 64, 9, 9, 64, 3, 3, 1)
    gy = torch.randn((B, 64, 7, 7), device=dev).contiguous(memory_format=torch.channels_last)
    wt = (torch.randn((64, 64, 3, 3), device=dev) * 0.05).contiguous(memory_format=torch.channels_last)
    gx = torch.empty((B, 64, 9, 9), device=dev).contiguous(memory_format=torch.channels_last)
    for _ in range(20):
        _lib.call("rth_conv_dgrad", _lib.ctypes.byref(shp), gy.data_ptr(), B, wt.data_ptr(), gx.data_ptr(),
                  _lib.stream_ptr())
    torch.cuda.synchronize()
for tag, (cin, h, cout, k, s) in (("w2", (32, 20, 64, 4, 2)), ("w3", (64, 9, 64, 3, 1))):
    if tag not in layers:
        continue
    B = n // 2
    ho = (h - k) // s + 1
    shp = _lib.ConvShape(0, cin, h, h, cout, k, k, s)
    x = torch.rand((B, cin, h, h), device=dev).contiguous(memory_format=torch.channels_last)
    gy = torch.randn((B, cout, ho, ho), device=dev).contiguous(memory_format=torch.channels_last)
    gw = torch.empty((cout, cin, k, k), device=dev).contiguous(memory_format=torch.channels_last)
    ws = torch.empty(_lib.lib().rth_conv_wgrad_x9_workspace(_lib.ctypes.byref(shp)) // 4, device=dev)
    for _ in range(20):
        _lib.call("rth_conv_wgrad_x9", _lib.ctypes.byref(shp), x.data_ptr(), B, gy.data_ptr(), gw.data_ptr(),
                  ws.data_ptr(), _lib.stream_ptr())
    torch.cuda.synchronize()
print("ok")
