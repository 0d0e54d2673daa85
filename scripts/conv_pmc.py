"""rth_conv_bias_relu alone (for PMC passes): each torso layer at n = 512, 20 launches."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from reth_amd import _lib  # noqa: E402

dev = torch.device("cuda")
n = int(os.environ.get("CONV_N", "512"))
for li, (mode, cin, h, w, cout, k, s) in enumerate([(1, 4, 84, 84, 32, 8, 4), (0, 32, 20, 20, 64, 4, 2),
                                                     (0, 64, 9, 9, 64, 3, 1)]):
    x = (torch.randint(0, 256, (n, cin, h, w), dtype=torch.uint8, device=dev) if mode else
         torch.randn((n, h, w, cin), device=dev))
    wt = (torch.randn((cout, cin, k, k), device=dev) * 0.05).contiguous(memory_format=torch.channels_last)
    b = torch.randn(cout, device=dev) * 0.1
    ho, wo = (h - k) // s + 1, (w - k) // s + 1
    y = torch.empty((n, ho, wo, cout), device=dev)
    shp = _lib.ConvShape(mode, cin, h, w, cout, k, k, s)
    pk = torch.empty(_lib.lib().rth_conv_packed_bytes(_lib.ctypes.byref(shp)) // 4, device=dev)
    _lib.call("rth_conv_pack", _lib.ctypes.byref(shp), wt.data_ptr(), pk.data_ptr(), _lib.stream_ptr())
    for _ in range(20):
        _lib.call("rth_conv_bias_relu", _lib.ctypes.byref(shp), x.data_ptr(), None, n, pk.data_ptr(), b.data_ptr(),
                  y.data_ptr(), _lib.stream_ptr())
    torch.cuda.synchronize()
print("ok")
