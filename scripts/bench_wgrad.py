"""Microbench: rth_conv_relu_wgrad (conv1 weight gradient from uint8 stacks) at the learner's
batch (B = 512 stacks), HIP-event timed; RTH_LIB_PATH selects a build variant."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from reth_amd import _lib  # noqa: E402

dev = torch.device("cuda")
n = int(os.environ.get("WGRAD_N", "512"))
shape = _lib.ConvShape(_lib.CONV_U8_CHW, 4, 84, 84, 32, 8, 8, 4)
x = torch.randint(0, 256, (n, 4, 84, 84), dtype=torch.uint8, device=dev)
g = torch.randn(n, 20, 20, 32, device=dev)
y = torch.randn(n, 20, 20, 32, device=dev)
gw = torch.empty(32, 8, 8, 4, device=dev)
gb = torch.empty(32, device=dev)
ws = torch.empty(_lib.lib().rth_conv_wgrad_workspace(_lib.ctypes.byref(shape)) // 4, device=dev)


def run():
    _lib.call("rth_conv_relu_wgrad", _lib.ctypes.byref(shape), x.data_ptr(), None, n, g.data_ptr(), y.data_ptr(),
              gw.data_ptr(), gb.data_ptr(), ws.data_ptr(), _lib.stream_ptr())


for _ in range(5):
    run()
ts = []
for _ in range(30):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    run()
    e1.record()
    torch.cuda.synchronize()
    ts.append(e0.elapsed_time(e1) * 1e3)
ts.sort()
flops = 2.0 * n * 400 * 32 * 256
print(f"{os.path.basename(_lib.LIB_PATH)} n={n}: median {ts[15]:.1f} us ({flops / ts[15] / 1e6:.1f} TF/s), min {ts[0]:.1f} us")
