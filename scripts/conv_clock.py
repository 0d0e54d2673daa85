"""In-kernel clock of conv2's fp32-MFMA forward (k_conv_bias_relu, the bench's `roofline`
kernel) at the learner's 1,024 samples: back-to-back launches for ~3 s on random data, then the
per-workgroup shader-clock / wall-clock tick ratio (MI355X_MICROARCH.md, DVFS item 6) from the
diagnostic build (scripts/build_clock_lib.sh; run with RTH_LIB_PATH=reth_amd/libreth_hip_clk.so).
Prints the kernel time, TF/s, the median in-kernel clock and the fraction of the fp32 MFMA peak
at that clock (64 FLOP per clock per SIMD, 1,024 SIMDs).  Development aid."""
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from reth_amd import _lib  # noqa: E402

dev = torch.device("cuda")
n = int(os.environ.get("CLK_N", "1024"))
cin, h, w, cout, k, s = 32, 20, 20, 64, 4, 2
x = torch.randn((n, cin, h, w), device=dev).contiguous(memory_format=torch.channels_last)
wt = (torch.randn((cout, cin, k, k), device=dev) * 0.05).contiguous(memory_format=torch.channels_last)
b = torch.randn(cout, device=dev) * 0.1
ho = (h - k) // s + 1
y = torch.empty((n, ho, ho, cout), device=dev)
shp = _lib.ConvShape(_lib.CONV_F32_NHWC, cin, h, w, cout, k, k, s)
pk = torch.empty(_lib.lib().rth_conv_packed_bytes(_lib.ctypes.byref(shp)) // 4, device=dev)
_lib.call("rth_conv_pack", _lib.ctypes.byref(shp), wt.data_ptr(), pk.data_ptr(), _lib.stream_ptr())
flops = 2.0 * n * ho * ho * cout * cin * k * k


def launch():
    _lib.call("rth_conv_bias_relu", _lib.ctypes.byref(shp), x.data_ptr(), None, n, pk.data_ptr(), b.data_ptr(),
              y.data_ptr(), _lib.stream_ptr())


for _ in range(20):
    launch()
torch.cuda.synchronize()
t_end, iters = time.time() + 3.0, 0
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
while time.time() < t_end:
    for _ in range(100):
        launch()
    iters += 100
    torch.cuda.synchronize()
e1.record()
torch.cuda.synchronize()
us = e0.elapsed_time(e1) / iters * 1000.0
buf = np.zeros(2 * 1024, dtype=np.uint64)
_lib.call("rth_debug_conv_clock", buf.ctypes.data, 1024)
clk, wall = buf[0::2].astype(np.float64), buf[1::2].astype(np.float64)
ok = wall > 0
ghz = clk[ok] / wall[ok] * 0.1  # wall ticks are 100 MHz
med = float(np.median(ghz))
tf = flops / us / 1e6
peak_at = 64 * 1024 * med * 1e9 / 1e12
print(json.dumps({"kernel": "k_conv_bias_relu conv2 fp32 MFMA", "samples": n, "launches": iters, "us": round(us, 2),
                  "tflops": round(tf, 1), "clock_ghz_median": round(med, 3),
                  "clock_ghz_p10_p90": [round(float(np.percentile(ghz, 10)), 3), round(float(np.percentile(ghz, 90)), 3)],
                  "workgroups_stamped": int(ok.sum()), "fp32_peak_at_clock_tf": round(peak_at, 1),
                  "frac_of_peak_at_clock": round(tf / peak_at, 3), "frac_of_157.3": round(tf / 157.3, 3)}))
