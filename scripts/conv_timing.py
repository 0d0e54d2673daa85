"""Probe (with a CONV_PROBE_TIMING build via RTH_LIB_PATH): per-wave timestamps of
rth_conv_bias_relu -> staging time, loop time, tiles per wave, effective shader clock."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from reth_amd import _lib  # noqa: E402

dev = torch.device("cuda")
for n in (512, 1536):
    for li, (mode, cin, h, w, cout, k, s) in enumerate([(1, 4, 84, 84, 32, 8, 4), (0, 32, 20, 20, 64, 4, 2),
                                                         (0, 64, 9, 9, 64, 3, 1)]):
        x = (torch.randint(0, 256, (n, cin, h, w), dtype=torch.uint8, device=dev) if mode else
             torch.randn((n, h, w, cin), device=dev))
        wt = (torch.randn((cout, cin, k, k), device=dev) * 0.05).contiguous(memory_format=torch.channels_last)
        b = torch.randn(cout, device=dev) * 0.1
        ho, wo = (h - k) // s + 1, (w - k) // s + 1
        y = torch.zeros((n * ho * wo * cout + (1 << 20),), device=dev)
        shp = _lib.ConvShape(mode, cin, h, w, cout, k, k, s)
        pk = torch.empty(_lib.lib().rth_conv_packed_bytes(_lib.ctypes.byref(shp)) // 4, device=dev)
        _lib.call("rth_conv_pack", _lib.ctypes.byref(shp), wt.data_ptr(), pk.data_ptr(), _lib.stream_ptr())
        for _ in range(3):
            y.zero_()
            _lib.call("rth_conv_bias_relu", _lib.ctypes.byref(shp), x.data_ptr(), None, n, pk.data_ptr(),
                      b.data_ptr(), y.data_ptr(), _lib.stream_ptr())
        torch.cuda.synchronize()
        off = (n * ho * wo * cout + 1) // 2
        rec = y.view(torch.int64)[off: off + 6 * 8192].cpu().numpy().reshape(-1, 6)
        rec = rec[rec[:, 0] > 0]
        t0 = rec[:, 0].min()
        start, staged, end = (rec[:, 0] - t0) / 100.0, (rec[:, 1] - t0) / 100.0, (rec[:, 2] - t0) / 100.0  # us
        clk = rec[:, 3] / np.maximum(rec[:, 2] - rec[:, 0], 1) * 100e6 / 1e9
        tiles = rec[:, 4]
        cu = (rec[:, 5] >> 8) & 0xF
        simd = (rec[:, 5] >> 4) & 0x3
        se = (rec[:, 5] >> 13) & 0x7
        print(f"n={n} conv{li + 1}: waves {len(rec)} | start max {start.max():.2f} us | staged-start "
              f"med {np.median(staged - start):.2f} max {(staged - start).max():.2f} | end max {end.max():.2f} "
              f"med {np.median(end):.2f} | tiles/wave min {tiles.min()} max {tiles.max()} | clock GHz med "
              f"{np.median(clk):.2f} | simd ids {np.bincount(simd, minlength=4).tolist()}", flush=True)
        per_tile = (end - staged) / np.maximum(tiles, 1)
        mf = {0: 128, 1: 512, 2: 576}[li]
        print(f"    loop us/tile med {np.median(per_tile):.2f} (MFMA-bound at 2 waves/SIMD, 2.4 GHz: "
              f"{2 * mf * 32 / 2.4e3:.2f}) | waves ending after 90% of max: {(end > 0.9 * end.max()).sum()}")
