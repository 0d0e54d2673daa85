"""Probe: phase timing of one k_tree_update (768 keys: 512 random + 256 FIFO) on a 1M tree
with caches flushed first (development aid)."""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from reth_amd import _lib
from reth_amd.replay import Column, HbmReplay

dev = torch.device("cuda:0")
rep = HbmReplay(1 << 20, [Column((), torch.int64)], alpha=0.5, device=dev)
n = 16384
for k in range(0, 1 << 20, n):
    rep.append([torch.arange(n, device=dev)], torch.rand(n, device=dev) + 0.01)
flush = torch.empty(1 << 28, dtype=torch.float32, device=dev)
g = torch.Generator(device=dev).manual_seed(0)
out = (ctypes.c_longlong * 5)()
for trial in range(5):
    idx = torch.randint(0, 1 << 20, (512,), device=dev, generator=g)
    td = torch.rand(512, device=dev, generator=g)
    rep.update_priorities(idx, td, step=True, deferred=True)
    flush.fill_(1.0)
    torch.cuda.synchronize()
    rep.append([torch.arange(256, device=dev)], torch.rand(256, device=dev, generator=g))  # merged launch
    torch.cuda.synchronize()
    _lib.call("rth_debug_tree_timing", ctypes.cast(out, _lib.c_vp))
    t = [x / 100.0 for x in out]  # 100 MHz ticks -> us
    print(f"prefetch {t[1] - t[0]:6.1f}  sort {t[2] - t[1]:6.1f}  vals {t[3] - t[2]:6.1f}  levels {t[4] - t[3]:6.1f}  "
          f"total {t[4] - t[0]:6.1f} us", flush=True)
