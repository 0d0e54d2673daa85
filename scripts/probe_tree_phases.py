"""Probe: phase timing of the sum-tree update in the Ape-X loop's launch shape -- the
previous learner update's 512 deferred priorities merged into one append -- on a full
Pong shard (1M rows, 256 appended) and a Breakout shard (4M rows, 2,048 appended), caches
flushed first (development aid; kernel durations: rocprofv3 --kernel-trace of this script)."""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from reth_amd import _lib
from reth_amd.replay import Column, HbmReplay

dev = torch.device("cuda:0")
flush = torch.empty(1 << 28, dtype=torch.float32, device=dev)
out = (ctypes.c_longlong * 9)()
for cap, n_app in ((1_000_000, 256), (4_000_000, 2048)):
    rep = HbmReplay(cap, [Column((), torch.int64)], alpha=0.5, device=dev)
    n = 1 << 18
    for k in range(0, cap, n):
        m = min(n, cap - k)
        rep.append([torch.arange(m, device=dev)], torch.rand(m, device=dev) + 0.01)
    m = cap // 2 + 12345  # the FIFO tail somewhere mid-ring (slot 0 would put the append in the top levels)
    rep.append([torch.arange(m, device=dev)], torch.rand(m, device=dev) + 0.01)
    g = torch.Generator(device=dev).manual_seed(0)
    torch.cuda.synchronize()
    _lib.call("rth_debug_tree_timing", ctypes.cast(out, _lib.c_vp))
    for trial in range(12):
        idx = torch.randint(0, cap, (512,), device=dev, generator=g)
        td = torch.rand(512, device=dev, generator=g)
        rep.update_priorities(idx, td, step=True, deferred=True)
        flush.fill_(1.0)
        torch.cuda.synchronize()
        rep.append([torch.arange(n_app, device=dev)], torch.rand(n_app, device=dev, generator=g))  # merged launch
        torch.cuda.synchronize()
        _lib.call("rth_debug_tree_timing", ctypes.cast(out, _lib.c_vp))
        t = [x / 100.0 for x in out]  # 100 MHz ticks -> us
        print(f"cap {cap} +{n_app}: sub wg0 loads {t[1] - t[0]:6.1f}  sub last end {t[5] - t[0]:6.1f}  "
              f"gap {t[2] - t[5]:6.1f}  top scan {t[3] - t[2]:6.1f}  top rest {t[4] - t[3]:6.1f}  "
              f"total {t[4] - t[0]:6.1f} us | top: prio {t[6] - t[3]:5.1f} bottom {t[7] - t[6]:5.1f} "
              f"levels {t[8] - t[7]:5.1f} state {t[4] - t[8]:5.1f}", flush=True)
    del rep
    torch.cuda.synchronize()
