"""Probe: sum-tree find/sample/update kernel latency vs capacity on the GPU, with caches
flushed before every launch (a 1 GiB buffer rewritten), as in the Ape-X loop where the
replay gather streams >100 MB between tree operations (development aid; read the kernel
durations from a rocprofv3 --kernel-trace of this script)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from reth_amd.replay import SumTree

dev = torch.device("cuda:0")
flush = torch.empty(1 << 28, dtype=torch.float32, device=dev)
cold = os.environ.get("PROBE_WARM") is None


def run(fn, n=55):
    for _ in range(n):
        if cold:
            flush.fill_(1.0)
        fn()
    torch.cuda.synchronize()


for cap in (1024, 65536, 1 << 20, 4 << 20):
    t = SumTree(cap, device=dev)
    g = torch.Generator(device=dev).manual_seed(0)
    t.update(torch.arange(cap, device=dev), torch.rand(cap, device=dev, generator=g, dtype=torch.float64) + 0.01)
    total = float(t.sum())
    tg = torch.sort(torch.rand(512, device=dev, dtype=torch.float64, generator=g) * total).values
    idx = torch.randint(0, cap, (512,), device=dev, generator=g)
    w = torch.rand(512, device=dev, dtype=torch.float64, generator=g)

    def finds():
        t.find(tg)
        if cold:
            flush.fill_(1.0)
        t.find(tg[:1])

    run(finds)
    run(lambda: t.sample(512))
    run(lambda: t.update(idx, w))
    print(f"cap {cap} done", flush=True)
