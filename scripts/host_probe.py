"""Is the Ape-X iteration host-bound?  Host time to enqueue one iteration (queue drained
first, so nothing blocks) vs its GPU wall time, with a per-phase host breakdown.

    python scripts/host_probe.py [--capacity C] [--iters K]
"""
import argparse
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--capacity", type=int, default=200_000)
    ap.add_argument("--iters", type=int, default=50)
    args = ap.parse_args()
    from reth_amd import apex as apex_mod
    from reth_amd.apex import ApexConfig, ApexDQN

    cfg = ApexConfig(capacity=args.capacity, seed=0, conv_benchmark=True, hip_graph=True)
    ax = ApexDQN(cfg, device=torch.device("cuda", 0))
    ax.prefill(cfg.capacity)
    for _ in range(30):
        ax.iteration()
    torch.cuda.synchronize()

    # per-phase host time: wrap the methods the overlapped iteration calls
    phases = {}

    def wrap(obj, name, label):
        f = getattr(obj, name)

        def g(*a, **k):
            t = time.perf_counter()
            r = f(*a, **k)
            phases[label] = phases.get(label, 0.0) + time.perf_counter() - t
            return r
        setattr(obj, name, g)

    wrap(ax, "_actor_block_graph", "actor_block (graph replay + append)")
    wrap(ax.actors, "append", "  of which append (copy + tree launch)")
    wrap(ax, "_learner_host", "learner_host")
    wrap(ax.loader, "issue", "loader.issue (sample + gather)")
    wrap(ax.replay, "update_priorities", "update_priorities (deferred)")
    t_replay = [0.0]
    orig = torch.cuda.CUDAGraph.replay

    def rep(self):
        t = time.perf_counter()
        orig(self)
        t_replay[0] += time.perf_counter() - t
    torch.cuda.CUDAGraph.replay = rep

    host, wall = [], []
    for _ in range(args.iters):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        ax.iteration()
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        host.append(t1 - t0)
        wall.append(t2 - t0)
    n = args.iters
    print(f"host enqueue per iteration {1e6 * sum(host) / n:8.1f} us (min {1e6 * min(host):.1f})")
    print(f"wall per isolated iteration {1e6 * sum(wall) / n:8.1f} us")
    print(f"  graph.replay() host calls  {1e6 * t_replay[0] / n:8.1f} us")
    for k, v in phases.items():
        print(f"  {k:40s} {1e6 * v / n:8.1f} us")
    # pipelined: back-to-back without syncs (what bench.py times)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        ax.iteration()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"pipelined: host {1e6 * (t1 - t0) / n:8.1f} us/iter, wall {1e6 * (t2 - t0) / n:8.1f} us/iter")
    # each block alone on the GPU (no concurrent work on the other stream)
    G = ax._graphs

    def alone(label, fn, reps=20):
        torch.cuda.synchronize()
        time.sleep(0.05)  # a gap that separates the sections in a kernel trace
        ts = []
        for _ in range(reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            fn()
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1) * 1e3)
        ts.sort()
        print(f"alone: {label:40s} median {ts[len(ts) // 2]:8.1f} us  min {ts[0]:8.1f} us")

    k = ax.loader._pending[0]
    alone("learner graph (pre, slot k)", lambda: ax._learner_replay(("pre", k)))
    alone("learner graph (full, slot k)", lambda: ax._learner_replay(("full", k)))
    alone("actor graph (dedup)", lambda: G["act"]["dedup", ax.actors.pushes % 2].replay())
    alone("actor graph (full)", lambda: G["act"]["full", ax.actors.pushes % 2].replay())
    alone("target pass graph", lambda: G["tgt"][k].replay())
    alone("sample + gather", lambda: ax.replay.sample_into(512, *ax.loader._slots[1 - k]))


if __name__ == "__main__":
    main()
