"""rth_clip_adam alone on the Q-net's parameter set (Pong: 1,685,927 fp32 params in 10 tensors),
HIP events around 200 graph replays; run once per form (RTH_ADAM_ONE_PASS=1: the one-launch form)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from reth_amd.model import DQNNetwork  # noqa: E402
from reth_amd.optim import ClipAdam  # noqa: E402

dev = torch.device("cuda")
net = DQNNetwork((4, 84, 84), 6, dueling=True).to(dev)
ps = [p for p in net.parameters()]
opt = ClipAdam(ps, lr=1e-4, eps=1.5e-4, max_norm=40.0)
for p in ps:
    p.grad = torch.randn_like(p) * 0.01
n = sum(p.numel() for p in ps)
for _ in range(20):
    opt.step()
torch.cuda.synchronize()
# replayed from a HIP graph (as in the learner graph): no host time between the events
st = torch.cuda.Stream()
st.wait_stream(torch.cuda.current_stream())
g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g, stream=st):
    opt.step()
torch.cuda.synchronize()
ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(200)]
for a, b in ev:
    a.record()
    g.replay()
    b.record()
torch.cuda.synchronize()
us = sorted(a.elapsed_time(b) * 1e3 for a, b in ev)
med = us[len(us) // 2]
form = "one-launch" if os.environ.get("RTH_ADAM_ONE_PASS", "0") != "0" else "two-launch"
print(f"clip_adam {form}: {n} params, median {med:.2f} us, min {us[0]:.2f} us, {28 * n / med / 1e3:.0f} GB/s "
      "(28 B/param)")
