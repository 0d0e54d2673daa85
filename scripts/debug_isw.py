import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
from oracle import oracle as orc
from reth_amd.replay import SumTree, PERSampler
dev = torch.device("cuda:0")
rng = np.random.default_rng(0)
n = 3000
td = rng.random(n, dtype=np.float32)
per = PERSampler(4096, alpha=0.5, beta=0.4, device=dev)
per.update(np.arange(n), td)
t = orc.Tree(4096); t.update(np.arange(n), orc.per_normalize(td, 0.5).astype(np.float64))
u = rng.random(64)
idx, isw = per.sample(64, uniforms=u)
oidx, oval = t.sample(u)
print("idx equal", np.array_equal(idx.cpu().numpy(), oidx))
print("device min", per.sumtree.min(), "oracle min", t.min())
oisw = orc.per_is_weights(oval, t.min(), 0.4)
g = isw.cpu().numpy()
rel = np.abs(g - oisw) / oisw
print("max rel", rel.max(), "n diff", (g != oisw).sum())
tp = torch.pow(torch.as_tensor(oval, device=dev) / t.min(), -0.4).cpu().numpy()
print("torch gpu pow vs oracle max rel", (np.abs(tp - oisw) / oisw).max(), " torch vs ours", (np.abs(tp - g)/g).max())
print(g[:4], oisw[:4])
b32 = float(np.float32(0.4))
alt = np.power(oval / t.min(), -b32)
print("f32-beta hypothesis max rel", (np.abs(alt - g) / g).max())
import ctypes
from reth_amd import _lib
print("argtypes", _lib.lib().rth_per_sample.argtypes)
for beta in (0.5, 0.4, 0.25, 0.123456789):
    per.beta = __import__("reth_amd.schedule", fromlist=["Schedule"]).Schedule.from_str(beta)
    idx, isw = per.sample(64, uniforms=u)
    g = isw.cpu().numpy()
    o = orc.per_is_weights(oval, t.min(), beta)
    print("beta", beta, "max rel", (np.abs(g - o) / o).max(), "f32beta-hyp", (np.abs(np.power(oval / t.min(), -float(np.float32(beta))) - g) / g).max())
