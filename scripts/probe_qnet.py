"""Probe: kernel counts / time of Q-network forward variants on the GPU (development aid)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import torch.nn.functional as F

from reth_amd.model import DQNNetwork

torch.backends.cudnn.benchmark = True
dev = torch.device("cuda:0")
torch.manual_seed(0)
net = DQNNetwork((4, 84, 84), 6).to(dev, memory_format=torch.channels_last).requires_grad_(False)
x = (torch.rand(512, 4, 84, 84, device=dev) * 255).floor().contiguous(memory_format=torch.channels_last)


def fused_forward(x):
    f = net.features
    h = torch.miopen_convolution_relu(x, f[0].weight, f[0].bias, [4, 4], [0, 0], [1, 1], 1)
    h = torch.miopen_convolution_relu(h, f[2].weight, f[2].bias, [2, 2], [0, 0], [1, 1], 1)
    h = torch.miopen_convolution_relu(h, f[4].weight, f[4].bias, [1, 1], [0, 0], [1, 1], 1)
    h = h.flatten(1) if h.is_contiguous() else h.contiguous().flatten(1)
    return h


def ref_features(x):
    return net.features(x).flatten(1)


def timeit(fn, n=50):
    for _ in range(5):
        fn(x)
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(n):
        fn(x)
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / n * 1e6


with torch.no_grad():
    a = ref_features(x)
    b = fused_forward(x)
    print("features max abs diff", (a - b).abs().max().item(), "rel", ((a - b).abs().max() / a.abs().max()).item())
    print("ref features us", timeit(ref_features))
    print("fused features us", timeit(fused_forward))
    w1 = torch.cat([net.fc_adv[0].weight, net.fc_value[0].weight])
    b1 = torch.cat([net.fc_adv[0].bias, net.fc_value[0].bias])
    h = a
    r1 = torch.cat([F.relu(F.linear(h, net.fc_adv[0].weight, net.fc_adv[0].bias)),
                    F.relu(F.linear(h, net.fc_value[0].weight, net.fc_value[0].bias))], 1)
    r2 = torch._addmm_activation(b1, h, w1.t())
    print("fc1 fused diff", (r1 - r2).abs().max().item())
    print("fc1 ref us", timeit(lambda _: [F.relu(F.linear(h, net.fc_adv[0].weight, net.fc_adv[0].bias)),
                                           F.relu(F.linear(h, net.fc_value[0].weight, net.fc_value[0].bias))]))
    print("fc1 fused us", timeit(lambda _: torch._addmm_activation(b1, h, w1.t())))
    print("full ref forward us", timeit(lambda v: net(v)))
