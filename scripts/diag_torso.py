"""Per-layer accuracy of the HIP conv torso on the learner's own inputs (the golden Pong batch,
uint8 stacks, seeded reference init): each layer's output against a float64 CPU convolution
of the SAME input the kernel read, for the learner's pair batch (n = 2B) and single batch.
Diagnostic only (prints; the GPU tests hold the assertions)."""
import ctypes
import os
import sys

import numpy as np
import torch
import torch.nn.functional as F

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))

from dqn_batch import apex_batch  # noqa: E402

from reth_amd import _lib  # noqa: E402
from reth_amd.model import make_q_network, nchw_out  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    B, A, seed = 512, 6, 4242 + 512 + 6
    torch.manual_seed(seed)
    net = make_q_network((4, 84, 84), A).to(dev)
    s0, s1, *_ = apex_batch(seed, B, A)
    x_all = torch.as_tensor(np.concatenate([s0, s1])).to(dev)
    convs = net._convs()
    shapes = [sh for _, sh in net._torso_shapes((4, 84, 84), True)]
    packed = net.pack_convs(True)
    for n in (1024, 512, 64):
        h = x_all[:n].contiguous()
        for li, (conv, shape) in enumerate(zip(convs, shapes)):
            last = li == len(convs) - 1
            ho = (shape.hin - shape.kh) // shape.stride + 1
            y = torch.empty((n, shape.cout, ho, ho), dtype=torch.float32, device=dev,
                            memory_format=torch.contiguous_format if last else torch.channels_last)
            _lib.call("rth_conv_bias_relu", ctypes.byref(nchw_out(shape) if last else shape), h.data_ptr(), None, n,
                      net._packed_for(packed, li, True).data_ptr(), conv.bias.data_ptr(), y.data_ptr(),
                      _lib.stream_ptr())
            torch.cuda.synchronize()
            xin = h.double().cpu()
            pre = F.conv2d(xin, conv.weight.detach().double().cpu(), conv.bias.detach().double().cpu(),
                           stride=conv.stride)
            want = torch.relu(pre)
            got = y.double().cpu()
            err = (got - want).abs()
            scale = F.conv2d(xin.abs(), conv.weight.detach().double().cpu().abs(), stride=conv.stride)
            rel = (err / scale.clamp_min(1e-30)).max().item()
            t32 = torch.relu(F.conv2d(h.float().cpu(), conv.weight.detach().float().cpu(), conv.bias.detach().float().cpu(),
                                      stride=conv.stride)).double()
            e32 = (t32 - want).abs().max().item()
            near0 = (pre.abs() < 1e-3 * scale).sum().item()
            print(f"n={n} conv{li + 1}: max|err| {err.max().item():.3e} (torch fp32 {e32:.3e})  "
                  f"max err/sum|xw| {rel:.3e}  |out| max {want.max().item():.2e}  pre~0 {near0}", flush=True)
            worst = torch.nonzero(err == err.max())[0].tolist()
            print(f"    worst at {worst}: got {got[tuple(worst)].item():.6e} want {want[tuple(worst)].item():.6e} "
                  f"scale {scale[tuple(worst)].item():.3e}", flush=True)
            h = y


if __name__ == "__main__":
    main()
