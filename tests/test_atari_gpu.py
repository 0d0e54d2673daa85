"""Device Atari preprocessing (MaxAndSkip max, gray, INTER_AREA 84x84, FrameStack) against
the oracle's float32 restatement of OpenCV's 8-bit algorithms: bit-exact frames, and the
frame-stack ring semantics of FrameStack (+ reset) against a deque simulation."""
from collections import deque

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _frames(rng, n):
    f = rng.integers(0, 256, (n, 2, 210, 160, 3), dtype=np.uint8)
    f[0] = 77  # flat
    f[1, :, :, :, :] = np.arange(160, dtype=np.uint8)[None, None, :, None]  # ramps (ties at .5)
    f[2, 0], f[2, 1] = 0, 255  # max picks the second frame
    return f


def test_warp_bit_exact_vs_oracle(dev, orc):
    from reth_amd.atari import AtariPreprocessor

    rng = np.random.default_rng(0)
    raw = _frames(rng, 7)
    pre = AtariPreprocessor(device=dev)
    out = pre.warp(torch.as_tensor(raw, device=dev)).cpu().numpy()
    for i in range(len(raw)):
        assert np.array_equal(out[i], orc.warp_frame(raw[i, 0], raw[i, 1])), i
    assert np.all(out[0] == 77) and np.all(out[2] == 255)


def test_frame_stack_ring_semantics(dev, orc):
    from reth_amd.atari import AtariPreprocessor

    rng = np.random.default_rng(1)
    n, ring, T = 5, 3, 9
    pre = AtariPreprocessor(device=dev)
    frames = torch.zeros((n * ring, 4, 84, 84), dtype=torch.uint8, device=dev)
    stacks = [deque(maxlen=4) for _ in range(n)]
    slot = np.zeros(n, np.int64)
    for t in range(T):
        raw = rng.integers(0, 256, (n, 2, 210, 160, 3), dtype=np.uint8)
        reset = (rng.random(n) < 0.3) | (t == 0)
        new = (slot + 1) % ring
        pre.step(torch.as_tensor(raw, device=dev), frames, ring, torch.as_tensor(slot, device=dev),
                 torch.as_tensor(new, device=dev), reset=torch.as_tensor(reset, device=dev))
        for i in range(n):
            f = orc.warp_frame(raw[i, 0], raw[i, 1])
            if reset[i]:
                stacks[i].extend([f] * 4)
            else:
                stacks[i].append(f)
        slot = new
        got = frames.view(n, ring, 4, 84, 84).cpu().numpy()
        for i in range(n):
            assert np.array_equal(got[i, slot[i]], np.stack(stacks[i])), (t, i)
