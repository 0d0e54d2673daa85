"""Device ingest of a Client.append wire-format message (the reference's own bytes) into
an HBM replay: float32 frames narrowed to uint8 storage, every column equal to the rows the
reference's actor serialized, priorities (w + 1e-6) ** alpha in the tree."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("frames_u8", [True, False])
def test_ingest_append_message(golden, orc, dev, frames_u8):
    from reth_amd.pack import ingest_append
    from reth_amd.replay import Column, HbmReplay

    g = golden("pack.npz")
    s0, s1 = g["app_s0"], g["app_s1"]
    fr = (lambda: Column(s0.shape[1:], torch.uint8, torch.float32)) if frames_u8 else \
        (lambda: Column(s0.shape[1:], torch.float32))
    cols = [fr(), Column((), torch.int64), Column((), torch.float32), fr(), Column((), torch.float32)]
    rep = HbmReplay(16, cols, alpha=0.5, device=dev)
    n = ingest_append(rep, g["app_msg"].tobytes())
    assert n == len(g["app_w"])
    out = rep.gather(torch.arange(n, device=dev))
    for o, ref in zip(out, [s0, g["app_a"], g["app_r"], s1, g["app_done"]]):
        assert np.array_equal(o.cpu().numpy(), ref)
    _, _, v = rep.tree.export()
    assert np.array_equal(v.cpu().numpy()[:n], orc.per_normalize(g["app_w"], 0.5).astype(np.float64))


def test_service_append_message(golden, dev):
    """ReplayService side: the first message creates the shard (frames stored as bytes via
    widen_u8), later messages go through the same device ingest"""
    from reth_amd.reth_buffer import Client, NumpyLoader, start_per

    g = golden("pack.npz")
    svc, addr = start_per(64, 4, sample_start=4, device=dev, widen_u8={0, 3})
    c = Client(addr)
    for _ in range(3):
        c.append_message(g["app_msg"].tobytes())
    rep = svc.replay
    assert rep.columns[0].dtype == torch.uint8 and rep.columns[0].out_dtype == torch.float32
    assert rep.info()[0] == 18
    data, idx, w = NumpyLoader(addr).sample()
    assert np.array_equal(data[0], g["app_s0"][idx % 6]) and np.array_equal(data[1], g["app_a"][idx % 6])
    svc.terminate()
