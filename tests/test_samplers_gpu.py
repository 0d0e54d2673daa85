"""Uniform / FIFO samplers and the in-process reth.buffer buffers on the device, against
the reference's own outputs (tests/golden/buffers.npz) and its test_buffer.py properties."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _ops(g, key):
    return [(str(x)[0], int(str(x)[1:])) for x in g[key]]


def _scalar_replay(cap, sampler, dev):
    from reth_amd.replay import Column, HbmReplay

    return HbmReplay(cap, [Column((), torch.int64)], device=dev, sampler=sampler)


def test_fifo_sampler_device_matches_reference(golden, dev):
    """FIFOSampler: appends push their FIFO slots, update_priorities pushes its indices;
    samples pop the oldest, with the pushed weights (fifo_sampler.py:8-29)"""
    g = golden("buffers.npz")
    rep = _scalar_replay(50, "fifo", dev)
    for k, (op, n) in enumerate(_ops(g, "fifo_ops")):
        if op == "s":
            assert rep.ready_sample(n) == bool(g[f"fifo{k}_ready"])
            _, idx, w = rep.sample(n)
            assert np.array_equal(idx.cpu().numpy(), g[f"fifo{k}_idx"])
            assert np.array_equal(w.cpu().numpy(), g[f"fifo{k}_w"])
        elif op == "a":
            slots = torch.empty(n, dtype=torch.int64, device=dev)
            rep.append([torch.zeros(n, dtype=torch.int64, device=dev)], torch.as_tensor(g[f"fifo{k}_in_w"], device=dev),
                       idx_out=slots)
            assert np.array_equal(slots.cpu().numpy(), g[f"fifo{k}_in_idx"])
        else:
            rep.update_priorities(g[f"fifo{k}_in_idx"], g[f"fifo{k}_in_w"])
    with pytest.raises(RuntimeError):  # deque.pop() from an empty deque
        rep.sample(rep.sampler_len + 1)


def test_uniform_sampler_device_matches_reference(golden, dev):
    from test_oracle_golden import uniforms_for_positions

    g = golden("buffers.npz")
    rep = _scalar_replay(64, "uniform", dev)
    for k, (op, n) in enumerate(_ops(g, "uni_ops")):
        if op == "s":
            tail = int(g[f"uni{k}_tail"])
            assert rep.sampler_len == tail
            _, idx, w = rep.sample(n, uniforms=uniforms_for_positions(g[f"uni{k}_pos"], tail))
            assert np.array_equal(idx.cpu().numpy(), g[f"uni{k}_idx"])
            assert torch.all(w == 1)
        elif op == "a":
            rep.append([torch.zeros(n, dtype=torch.int64, device=dev)], torch.ones(n, device=dev))
        else:
            rep.update_priorities(g[f"uni{k}_in_idx"], np.ones(n, np.float32))
    # Philox draws cover the list uniformly (reference test_rb-style L1 bound)
    rep2 = _scalar_replay(100, "uniform", dev)
    rep2.append([torch.arange(100, device=dev)], torch.ones(100, device=dev))
    cnt = np.zeros(100)
    for _ in range(200):
        _, idx, _ = rep2.sample(64)
        np.add.at(cnt, idx.cpu().numpy(), 1)
    assert np.mean(np.abs(cnt - cnt.mean()) / cnt.mean()) < 0.1


def test_service_with_uniform_and_fifo_samplers(dev):
    """reth_buffer.start_server with UniformSampler / FIFOSampler: the loaders' weights are
    int64 ones (uniform) or the pushed weights (FIFO)"""
    from reth_amd.reth_buffer import Client, NumpyLoader, TorchCudaLoader, start_server

    for name in ("UniformSampler", "FIFOSampler"):
        svc, addr = start_server(256, 32, samplers=[{"sampler_cls": name, "num_procs": 1, "sample_start": 64}],
                                 device=dev)
        c = Client(addr)
        rows = np.arange(100, dtype=np.float32).reshape(100, 1).repeat(3, 1)
        c.append([rows, np.arange(100)], np.full(100, 0.5, np.float32))
        data, idx, w = NumpyLoader(addr).sample()
        assert np.array_equal(data[1], idx) and np.array_equal(data[0][:, 0], idx.astype(np.float32))
        if name == "UniformSampler":
            assert w.dtype == np.int64 and np.all(w == 1)
        else:
            assert np.array_equal(idx, np.arange(32)) and np.all(w == 0.5)
            data, idx, w = TorchCudaLoader(addr, prefetch=1).sample()
            assert np.array_equal(idx, np.arange(32, 64))
        svc.terminate()


def test_numpy_buffer_device_matches_reference(golden, dev):
    from reth_amd.buffer import DynamicSizeBuffer, NumpyBuffer

    g = golden("buffers.npz")
    nb = NumpyBuffer(10, device=dev)
    for k in range(int(g["nb_steps"])):
        cols = [g[f"nb{k}_in{c}"] for c in range(3)]
        if len(cols[0]) == 1:
            ret = np.array([nb.append([c[0] for c in cols])])
        else:
            ret = np.asarray(nb.append_batch(cols))
        assert np.array_equal(ret, g[f"nb{k}_ret"])
        assert nb._tail == int(g[f"nb{k}_tail"]) and nb.size == int(g[f"nb{k}_size"])
    for c, col in enumerate(nb.data):
        assert np.array_equal(col.cpu().numpy(), g[f"nb_data{c}"])
    assert nb.data[2].dtype == torch.bool
    sel = nb.select(np.array([3, 0, 9, 3]))
    assert np.array_equal(sel[0].cpu().numpy(), g["nb_data0"][[3, 0, 9, 3]])
    u = np.array([0.0, 0.999999, 0.55, 0.1])
    s = nb.sample(4, uniforms=u)
    assert np.array_equal(s[1].cpu().numpy(), g["nb_data1"][(u * nb.size).astype(np.int64)])
    dyn = DynamicSizeBuffer(4, device=dev)
    rng = np.random.default_rng(0)
    caps = []
    for n in (1, 1, 1, 1, 1, 3, 10):
        r = [rng.standard_normal((n, 4)), rng.integers(0, 6, n), rng.random(n) < 0.3]
        if n == 1:
            dyn.append([c[0] for c in r])
        else:
            dyn.append_batch(r)
        caps.append((dyn.capacity, dyn.size))
    assert caps == [tuple(x) for x in g["dyn_caps"].tolist()]


def test_prioritized_buffer_device_matches_reference(golden, dev):
    """reth.buffer.PrioritizedBuffer: appended rows, sampled indices (the reference's own
    uniforms injected), IS weights with alpha/beta stepped on sample, tree sums.  Exact
    while the priorities are f64; after the f32 update_priorities the reference's numpy f32
    pow (SVML on this host) and the device's correctly rounded one may differ by 1 ulp."""
    from reth_amd.buffer import PrioritizedBuffer

    g = golden("buffers.npz")
    pb = PrioritizedBuffer(100, alpha=0.6, beta="0.4,1,1000", device=dev)
    store = {}
    tail = -1
    rtol = 0.0
    for k, op in enumerate(str(x) for x in g["pb_ops"]):
        if op in ("batch_w", "batch"):
            d0, d1 = g[f"pb{k}_d0"], g[f"pb{k}_d1"]
            pb.append_batch([d0, d1], weights=g[f"pb{k}_w"] if op == "batch_w" else None)
            for r in range(len(d1)):
                tail = (tail + 1) % 100
                store[tail] = d0[r]
        elif op == "update":
            pb.update_priorities(g[f"pb{k}_idx"], g[f"pb{k}_w"])
            rtol = 1e-6  # f32 normalisation from here on
        else:
            data, idx, w = pb.sample(len(g[f"pb{k}_u"]), uniforms=g[f"pb{k}_u"])
            assert np.array_equal(idx.cpu().numpy(), g[f"pb{k}_idx"])
            np.testing.assert_allclose(w.cpu().numpy(), g[f"pb{k}_isw"], rtol=max(rtol, 1e-12), atol=0)
            assert np.array_equal(data[0].cpu().numpy(), g[f"pb{k}_rows0"])
        s, _, _ = pb.replay.tree.export()
        np.testing.assert_allclose(s.cpu().numpy(), g[f"pb{k}_sum"], rtol=max(rtol, 1e-14), atol=0)


def test_prioritized_buffer_reference_properties(dev):
    """reth/test/test_buffer.py:113-167 (test_per, test_per_distribution) on the device"""
    from reth_amd.buffer import PrioritizedBuffer

    rng = np.random.default_rng(3)
    cap = 1000
    buf = PrioritizedBuffer(cap, device=dev)
    data = [rng.standard_normal((cap, 3)), np.arange(cap)]
    weights = rng.random(cap)
    buf.append_batch(data, weights=weights)
    res, indices, w = buf.sample(64)
    assert np.array_equal(res[1].cpu().numpy(), indices.cpu().numpy())
    out_w = (weights + 1e-6) ** buf.alpha.value()
    out_w = (out_w / out_w.min()) ** (-buf.beta.value())
    assert np.all(np.abs(out_w[indices.cpu().numpy()] - w.cpu().numpy()) < 1e-3)
    cap = 100
    buf = PrioritizedBuffer(cap, device=dev)
    buf.append_batch([rng.standard_normal((cap, 3)), np.arange(cap)], weights=rng.random(cap))
    for _ in range(2):
        cnt = np.zeros(cap)
        for _ in range(100):
            _, idx, _ = buf.sample(64)
            np.add.at(cnt, idx.cpu().numpy(), 1)
        s, _, v = buf.replay.tree.export()
        p = v.cpu().numpy() / s[0].item()
        assert np.mean(np.abs(cnt / cnt.sum() - p) / p) < 0.1
        buf.update_priorities(np.arange(cap), rng.random(cap))
