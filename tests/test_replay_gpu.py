"""HBM replay shard + the reth_buffer-compatible API (start_per / Client / loaders).

Mirrors reth_buffer/test/test_rb.py (identity column pins index <-> row), reth/test/
test_buffer.py::test_per (rows and IS weights), plus FIFO wrap-around, exact u8 -> f32
widening, the sample-start gate, and the sample-ahead order, all against the oracle."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_rb_basic_identity_column(dev):
    """reth_buffer/test/test_rb.py:12-35 through the drop-in API"""
    from reth_amd import reth_buffer

    svc, addr = reth_buffer.start_server(100000, 32, device=dev)
    client = reth_buffer.Client(addr)
    loader = reth_buffer.NumpyLoader(addr)
    data = [np.random.rand(1000, 4, 84), np.random.rand(1000), np.arange(1000)]
    w = np.random.rand(1000) + 1
    for start in range(0, 1000, 100):
        client.append([x[start:start + 100] for x in data], w[start:start + 100])
    for _ in range(10):
        batch, indices, weights = loader.sample()
        assert indices.dtype == np.int64 and weights.dtype == np.float64 and len(indices) == 32
        for i, idx in enumerate(indices):
            assert batch[2][i] == idx
            assert batch[1][i] == data[1][idx]
            assert np.array_equal(batch[0][i], data[0][idx])
    client.update_priorities(np.arange(1000), np.random.rand(1000) + 10)
    svc.terminate()
    svc.join()


def test_per_rows_and_is_weights(dev, orc):
    """reth/test/test_buffer.py:113-132: sampled rows equal data[idx]; IS weights equal
    ((w + 1e-6)^alpha / min)^-beta"""
    from reth_amd.replay import Column, HbmReplay

    cap, B = 1000, 64
    rng = np.random.default_rng(0)
    cols = [Column((), torch.int64), Column((4, 84, 84), torch.float32), Column((), torch.int64),
            Column((), torch.float32), Column((4, 84, 84), torch.float32), Column((), torch.float32)]
    rep = HbmReplay(cap, cols, alpha=0.6, beta=0.4, device=dev)
    data = [np.arange(cap), rng.random((cap, 4, 84, 84), dtype=np.float32), rng.integers(0, 10, cap),
            rng.random(cap, dtype=np.float32), rng.random((cap, 4, 84, 84), dtype=np.float32),
            rng.integers(0, 2, cap).astype(np.float32)]
    w = rng.random(cap)
    rep.append([torch.as_tensor(x, device=dev) for x in data], w)
    out, idx, isw = rep.sample(B)
    idx = idx.cpu().numpy()
    for c, col in enumerate(out):
        assert np.array_equal(col.cpu().numpy(), data[c][idx])
    ow = (w + 1e-6) ** 0.6
    np.testing.assert_allclose(isw.cpu().numpy(), (ow[idx] / ow.min()) ** -0.4, atol=1e-3)  # the reference's bound
    p = orc.per_normalize(w, 0.6)
    np.testing.assert_allclose(isw.cpu().numpy(), orc.per_is_weights(p[idx], p.min(), 0.4), rtol=1e-12)


def test_fifo_wraparound_and_u8_widening(dev, orc):
    """FIFO slots wrap (fifo_policy.py:11-18); uint8 frames come back as exact float32"""
    from reth_amd.replay import Column, HbmReplay

    cap = 300
    rep = HbmReplay(cap, [Column((4, 84, 84), torch.uint8, torch.float32), Column((), torch.int64)], alpha=0.5,
                    device=dev)
    rng = np.random.default_rng(1)
    tree = orc.Tree(cap)
    tail = 0
    written = {}
    for step in range(7):
        n = int(rng.integers(1, 130))
        frames = rng.integers(0, 256, (n, 4, 84, 84), dtype=np.uint8)
        ids = np.arange(100 * step, 100 * step + n)
        td = rng.random(n, dtype=np.float32)
        slots_out = torch.empty(n, dtype=torch.int64, device=dev)
        rep.append([torch.as_tensor(frames, device=dev), torch.as_tensor(ids, device=dev)], torch.as_tensor(td, device=dev),
                   idx_out=slots_out)
        slots, tail = orc.fifo_indices(cap, tail, n)
        assert np.array_equal(slots_out.cpu().numpy(), slots)
        tree.update(slots, orc.per_normalize(td, 0.5).astype(np.float64))
        for k, s in enumerate(slots):
            written[int(s)] = (frames[k], ids[k])
    size, gtail, cnt, _, _ = rep.info()
    assert gtail == tail and size == min(cap, cnt)
    s, m, v = rep.tree.export()
    assert np.array_equal(s.cpu().numpy(), tree.sum) and np.array_equal(v.cpu().numpy(), tree.val)
    keys = np.array(sorted(written))
    out = rep.gather(keys)
    assert out[0].dtype == torch.float32
    for k, s_ in enumerate(keys):
        f, i = written[int(s_)]
        assert out[1][k].item() == i
        assert torch.equal(out[0][k].cpu(), torch.as_tensor(f).float())


@pytest.mark.parametrize("planes,shape", [(4, (4, 84, 84)), (3, (3, 5, 7)), (4, (4, 100, 100)), (4, (4, 9, 9)),
                                          (4, (4, 3, 5)), (2, (2, 30, 30))])
def test_channels_last_gather(dev, planes, shape):
    """uint8 (C,H,W) rows sampled as channels-last float32 (the NHWC conv input), exact:
    multi-chunk rows with a partial last chunk (4x84x84: 7 chunks of 1024 pixels), pixel
    counts not divisible by 4 (scalar lanes), rows small enough for one lane per row"""
    from reth_amd import _lib
    from reth_amd.replay import Column, HbmReplay

    rng = np.random.default_rng(planes)
    n = 50
    rows = torch.as_tensor(rng.integers(0, 256, (n, *shape), dtype=np.uint8), device=dev)
    rep = HbmReplay(64, [Column(shape, torch.uint8, torch.float32, channels_last=True), Column((), torch.int64)],
                    device=dev)
    rep.append([rows, torch.arange(n, device=dev)], torch.ones(n, device=dev))
    idx = torch.as_tensor(rng.integers(0, n, 33), device=dev)
    out = rep.gather(idx)
    assert out[0].is_contiguous(memory_format=torch.channels_last)
    assert torch.equal(out[0], rows[idx].float())
    # the raw copy kernel in the same mode (actors' acting / priority batches)
    dst = torch.empty((33, *shape), dtype=torch.float32, device=dev, memory_format=torch.channels_last)
    _lib.call("rth_copy_rows", dst.data_ptr(), 0, None, rows.data_ptr(), 0, idx.data_ptr(), 33, int(np.prod(shape)),
              _lib.RTH_U8, _lib.RTH_F32, planes, _lib.stream_ptr())
    assert torch.equal(dst, rows[idx].float())
    dst2 = torch.empty((33, *shape), dtype=torch.float32, device=dev)
    _lib.call("rth_copy_rows", dst2.data_ptr(), 0, None, rows.data_ptr(), 0, idx.data_ptr(), 33, int(np.prod(shape)),
              _lib.RTH_U8, _lib.RTH_F32, 0, _lib.stream_ptr())
    assert torch.equal(dst2, rows[idx].float())


@pytest.mark.parametrize("nbytes,stride", [(28224, 28224), (1000, 1003), (4096, 4096), (17, 17), (64, 80), (65, 65)])
def test_copy_rows_chunked_bytes(dev, nbytes, stride):
    """raw row copy and u8->f32 widening over the chunked grid: unaligned strides fall back
    to byte lanes, rows <= 64 B take one lane per row, destination rows scattered"""
    from reth_amd import _lib

    rng = np.random.default_rng(nbytes + stride)
    n = 37
    src = torch.as_tensor(rng.integers(0, 256, n * stride, dtype=np.uint8), device=dev)
    view = src.as_strided((n, nbytes), (stride, 1))
    idx = torch.as_tensor(rng.permutation(n), device=dev)
    drow = torch.as_tensor(rng.permutation(n), device=dev)
    dst = torch.zeros((n, nbytes), dtype=torch.uint8, device=dev)
    _lib.call("rth_copy_rows", dst.data_ptr(), 0, drow.data_ptr(), src.data_ptr(), stride, idx.data_ptr(), n, nbytes,
              _lib.RTH_U8, _lib.RTH_U8, 0, _lib.stream_ptr())
    ref = torch.zeros_like(dst)
    ref[drow] = view[idx]
    assert torch.equal(dst, ref)
    dstf = torch.zeros((n, nbytes), dtype=torch.float32, device=dev)
    _lib.call("rth_copy_rows", dstf.data_ptr(), 0, None, src.data_ptr(), stride, idx.data_ptr(), n, nbytes,
              _lib.RTH_U8, _lib.RTH_F32, 0, _lib.stream_ptr())
    assert torch.equal(dstf, view[idx].float())


def test_append_exact_capacity_and_errors(dev):
    from reth_amd import reth_buffer
    from reth_amd.replay import Column, HbmReplay

    rep = HbmReplay(16, [Column((3,), torch.float32)], device=dev)
    rep.append([torch.ones(16, 3, device=dev)], torch.ones(16, device=dev))
    assert rep.info()[:2] == (16, 0)
    with pytest.raises(AssertionError):  # fifo_policy.py:12 assert batch_size <= capacity
        rep.append([torch.ones(17, 3, device=dev)], torch.ones(17, device=dev))
    with pytest.raises(ValueError):
        rep.append([torch.ones(4, 3, device=dev)], torch.ones(5, device=dev))
    svc, addr = reth_buffer.start_per(1000, 64, sample_start=100, device=dev)
    client, loader = reth_buffer.Client(addr), reth_buffer.TorchCudaLoader(addr)
    client.append([np.zeros((50, 2), np.float32)], np.ones(50, np.float32))
    with pytest.raises(RuntimeError):  # cnt 50 < max(sample_start, batch) = 100
        loader.sample()
    client.append([np.zeros((50, 2), np.float32)], np.ones(50, np.float32))
    data, idx, w = loader.sample()
    assert data[0].is_cuda and w.dtype == torch.float64 and idx.shape == (64,)
    with pytest.raises(ValueError):
        reth_buffer.Client("hbm://0/does-not-exist")


@pytest.mark.parametrize("beta_spec", ["0.4,1,1000", "exp,0.4,1,1000"])
def test_torch_cuda_loader_sample_ahead_order(dev, orc, beta_spec):
    """batch k+1 is drawn before batch k's priorities are written back (the sampler's HWM-1
    PUSH, sampler_loop.py:13-15/36-39), with beta stepped by each update message; beta from
    the device Schedule (schedule.py:4-52) in both forms, linear and exp, against the oracle's"""
    from reth_amd import reth_buffer

    cap, B = 5000, 128
    svc, addr = reth_buffer.start_per(cap, B, alpha=0.5, beta=beta_spec, sample_start=B, device=dev, seed=3)
    method = "exp" if beta_spec.startswith("exp") else "linear"
    client, loader = reth_buffer.Client(addr), reth_buffer.TorchCudaLoader(addr, buffer_size=4)
    rng = np.random.default_rng(2)
    ids = np.arange(cap)
    td0 = rng.random(cap, dtype=np.float32)
    client.append([ids], td0)
    tree = orc.Tree(cap)
    tree.update(ids, orc.per_normalize(td0, 0.5).astype(np.float64))
    beta_steps = 0
    pending = None  # oracle's pre-sampled batch
    calls = 0

    def oracle_sample():
        nonlocal calls
        u = np.array([orc.philox_uniform(3, calls, i, orc.STREAM_SAMPLE) for i in range(B)])
        calls += 1
        idx, p = tree.sample(u)
        beta = orc.schedule_value(method, 0.4, 1.0, 1000, beta_steps)
        return idx, orc.per_is_weights(p, tree.min(), beta)

    for k in range(6):
        data, idx, w = loader.sample()
        if pending is None:
            pending = oracle_sample()
        want_idx, want_w = pending
        pending = oracle_sample()  # sample-ahead happens before this batch's update
        assert np.array_equal(idx, want_idx)
        assert np.array_equal(data[0].cpu().numpy(), want_idx)
        np.testing.assert_allclose(w.cpu().numpy(), want_w, rtol=1e-12)
        new = rng.random(B, dtype=np.float32)
        client.update_priorities(idx, new)  # step=True: beta.step() then update
        beta_steps += 1
        tree.update(idx, orc.per_normalize(new, 0.5).astype(np.float64))


def test_deferred_update_merged_into_append(dev, orc):
    """a deferred update_priorities is applied by the next append's tree launch (before the
    append's rows), or before a sample / flush: the tree equals the immediate schedule's"""
    from reth_amd.replay import Column, HbmReplay

    rng = np.random.default_rng(5)
    cap = 700

    def run(deferred):
        rep = HbmReplay(cap, [Column((), torch.int64)], alpha=0.6, beta="0.4,1,100", device=dev, seed=3)
        out = []
        for step in range(12):
            n = ns[step]
            rep.append([torch.arange(n, device=dev)], torch.as_tensor(tds[step], device=dev))
            if step % 3 == 2:
                _, idx, isw = rep.sample(64)
                out += [idx.cpu(), isw.cpu()]
            rep.update_priorities(torch.as_tensor(upd_idx[step], device=dev),
                                  torch.as_tensor(upd_w[step], device=dev), step=True, deferred=deferred)
        s, m, v = rep.tree.export()  # applies a pending update
        return out + [s.cpu(), m.cpu(), v.cpu()], rep.info()

    ns = [int(x) for x in rng.integers(1, 120, 12)]
    tds = [rng.random(n).astype(np.float32) for n in ns]
    upd_idx = [rng.integers(0, min(cap, sum(ns[:k + 1])), 50) for k in range(12)]
    upd_w = [rng.random(50).astype(np.float32) for _ in range(12)]
    a, ia = run(False)
    b, ib = run(True)
    assert ia == ib
    for x, y in zip(a, b):
        assert torch.equal(x, y)


@pytest.mark.parametrize("sampler", ["per", "uniform"])
def test_sample_counter_advance_forms(dev, sampler):
    """the sampler's Philox counter advances once per sample whichever launch carries it: the
    fused gather (sample with outputs), a separate rth_replay_gather (the bench's timed form),
    or the next sample (no gather at all) -- the index sequences are identical"""
    from reth_amd._lib import c_vp, call, ptr, stream_ptr
    from reth_amd.replay import Column, HbmReplay

    cap, B = 4096, 64
    rng = np.random.default_rng(5)
    ids = torch.arange(cap, device=dev)
    w = rng.random(cap) + 0.1

    streams = [torch.cuda.Stream(dev), torch.cuda.Stream(dev)]

    def run(form):
        rep = HbmReplay(cap, [Column((), torch.int64)], alpha=0.6, beta=0.4, device=dev, seed=11,
                        sampler=sampler)
        rep.append([ids], w)
        torch.cuda.synchronize()
        for st in streams:
            st.wait_stream(torch.cuda.current_stream())
        seq, keep = [], []
        for k in range(4):
            cols, idx, isw = rep.new_batch(B)
            arr = (c_vp * 1)(ptr(cols[0]))
            if form == "fused":
                rep.sample_into(B, cols, idx, isw)
            elif form == "cross":  # the gather (which launches the owed counter advance on
                # the sample's stream) on another stream, the next sample on the gather's stream;
                # the advance is held back behind a spin on the sample's stream, so a sample that
                # did not wait for it would read the old counter and repeat the previous draw
                s_sample = streams[k % 2]
                s_gather = streams[(k + 1) % 2]
                call("rth_replay_sample", rep._h, B, None, None, ptr(idx), ptr(isw), s_sample.cuda_stream)
                s_gather.wait_stream(s_sample)  # the gather reads idx
                with torch.cuda.stream(s_sample):
                    torch.cuda._sleep(20_000_000)
                call("rth_replay_gather", rep._h, ptr(idx), B, arr, s_gather.cuda_stream)
                keep.append((cols, idx))
                continue
            else:
                call("rth_replay_sample", rep._h, B, None, None, ptr(idx), ptr(isw), stream_ptr())
                if form == "split":
                    call("rth_replay_gather", rep._h, ptr(idx), B, arr, stream_ptr())
            seq.append(idx.cpu().numpy().copy())
            if form != "none":
                assert np.array_equal(cols[0].cpu().numpy(), seq[-1])
        if keep:
            torch.cuda.synchronize()
            for cols, idx in keep:
                seq.append(idx.cpu().numpy().copy())
                assert np.array_equal(cols[0].cpu().numpy(), seq[-1])
        return np.stack(seq)

    fused = run("fused")
    assert len({tuple(r) for r in fused}) == 4  # every call draws anew
    assert np.array_equal(fused, run("split"))
    assert np.array_equal(fused, run("none"))
    assert np.array_equal(fused, run("cross"))
