"""Remote ingest into the HBM replay over ZMTP: the service started the way
test/apex-dqn/trainer.py:52-61 starts it (start_per(..., port=...)) serves the reference's
meta / append / update sockets (reth_amd/zmtp.py); messages from a hand-built ZMTP peer and
from a separate worker process (the reference's Client over the wire, worker.py:21-61's
append shape: 64-row batches of float32 frames, compress=True) land in HBM bit for bit."""
import json
import os
import subprocess
import sys
import time

import numpy as np
import pytest
import torch

from test_zmtp_cpu import connect, long, read_frame, short

pytestmark = pytest.mark.gpu


def _wait_ready(svc, timeout=60.0):
    t0 = time.time()
    while not svc.ready():
        assert time.time() - t0 < timeout, "remote messages did not arrive"
        time.sleep(0.01)


def test_remote_append_and_update_over_zmtp(golden, orc, dev):
    from reth_amd import zmtp
    from reth_amd.reth_buffer import NumpyLoader, start_per

    g = golden("pack.npz")
    svc, addr = start_per(64, 4, alpha=0.5, sample_start=18, host="127.0.0.1", port=0, device=dev, widen_u8={0, 3})
    try:
        assert addr.startswith("tcp://127.0.0.1:")
        meta = zmtp.Endpoint.__new__(zmtp.Endpoint)  # the REQ side by hand: the config
        meta.host, meta.port = "127.0.0.1", int(addr.rsplit(":", 1)[1])
        s, _ = connect(meta, b"REQ")
        s.sendall(short(b"", more=True) + short(b""))
        read_frame(s)
        cfg = json.loads(read_frame(s)[1])
        s.close()
        assert cfg["meta_addr"] == addr and cfg["batch_size"] == 4 and cfg["capacity"] == 64
        app = zmtp.Endpoint.__new__(zmtp.Endpoint)
        app.host, app.port = "127.0.0.1", int(cfg["append_addr"].rsplit(":", 1)[1])
        s, _ = connect(app, b"PUSH")
        msg = g["app_msg"].tobytes()
        for _ in range(3):
            s.sendall(long(msg))
        _wait_ready(svc)  # 18 rows: the drain ran on this (the owner) thread
        rep = svc.replay
        assert rep.info()[0] == 18
        n = len(g["app_w"])
        out = rep.gather(torch.arange(18, device=dev))
        for o, ref in zip(out, [g["app_s0"], g["app_a"], g["app_r"], g["app_s1"], g["app_done"]]):
            assert np.array_equal(o.cpu().numpy(), np.concatenate([ref] * 3))
        _, _, v = rep.tree.export()
        want = orc.per_normalize(g["app_w"], 0.5).astype(np.float64)
        assert np.array_equal(v.cpu().numpy()[:18], np.concatenate([want] * 3))
        # a priority update message (indices 0..4, the reference's own bytes) over the update socket
        upd = zmtp.Endpoint.__new__(zmtp.Endpoint)
        upd.host, upd.port = "127.0.0.1", int(cfg["update_addr"].rsplit(":", 1)[1])
        u, _ = connect(upd, b"PUSH")
        u.sendall(long(g["upd_msg"].tobytes()))
        t0 = time.time()
        while svc.drain() == 0:
            assert time.time() - t0 < 30
            time.sleep(0.01)
        _, _, v = rep.tree.export()
        assert np.array_equal(v.cpu().numpy()[:5], orc.per_normalize(g["app_w"][:5], 0.5).astype(np.float64))
        assert rep.info()[4] == 1  # step=True: beta stepped once
        data, idx, w = NumpyLoader(addr).sample()
        assert np.array_equal(data[0], g["app_s0"][idx % n])
        s.close()
        u.close()
    finally:
        svc.terminate()


WORKER = r'''
import sys
import numpy as np
sys.path.insert(0, sys.argv[2])
from reth_buffer import Client   # reth_amd/compat: the reference's import name
rng = np.random.default_rng(int(sys.argv[3]))
client = Client(sys.argv[1])     # a tcp:// address not served in this process: the wire path
for _ in range(int(sys.argv[4])):  # test/apex-dqn/worker.py:44-60: 64-row batches, compress=True
    s0 = rng.integers(0, 256, (64, 4, 84, 84)).astype("f4")
    s1 = rng.integers(0, 256, (64, 4, 84, 84)).astype("f4")
    a = rng.integers(0, 6, 64).astype("i8")
    r = rng.choice(np.array([-1, 0, 1], "f4"), 64)
    d = (rng.random(64) < 0.01).astype("f4")
    w = rng.random(64).astype("f4")
    client.append([s0, a, r, s1, d], w, compress=True)
print("sent", flush=True)
'''


def test_worker_process_feeds_the_hbm_replay(orc, dev):
    """a separate CPU process -- the reference's worker append loop under the compat import
    names, no GPU -- feeds a GPU-resident shard through TCP"""
    from reth_amd.reth_buffer import start_per

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    batches, seed = 5, 11
    svc, addr = start_per(1024, 64, alpha=0.5, sample_start=64 * batches, host="127.0.0.1", port=0, device=dev,
                          widen_u8={0, 3})
    try:
        env = dict(os.environ, HIP_VISIBLE_DEVICES="", CUDA_VISIBLE_DEVICES="", PYTHONPATH=root)
        p = subprocess.Popen([sys.executable, "-c", WORKER, addr, os.path.join(root, "reth_amd", "compat"), str(seed),
                              str(batches)], env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
        t0 = time.time()
        while not svc.ready():  # drains as the messages arrive (HWM 10: the worker may block on us)
            assert p.poll() is None or p.returncode == 0, p.stderr.read()
            assert time.time() - t0 < 120, "worker messages did not arrive"
            time.sleep(0.01)
        out, err = p.communicate(timeout=60)
        assert p.returncode == 0 and "sent" in out, err
        rng = np.random.default_rng(seed)
        rep = svc.replay
        assert rep.info()[0] == 64 * batches
        got = rep.gather(torch.arange(64 * batches, device=dev))
        _, _, v = rep.tree.export()
        v = v.cpu().numpy()
        for b in range(batches):
            s0 = rng.integers(0, 256, (64, 4, 84, 84)).astype("f4")
            s1 = rng.integers(0, 256, (64, 4, 84, 84)).astype("f4")
            a = rng.integers(0, 6, 64).astype("i8")
            r = rng.choice(np.array([-1, 0, 1], "f4"), 64)
            d = (rng.random(64) < 0.01).astype("f4")
            w = rng.random(64).astype("f4")
            sl = slice(64 * b, 64 * (b + 1))
            for o, ref in zip(got, [s0, a, r, s1, d]):
                assert np.array_equal(o[sl].cpu().numpy(), ref)
            assert np.array_equal(v[sl], orc.per_normalize(w, 0.5).astype(np.float64))
    finally:
        svc.terminate()


def test_loader_waits_for_a_worker_started_after_it(dev):
    """the reference trainer's order (test/apex-dqn/trainer.py:22-34): the shard and its
    TorchCudaLoader exist before any worker has sent a row; the first sample() waits -- as
    torch_cuda_loader.py:94-107,152-163 and sampler_loop.py:23-28 do -- draining the remote
    appends as they arrive, then returns rows bit-identical to the worker's"""
    from reth_amd.reth_buffer import NumpyLoader, TorchCudaLoader, start_per

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    batches, seed = 4, 5
    svc, addr = start_per(1024, 32, alpha=0.5, sample_start=64 * batches, host="127.0.0.1", port=0, device=dev,
                          widen_u8={0, 3})
    try:
        loader = TorchCudaLoader(addr, buffer_size=4, num_procs=2, timeout=180)  # no rows yet
        with pytest.raises(TimeoutError):
            NumpyLoader(addr, timeout=0.2).sample()  # nothing sent yet: a bounded wait ends
        env = dict(os.environ, HIP_VISIBLE_DEVICES="", CUDA_VISIBLE_DEVICES="", PYTHONPATH=root)
        p = subprocess.Popen([sys.executable, "-c", WORKER, addr, os.path.join(root, "reth_amd", "compat"), str(seed),
                              str(batches)], env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
        t0 = time.time()
        data, idx, w = loader.sample()  # blocks until 256 rows are in
        waited = time.time() - t0
        out, err = p.communicate(timeout=60)
        assert p.returncode == 0 and "sent" in out, err
        assert svc.replay.cnt >= 64 * batches and waited > 0
        rng = np.random.default_rng(seed)
        ref = [[] for _ in range(5)]
        for _ in range(batches):
            s0 = rng.integers(0, 256, (64, 4, 84, 84)).astype("f4")
            s1 = rng.integers(0, 256, (64, 4, 84, 84)).astype("f4")
            a = rng.integers(0, 6, 64).astype("i8")
            r = rng.choice(np.array([-1, 0, 1], "f4"), 64)
            d = (rng.random(64) < 0.01).astype("f4")
            rng.random(64)
            for k, c in enumerate((s0, a, r, s1, d)):
                ref[k].append(c)
        ref = [np.concatenate(c) for c in ref]
        assert idx.shape == (32,) and w.dtype == torch.float64
        for o, c in zip(data, ref):
            assert np.array_equal(o.cpu().numpy(), c[idx])
        assert not getattr(svc, "ingest_errors", None)
    finally:
        svc.terminate()
