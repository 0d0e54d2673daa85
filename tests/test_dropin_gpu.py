"""test/apex-dqn/trainer.py:19-41's loop body through reth_amd under the reference's own
import names (reth_amd/compat on sys.path): K = 4 start_per shards of C // K (:52-61),
reth_buffer.TorchCudaLoader(buffer_size=4, num_procs=2), get_trainer from the restated
config.yaml, trainer.step -> CPU |td| -> update_priorities(np.asarray(...)), and the
torch.save weights stream every send_weights_interval updates over perwez's broadcast to a
CPU worker solver (latest wins).  The shards are filled with worker.py-shaped rows (float32
frames, compress=True).  Capacity is scaled from 1 M to 4 x 1,200 rows: the loop shape, not
the size, is under test (float32 frames at 1 M rows would be 226 GB)."""
import io
import os
import sys

import numpy as np
import pytest
import torch
import yaml

from test_dropin_cpu import APEX_CONFIG, COMPAT

pytestmark = pytest.mark.gpu


def test_apex_trainer_loop_shape(dev, orc):
    sys.path.insert(0, COMPAT)
    try:
        import perwez
        import reth_buffer
        from reth.presets.config import get_solver, get_trainer
    finally:
        sys.path.remove(COMPAT)
    config = yaml.safe_load(APEX_CONFIG)
    config["replay_buffer"]["capacity"] = 4 * 1200
    K, B = 4, config["common"]["batch_size"]
    perwez_proc, perwez_config = perwez.start_server(port=None)
    rb_procs, rb_addrs = [], []
    for port in [0] * K:  # trainer.py:52-61 (port 0: an unused one each; the shards serve ZMTP on it)
        proc, addr = reth_buffer.start_per(capacity=config["replay_buffer"]["capacity"] // K,
                                           alpha=config["replay_buffer"]["alpha"], beta=config["replay_buffer"]["beta"],
                                           batch_size=B, port=port)
        assert addr.startswith("tcp://")
        rb_procs.append(proc)
        rb_addrs.append(addr)
    # worker.py:44-60-shaped appends: 64-row batches of float32 frames, |td| from calc_loss
    rng = np.random.default_rng(0)
    pool = rng.integers(0, 256, (96, 4, 84, 84), dtype=np.uint8)
    for addr in rb_addrs:
        client = reth_buffer.Client(addr)
        for _ in range(17):  # 1,088 rows >= sample_start (1,000)
            pick = rng.integers(0, 96, (2, 64))
            data = [pool[pick[0]].astype("f4"), rng.integers(0, 9, 64).astype("i8"),
                    rng.choice([-1.0, 0.0, 1.0], 64, p=[0.01, 0.98, 0.01]).astype("f4"), pool[pick[1]].astype("f4"),
                    (rng.random(64) < 1 / 2000).astype("f4")]
            client.append(data, rng.random(64).astype("f4"), compress=True)
    # ---------------------------------------------------- trainer_main (trainer.py:19-41)
    weights_send = perwez.SendSocket(perwez_config["url"], "weights", broadcast=True)
    weight_recv = perwez.RecvSocket(perwez_config["url"], "weights", broadcast=True)  # a worker's view
    rb_clients = [reth_buffer.Client(addr) for addr in rb_addrs]
    rb_loaders = [reth_buffer.TorchCudaLoader(addr, buffer_size=4, num_procs=2) for addr in rb_addrs]
    trainer = get_trainer(config)
    send_weights_interval = config["common"]["send_weights_interval"]
    last, sent = {}, None
    ts = 0
    while ts < 24:
        ts += 1
        idx = ts % len(rb_clients)
        data, indices, weights = rb_loaders[idx].sample()
        loss = trainer.step(data, weights=weights)
        rb_clients[idx].update_priorities(np.asarray(indices), np.asarray(loss))
        last[idx] = (np.asarray(indices).copy(), np.asarray(loss).copy())
        if ts % send_weights_interval == 0:
            stream = io.BytesIO()
            trainer.save_weights(stream)
            weights_send.send(stream.getbuffer())
            sent = {k: v.detach().cpu().clone() for k, v in trainer.solver.q_network.state_dict().items()}
    torch.cuda.synchronize()
    # ---------------------------------------------------- checks
    assert trainer.cur_step == 24
    for k, proc in enumerate(rb_procs):
        rep = proc.replay
        size, tail, cnt, calls, steps = rep.info()
        assert steps == 6 and size == 1088  # 24 updates round-robin over 4 shards
        ind, td = last[k]
        assert ind.shape == (B,) and td.shape == (B,) and np.isfinite(td).all()
        want = {}
        for i, w in zip(ind, orc.per_normalize(td.astype(np.float32), 0.5)):
            want[int(i)] = float(w)  # duplicate indices: the last writer wins (sumtree.py:61-79)
        _, _, val = rep.tree.export()
        val = val.cpu().numpy()
        assert all(val[i] == w for i, w in want.items())
    # the worker's side: two sends (ts 10, 20), one delivery of the newest
    assert not weight_recv.empty()
    worker_solver = get_solver(config, device="cpu")
    worker_solver.load_weights(io.BytesIO(weight_recv.recv()))
    assert weight_recv.empty()
    got = worker_solver.q_network.state_dict()
    assert all(torch.equal(got[k], sent[k]) for k in sent)
    for p in rb_procs:
        p.terminate()
        p.join()
    perwez_proc.terminate()
