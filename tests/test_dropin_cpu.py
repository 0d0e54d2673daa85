"""The reference's apex scripts against reth_amd through the import-compatible names of
reth_amd/compat (PYTHONPATH): the host pieces of test/apex-dqn/worker.py -- perwez weights
broadcast, get_solver(device="cpu") / get_worker, reth.buffer.NumpyBuffer (host), the host
NStepAdder -- with no GPU.  The trainer side (TorchCudaLoader, HBM shards) is
tests/test_dropin_gpu.py."""
import io
import os
import sys

import numpy as np
import pytest
import torch
import yaml

COMPAT = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "reth_amd", "compat")

# test/apex-dqn/config.yaml, restated (the reference's values)
APEX_CONFIG = """
common:
  batch_size: 512
  rollout_batch_size: 64
  num_workers: 16
  send_weights_interval: 10
  recv_weights_interval: 400
env:
  name: BeamRiderNoFrameskip-v4
solver:
  name: 'dqn'
  clip_value: 40
  double_q: True
  dueling: True
  gamma: 0.99
  learning_rate: 0.0001
  adam_epsilon: .00015
  update_target_interval: 100
  n_step: 3
worker:
  exploration: 0
  print_interval: 10000
trainer:
  print_interval: 1000
replay_buffer:
  prioritized: True
  alpha: 0.5
  beta: 0.4,1,2000000
  capacity: 1000000
"""


@pytest.fixture
def compat():
    sys.path.insert(0, COMPAT)
    try:
        yield
    finally:
        sys.path.remove(COMPAT)


def test_compat_names_resolve_to_reth_amd(compat):
    import perwez
    import reth_buffer
    from reth.buffer import NumpyBuffer, PrioritizedBuffer
    from reth.presets.config import get_replay_buffer, get_solver, get_trainer, get_worker
    from reth.utils import NStepAdder, getLogger

    import reth_amd.buffer
    import reth_amd.perwez
    import reth_amd.presets
    import reth_amd.reth_buffer

    assert perwez.SendSocket is reth_amd.perwez.SendSocket and perwez.start_server is reth_amd.perwez.start_server
    assert reth_buffer.TorchCudaLoader is reth_amd.reth_buffer.TorchCudaLoader
    assert reth_buffer.start_per is reth_amd.reth_buffer.start_per and reth_buffer.Client is reth_amd.reth_buffer.Client
    assert get_trainer is reth_amd.presets.get_trainer and get_worker is reth_amd.presets.get_worker
    assert get_solver is reth_amd.presets.get_solver and get_replay_buffer is reth_amd.presets.get_replay_buffer
    assert PrioritizedBuffer is reth_amd.buffer.PrioritizedBuffer
    assert type(NumpyBuffer(8, circular=False)).__name__ == "HostNumpyBuffer"  # worker.py:35: a host batch
    assert NStepAdder(0.99, 3).step == 3 and getLogger("x") is not None


def test_host_nstep_adder_matches_golden_nep50(golden):
    """mode 1 (numpy >= 2) bit-exact against the reference NStepAdder's recorded streams, the
    rows pushed as worker.py:47-52 does (0-d arrays)"""
    from reth_amd.nstep import NStepAdder

    g = golden("nstep.npz")
    tags = sorted({k.rsplit("/", 1)[0] for k in g.keys() if k.count("/") == 2})
    for tag in tags:
        ad = NStepAdder(0.99, int(tag.split("/")[0][1:]), mode=1)
        rows = []
        for t, (a, r, d) in enumerate(zip(g[f"{tag}/actions"], g[f"{tag}/rewards"], g[f"{tag}/dones"])):
            row = ad.push(np.asarray(t, "f4"), np.asarray(a, "i8"), np.asarray(r, "f4"), np.asarray(t + 1000, "f4"),
                          np.asarray(d, "f4"))
            if row is not None:
                rows.append((t, row))
        assert [t for t, _ in rows] == list(g[f"{tag}/emit_t"]), tag
        for k, (_, row) in enumerate(rows):
            assert float(row[0]) == g[f"{tag}/emit_s0"][k] and int(row[1]) == g[f"{tag}/emit_a"][k]
            assert float(row[3]) - 1000 == g[f"{tag}/emit_s1"][k] and float(row[4]) == g[f"{tag}/emit_done"][k]
            assert np.float32(row[2]).tobytes() == g[f"{tag}/emit_r"][k].tobytes(), (tag, k)


@pytest.mark.parametrize("n", [1, 3, 5])
def test_host_nstep_adder_legacy_mode_matches_oracle(orc, n):
    """mode 0 (numpy 1.19 promotion, the reference's pin) against the oracle's restatement"""
    from reth_amd.nstep import NStepAdder

    rng = np.random.default_rng(n)
    ad, od = NStepAdder(0.99, n, mode=0), orc.NStep(n, 0.99, mode=0)
    for t in range(400):
        r = np.float32(rng.choice([-1.0, 1.0, 0.0, rng.random()]))
        d = np.float32(rng.random() < 0.07)
        row = ad.push(np.asarray(t, "i8"), np.asarray(t % 6, "i8"), np.asarray(r, "f4"), np.asarray(t + 1, "i8"),
                      np.asarray(d, "f4"))
        orow = od.push(t, t % 6, r, t + 1, d)
        assert (row is None) == (orow is None)
        if row is not None:
            assert (int(row[0]), int(row[1]), int(row[3])) == (orow[0], orow[1], orow[3])
            assert np.float32(row[2]).tobytes() == np.float32(orow[2]).tobytes() and float(row[4]) == orow[4]


def test_apex_worker_host_loop(compat):
    """test/apex-dqn/worker.py:21-61's loop body on the host (the replay append itself is the
    GPU test's): CPU solver + worker from the YAML factories, weights through perwez's
    broadcast with the recv interval, n-step rows staged in a 64-row host NumpyBuffer and
    scored by calc_loss"""
    import perwez
    from reth.buffer import NumpyBuffer
    from reth.presets.config import get_solver, get_worker
    from reth.utils import NStepAdder, getLogger

    config = yaml.safe_load(APEX_CONFIG)
    config["common"]["recv_weights_interval"] = 20  # reach a reload in a short test
    _, pz = perwez.start_server()
    weight_recv = perwez.RecvSocket(pz["url"], "local-weights", broadcast=True)
    weight_send = perwez.SendSocket(pz["url"], "local-weights", broadcast=True)
    idx, size = 3, 16
    batch_size = config["common"]["rollout_batch_size"]
    eps = 0.4 ** (1 + (idx / (size - 1)) * 7)
    solver = get_solver(config, device="cpu")
    worker = get_worker(config, exploration=eps, solver=solver, logger=getLogger(f"worker{idx}"))
    assert worker.env.observation_space.shape == (4, 84, 84) and worker.env.action_space.n == 9
    # the learner's weights: another CPU solver's torch.save stream, sent twice (conflate)
    torch.manual_seed(123)
    learner = get_solver(config, device="cpu")
    for _ in range(2):
        stream = io.BytesIO()
        learner.save_weights(stream)
        weight_send.send(stream.getbuffer())
    recv_weights_interval = config["common"]["recv_weights_interval"]
    prev_load, loads, appended = 0, 0, []
    adder = NStepAdder(config["solver"]["gamma"], config["solver"]["n_step"])
    buffer = NumpyBuffer(batch_size, circular=False)
    while len(appended) < 2:
        if (worker.cur_step - prev_load) > recv_weights_interval and not weight_recv.empty():
            worker.load_weights(io.BytesIO(weight_recv.recv()))
            prev_load = worker.cur_step
            loads += 1
        s0, a, r, s1, done = worker.step()
        row = adder.push(np.asarray(s0, dtype="f4"), np.asarray(a, dtype="i8"), np.asarray(r, dtype="f4"),
                         np.asarray(s1, dtype="f4"), np.asarray(done, dtype="f4"))
        if row is None:
            continue
        buffer.append(row)
        if buffer.size == buffer.capacity:
            loss = np.asarray(worker.solver.calc_loss(buffer.data), dtype="f4")
            appended.append(([np.array(c) for c in buffer.data], loss))
            buffer.clear()
    assert loads == 1 and weight_recv.empty()  # two sends, one delivery (latest wins)
    for p, q in zip(solver.q_network.parameters(), learner.q_network.parameters()):
        assert torch.equal(p, q)
    for data, loss in appended:
        assert [c.shape for c in data] == [(64, 4, 84, 84), (64,), (64,), (64, 4, 84, 84), (64,)]
        assert [c.dtype.name for c in data] == ["float32", "int64", "float32", "float32", "float32"]
        assert loss.shape == (64,) and np.isfinite(loss).all() and (loss >= 0).all()
