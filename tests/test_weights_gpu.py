"""The learner -> actor weights slot (rth_weights_publish / rth_weights_acquire): several
publishes before one acquire deliver the last (perwez CONFLATE, socket.py:302-328), the
device-side load decision follows worker.py:37-41 (newer version AND more than
recv_weights_interval steps since the previous load), and it replays from a captured graph
with no host decision."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _net(dev, seed):
    torch.manual_seed(seed)
    return torch.nn.Sequential(torch.nn.Linear(8, 16), torch.nn.ReLU(), torch.nn.Linear(16, 3)).to(dev)


def _same(a, b):
    return all(torch.equal(p, q) for p, q in zip(a.parameters(), b.parameters()))


def test_latest_wins(dev):
    from reth_amd.weights import WeightsSlot

    learner, actor = _net(dev, 0), _net(dev, 1)
    slot = WeightsSlot(learner)
    assert slot.device_version() == 0 and slot.version == 0  # the initial content is no message
    snaps = []
    for k in range(3):  # three publishes, no acquire in between
        with torch.no_grad():
            for p in learner.parameters():
                p.add_(1.0 + k)
        slot.publish(learner)
        snaps.append([p.clone() for p in learner.parameters()])
    with torch.no_grad():
        for p in learner.parameters():
            p.zero_()  # the learner moves on; the slot holds publish 3
    seen = torch.zeros((), dtype=torch.int64, device=dev)
    loaded = torch.full((), -1, dtype=torch.int32, device=dev)
    slot.acquire(actor, seen=seen, loaded=loaded)
    torch.cuda.synchronize()
    assert int(loaded) == 1 and int(seen) == 3 and slot.device_version() == 3 and slot.version == 3
    assert all(torch.equal(p, q) for p, q in zip(actor.parameters(), snaps[-1]))
    with torch.no_grad():
        for p in actor.parameters():
            p.fill_(7.0)
    slot.acquire(actor, seen=seen, loaded=loaded)  # nothing newer: no copy
    torch.cuda.synchronize()
    assert int(loaded) == 0 and all(bool((p == 7.0).all()) for p in actor.parameters())


def test_interval_gate_on_device(dev):
    from reth_amd.weights import WeightsSlot

    learner, actor = _net(dev, 2), _net(dev, 3)
    slot = WeightsSlot(learner)
    i64 = dict(dtype=torch.int64, device=dev)
    seen, step, prev = torch.zeros((), **i64), torch.zeros((), **i64), torch.zeros((), **i64)
    loaded = torch.zeros((), dtype=torch.int32, device=dev)
    slot.acquire(actor, seen=seen, loaded=loaded)  # the construction snapshot is not a message
    torch.cuda.synchronize()
    assert int(loaded) == 0 and not _same(actor, learner)
    slot.publish(learner)
    step.fill_(400)  # worker.py:38: strictly more than recv_weights_interval steps
    slot.acquire(actor, seen=seen, step=step, prev=prev, interval=400, loaded=loaded)
    torch.cuda.synchronize()
    assert int(loaded) == 0 and not _same(actor, learner)
    step.fill_(401)
    slot.acquire(actor, seen=seen, step=step, prev=prev, interval=400, loaded=loaded)
    torch.cuda.synchronize()
    assert int(loaded) == 1 and int(prev) == 401 and _same(actor, learner)
    slot.publish(learner)
    step.fill_(700)  # newer version, but only 299 steps since the load
    slot.acquire(actor, seen=seen, step=step, prev=prev, interval=400, loaded=loaded)
    torch.cuda.synchronize()
    assert int(loaded) == 0


def test_acquire_replays_from_a_graph(dev):
    """the captured acquire decides on every replay from the device counters"""
    from reth_amd.weights import WeightsSlot

    learner, actor = _net(dev, 4), _net(dev, 5)
    slot = WeightsSlot(learner)
    i64 = dict(dtype=torch.int64, device=dev)
    seen, step, prev = torch.zeros((), **i64), torch.zeros((), **i64), torch.zeros((), **i64)
    loaded = torch.zeros((), dtype=torch.int32, device=dev)
    s = torch.cuda.Stream(dev)
    s.wait_stream(torch.cuda.current_stream(dev))
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(s):
        with torch.cuda.graph(g, stream=s):
            step.add_(1)
            slot.acquire(actor, seen=seen, step=step, prev=prev, interval=2, loaded=loaded)
    torch.cuda.current_stream(dev).wait_stream(s)
    hist = []
    for k in range(8):
        if k == 5:
            with torch.no_grad():
                for p in learner.parameters():
                    p.mul_(-1.0)
            slot.publish(learner)
        g.replay()
        torch.cuda.synchronize()
        hist.append(int(loaded))
    # step 1, 2: gate closed (<= 2 since prev 0); step 3: the gate opens but nothing was
    # published (the construction snapshot is no message); step 6 (k=5): v1 published, 6 > 2
    # steps since prev 0 -> load; then nothing newer
    assert hist == [0, 0, 0, 0, 0, 1, 0, 0]
    assert _same(actor, learner)


def test_channels_last_dqn_network(dev):
    """the apex layout: channels_last conv weights are dense runs the slot copies as bytes; a
    consumer in another memory format is refused instead of receiving permuted weights"""
    from reth_amd.model import DQNNetwork
    from reth_amd.weights import WeightsSlot

    torch.manual_seed(0)
    cl = dict(memory_format=torch.channels_last)
    learner = DQNNetwork((4, 84, 84), 6).to(dev, **cl)
    actor = DQNNetwork((4, 84, 84), 6).to(dev, **cl)
    slot = WeightsSlot(learner)
    with torch.no_grad():
        for p in learner.parameters():
            p.add_(0.5)
    slot.publish(learner)
    slot.acquire(actor)
    torch.cuda.synchronize()
    assert _same(actor, learner)
    other = DQNNetwork((4, 84, 84), 6).to(dev)  # contiguous (NCHW) conv weights
    with pytest.raises(ValueError):
        slot.acquire(other)
