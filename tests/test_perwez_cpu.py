"""The in-process perwez facade: broadcast = conflated latest-wins per subscriber, late
subscribers miss older messages, PUSH/PULL = FIFO with a high-water mark, recv on nothing
raises TimeoutError (perwez/perwez/client/socket.py:19-122, 295-330)."""
import io

import pytest
import torch

from reth_amd import perwez


def test_broadcast_conflates_to_the_newest():
    proc, cfg = perwez.start_server()
    tx = perwez.SendSocket(cfg["url"], "weights", broadcast=True)
    rx = perwez.RecvSocket(cfg["url"], "weights", broadcast=True)
    assert rx.empty()
    for k in range(3):
        tx.send(memoryview(bytes([k]) * 4))
    assert not rx.empty()
    assert rx.recv() == bytes([2]) * 4  # several publishes before one receive: the last one
    assert rx.empty()
    with pytest.raises(TimeoutError):
        rx.recv()
    late = perwez.RecvSocket(cfg["url"], "weights", broadcast=True)
    assert late.empty()  # joined after the last send
    tx.send(b"x")
    assert rx.recv() == b"x" and late.recv() == b"x"
    proc.terminate()
    assert not proc.is_alive()


def test_push_pull_fifo_and_hwm():
    _, cfg = perwez.start_server()
    tx = perwez.SendSocket(cfg["url"], "q", broadcast=False, hwm=2)
    rx = perwez.RecvSocket(cfg["url"], "q", broadcast=False)
    tx.send(b"a")
    tx.send(b"b")
    assert tx.full()
    with pytest.raises(TimeoutError):
        tx.send(b"c")
    assert rx.recv() == b"a" and rx.recv() == b"b" and rx.empty()


def test_weights_stream_through_the_socket():
    """trainer.py:38-41 -> worker.py:37-41 with a torch.save stream"""
    _, cfg = perwez.start_server()
    tx = perwez.SendSocket(cfg["url"], "weights", broadcast=True)
    rx = perwez.RecvSocket(cfg["url"], "weights", broadcast=True)
    net = torch.nn.Linear(4, 2)
    stream = io.BytesIO()
    torch.save(net.state_dict(), stream)
    tx.send(stream.getbuffer())
    stream.close()  # the sender's buffer is gone; the message was copied
    got = torch.load(io.BytesIO(rx.recv()), weights_only=True)
    assert all(torch.equal(got[k], v) for k, v in net.state_dict().items())
