"""perwez's client surface for the apex scripts, in-process.

Reference: perwez/perwez/__init__.py:18-32 (start_server), perwez/perwez/client/socket.py:
19-122 (SendSocket / RecvSocket: PUB/SUB with CONFLATE for broadcast=True, PUSH/PULL with a
high-water mark otherwise), 295-330 (recv raises TimeoutError when nothing arrives).  The
apex scripts use it for one thing: the trainer's torch.save weight stream, broadcast to the
actors every send_weights_interval updates (test/apex-dqn/trainer.py:20,38-41; worker.py:
24,37-41, 65-70), where only the newest message matters.

Here the trainer and the actors of a GPU live in one process (one process per GPU), so the
"server" is a process-local hub keyed by (url, topic) and a message is handed over by
reference -- no ZeroMQ, no serialisation.  Semantics kept:
  * broadcast (SUB): every receiver sees only the newest message sent after it subscribed,
    once (conflate); empty() is True until a newer one is sent;
  * non-broadcast (PULL): a FIFO of at most `hwm` messages, each delivered to one receiver
    (a send into a full queue raises, where ZeroMQ would block);
  * recv() with nothing to deliver raises TimeoutError (nothing can arrive while a
    single-process caller blocks).
Device weights between learner and actors of one GPU go through reth_amd.weights (the C-ABI
slot, no bytes at all); this facade carries the reference's byte messages unchanged.
"""
import collections
import itertools
import threading

_HUBS = {}
_ids = itertools.count()
_lock = threading.Lock()


class _Topic:
    def __init__(self):
        self.seq = 0          # broadcast: sequence number of the newest message
        self.latest = None
        self.queue = collections.deque()


class _Hub:
    def __init__(self, url):
        self.url = url
        self.topics = collections.defaultdict(_Topic)


class _ServerHandle:
    """stands in for the server Process of start_server"""

    def __init__(self, url):
        self.url = url
        self._alive = True

    def is_alive(self):
        return self._alive

    def terminate(self):
        self._alive = False
        _HUBS.pop(self.url, None)

    def join(self, timeout=None):
        pass


def start_server(host="0.0.0.0", port=None):
    """-> (process handle, {"url": ...}) like perwez.start_server"""
    url = f"inproc://perwez/{next(_ids)}" if port is None else f"inproc://perwez/{host}:{port}"
    with _lock:
        _HUBS.setdefault(url, _Hub(url))
    return _ServerHandle(url), {"url": url}


def _hub(url):
    with _lock:
        hub = _HUBS.get(url)
        if hub is None:  # like a client connecting before the server answered: create it
            hub = _HUBS[url] = _Hub(url)
        return hub


def _payload(data):
    # a memoryview of the sender's buffer (trainer.py:41 sends stream.getbuffer()) is
    # copied: the sender may reuse or free that buffer right after send()
    return bytes(data) if isinstance(data, (memoryview, bytearray)) else data


class SendSocket:
    def __init__(self, server_url, topic, broadcast=None, sock_type=None, ctx=None, conflate=None, hwm=5,
                 public=True):
        if sock_type is None:
            assert broadcast is not None, "broadcast or sock_type should be specified"
            sock_type = "pub" if broadcast else "push"
        self.broadcast = sock_type in ("pub", 1)
        self.hwm = int(hwm)
        self.topic = _hub(server_url).topics[topic]

    def close(self, linger=0):
        pass

    def poll(self, timeout=None):
        return 0 if (not self.broadcast and len(self.topic.queue) >= self.hwm) else 1

    def full(self):
        return self.poll(0) == 0

    def send(self, data, timeout=None, compress=False):
        t = self.topic
        if self.broadcast:
            t.latest = _payload(data)
            t.seq += 1
        else:
            if len(t.queue) >= self.hwm:
                raise TimeoutError("perwez send: queue full (hwm reached)")
            t.queue.append(_payload(data))


class RecvSocket:
    def __init__(self, server_url, topic, broadcast=None, sock_type=None, ctx=None, conflate=None, hwm=5,
                 public=False):
        if sock_type is None:
            assert broadcast is not None, "broadcast or sock_type should be specified"
            sock_type = "sub" if broadcast else "pull"
        self.broadcast = sock_type in ("sub", 2)
        self.topic = _hub(server_url).topics[topic]
        self._seen = self.topic.seq  # a subscriber only sees messages sent after it joined

    def close(self, linger=0):
        pass

    def poll(self, timeout=None):
        t = self.topic
        return int(t.seq > self._seen) if self.broadcast else int(len(t.queue) > 0)

    def empty(self):
        return self.poll(0) == 0

    def recv(self, timeout=None):
        if self.poll(timeout) == 0:
            raise TimeoutError("perwez recv timeout (in-process hub: no message waiting)")
        t = self.topic
        if self.broadcast:
            self._seen = t.seq
            return t.latest
        return t.queue.popleft()
