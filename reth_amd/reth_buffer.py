"""Drop-in replacement for the `reth_buffer` client API, backed by an HBM replay shard.

Reference API kept (paths in the sosp2021/Reth checkout):
    start_server / start_per            reth_buffer/reth_buffer/__init__.py:11-49
    Client.append / update_priorities   reth_buffer/reth_buffer/client/client.py:21-39
    NumpyLoader.sample                  reth_buffer/reth_buffer/client/numpy_loader.py:27-51
    TorchCudaLoader.sample / iteration  reth_buffer/reth_buffer/client/torch_cuda_loader.py:69-163

What changes underneath: the service processes (ZMQ append/sampler loops, LMDB in /dev/shm,
CUDA-IPC loader processes) become one replay object resident in the GPU's HBM, owned by the
process that drives that GPU (one process per GPU).  `start_*` returns a handle standing in
for the service Process (terminate/join/is_alive) and an address string ("hbm://dev/id")
that Client and the loaders resolve in-process; with host / port the service also serves
the reference's ZeroMQ sockets (reth_amd.zmtp) so remote workers' Clients reach it.

Blocking: as in the reference, a loader asked for a batch before the sampler is ready
(`cnt >= max(sample_start, batch_size)` and `ready_sample`, sampler_loop.py:23-28) waits
(torch_cuda_loader.py:94-107,152-163; numpy_loader.py:27-51): the wait drains the remote
ingest queue as messages arrive until the shard is ready, forever by default or up to the
loader's `timeout` seconds (TimeoutError).  A shard with no remote ingest (started without
host / port) can only be filled by the calling thread itself, so there the wait raises
RuntimeError at once instead of hanging.  Differences, by design:
  * num_sampler_procs / num_procs / compress are accepted and ignored;
  * a loader can be built before any row exists (its slots are allocated by the first
    sample; the reference allocates them in __init__, blocking for a first batch to learn
    the row shapes);
  * TorchCudaLoader keeps the reference's sample-ahead: batch k+1 is drawn as soon as batch
    k is handed out, i.e. before k's priority update lands (the sampler's HWM-1 PUSH).
"""
import itertools
import queue
import sys
import time

import numpy as np
import torch

from .replay import Column, HbmReplay, _device, as_device

_SERVICES = {}
_ids = itertools.count()

_NP_TO_TORCH = {np.dtype("uint8"): torch.uint8, np.dtype("int32"): torch.int32, np.dtype("int64"): torch.int64,
                np.dtype("float32"): torch.float32, np.dtype("float64"): torch.float64}


class ReplayService:
    """Stands in for the service Process returned by the reference's start_server."""

    def __init__(self, capacity, batch_size, sampler, device, seed, widen_u8, kind="per"):
        self.capacity, self.batch_size = int(capacity), int(batch_size)
        self.kind = kind
        self.alpha = sampler.get("kwargs", {}).get("alpha", 0.6)
        self.beta = sampler.get("kwargs", {}).get("beta", 0.4)
        # main_loop.py:144-145: sample_start = max(sample_start, batch_size)
        self.sample_start = max(int(sampler.get("sample_start", 1000)), self.batch_size)
        self.device = _device(device)
        self.seed = seed
        self.widen_u8 = widen_u8
        self.replay = None  # created on the first append (the LMDB map is sized from it too)
        self.alive = True

    # ------------------------------------------------------------------ remote ingest (ZMTP)
    def listen(self, host, port, advertise=None, hwm=10, max_msg_size=None):
        """serve the reference's three service sockets over TCP (reth_amd.zmtp): the meta REP
        at tcp://host:port answering the JSON config (main_loop.py:64-76,162-170), the append
        PULL (main_loop.py:21-26) and the update PULL (update_proxy_loop, :79-88).  Received
        messages wait in one arrival-ordered queue of `hwm` entries (ZMQ_DEFAULT_HWM = 10,
        utils/__init__.py:12: a full queue stops the readers, and TCP stops the senders) until
        the owner thread drains them into the HBM replay (drain(): every ready() call, i.e.
        before every sample, and wait_ready() as they arrive while a loader waits).  Returns the meta address."""
        import json
        import queue

        from . import zmtp

        self.inbox = queue.Queue(maxsize=int(hwm))
        adv = advertise or (host if host not in ("0.0.0.0", "") else "127.0.0.1")
        mx = dict(max_msg_size=max_msg_size)  # per-message cap on the unauthenticated sockets
        self.append_ep = zmtp.Endpoint(b"PULL", lambda f: self.inbox.put(("append", f)), host, **mx)
        self.update_ep = zmtp.Endpoint(b"PULL", lambda f: self.inbox.put(("update", f)), host, **mx)
        reply = []
        self.meta_ep = zmtp.Endpoint(b"REP", lambda frames: reply, host, port, **mx)  # port 0: an unused one
        meta_addr = self.meta_ep.addr(adv)
        self.config = {"capacity": self.capacity, "batch_size": self.batch_size, "lmdb_path": None,
                       "meta_addr": meta_addr, "append_addr": self.append_ep.addr(adv),
                       "update_addr": self.update_ep.addr(adv),
                       "sampler_info": {"default": {"topic": "default", "sampler_cls": {
                           "per": "PERSampler", "uniform": "UniformSampler", "fifo": "FIFOSampler"}[self.kind],
                           "num_procs": 1, "kwargs": {"alpha": self.alpha, "beta": self.beta,
                                                      "capacity": self.capacity},
                           "addrs": [], "sample_start": self.sample_start, "batch_size": self.batch_size}}}
        reply.append(json.dumps(self.config).encode())
        return meta_addr

    def drain(self):
        """apply the queued remote messages in arrival order on the calling (owner) thread:
        an append message is append_loop's work (server/main_loop.py:40-58) on the HBM shard,
        an update message [indices, weights, step] is the sampler's update (sampler_loop.py:32-35).
        Returns the number of messages taken off the queue."""
        q = getattr(self, "inbox", None)
        n = 0
        while q is not None:
            try:
                item = q.get_nowait()
            except queue.Empty:
                break
            self._apply(item)
            n += 1
        return n

    def _apply(self, item):
        """one remote message; a message that does not deserialize or does not fit the shard
        is dropped and recorded in `ingest_errors` (the remote sender is unauthenticated: a
        bad message must not take the owner's loop down)"""
        kind, frames = item
        try:
            msg = b"".join(bytes(f) for f in frames) if len(frames) > 1 else frames[0]
            if kind == "append":
                Client(self).append_message(msg)
            else:
                from . import pack

                idx, w, step = pack.deserialize(msg)
                Client(self).update_priorities(np.asarray(idx), np.asarray(w), step=bool(step))
        except Exception as e:
            if not hasattr(self, "ingest_errors"):
                self.ingest_errors = []
            self.ingest_errors.append(f"{kind}: {type(e).__name__}: {e}")
            print(f"reth_buffer: dropped a malformed remote {kind} message ({type(e).__name__}: {e})",
                  file=sys.stderr)

    def wait_ready(self, timeout=None, poll=0.05):
        """block until the sampler can serve a batch (sampler_loop.py:23-28), applying remote
        messages as they arrive; `timeout` seconds (None: forever, as the reference) ->
        TimeoutError.  Without remote ingest nothing but the caller could fill the shard, so
        an unready shard raises RuntimeError at once."""
        if self.ready():
            return
        q = getattr(self, "inbox", None)
        if q is None:
            cnt = 0 if self.replay is None else self.replay.cnt
            raise RuntimeError(f"replay not ready: cnt={cnt} < sample_start={self.sample_start}, and the shard has "
                               "no remote ingest (start it with host/port) -- nothing else could fill it")
        deadline = None if timeout is None else time.monotonic() + float(timeout)
        while True:
            if not self.alive:
                raise RuntimeError("replay service terminated while a loader was waiting")
            wait = poll if deadline is None else min(poll, deadline - time.monotonic())
            if wait <= 0:
                cnt = 0 if self.replay is None else self.replay.cnt
                raise TimeoutError(f"replay not ready after {timeout} s: cnt={cnt} < sample_start={self.sample_start}")
            try:
                item = q.get(timeout=wait)
            except queue.Empty:
                continue
            self._apply(item)
            if self.ready():
                return

    def _widen(self, c):
        return self.widen_u8 is True or (isinstance(self.widen_u8, (set, list, tuple)) and c in self.widen_u8)

    def ensure(self, cols, row_shapes=None):
        """create the shard from the first append's columns.  widen_u8 (True or a set of
        column numbers): uint8 columns -- and float32 frame columns of a wire-format
        message -- are stored as bytes and sampled as float32."""
        if self.replay is None:
            columns = []
            for k, c in enumerate(cols):
                dt = c.dtype if torch.is_tensor(c) else _NP_TO_TORCH.get(np.asarray(c).dtype)
                if dt is None:
                    raise TypeError(f"unsupported column dtype {np.asarray(c).dtype}")
                shape = tuple(c.shape[1:]) if row_shapes is None else tuple(row_shapes[k])
                if dt == torch.float32 and row_shapes is not None and self._widen(k):
                    columns.append(Column(shape, torch.uint8, torch.float32))
                    continue
                widen = dt == torch.uint8 and self._widen(k)
                columns.append(Column(shape, dt, torch.float32 if widen else None))
            self.replay = HbmReplay(self.capacity, columns, self.alpha, self.beta, self.device, self.seed,
                                    sampler=self.kind)
        return self.replay

    def ready(self):
        """sampler_loop.py:23-28: cnt >= sample_start and sampler.ready_sample(batch_size)"""
        self.drain()
        return (self.replay is not None and self.replay.cnt >= self.sample_start
                and self.replay.ready_sample(self.batch_size))

    def weights_out(self, w):
        """the sampler's weight column: IS weights (PER, f64), ones as int64 (UniformSampler
        returns np.ones(batch, "i8")), or the pushed weights (FIFO, f64)"""
        return w.to(torch.int64) if self.kind == "uniform" else w

    def check_ready(self):
        """non-blocking: raise RuntimeError unless a batch can be drawn now"""
        if not self.ready():
            cnt = 0 if self.replay is None else self.replay.cnt
            raise RuntimeError(f"replay not ready: cnt={cnt} < sample_start={self.sample_start}")

    # Process-like surface used by the reference's launch scripts
    def terminate(self):
        self.alive = False
        self.replay = None
        for ep in ("meta_ep", "append_ep", "update_ep"):
            if getattr(self, ep, None) is not None:
                getattr(self, ep).close()
                setattr(self, ep, None)

    def join(self, timeout=None):
        return None

    def is_alive(self):
        return self.alive


def _lookup(addr):
    try:
        return _SERVICES[addr]
    except KeyError:
        raise ValueError(f"unknown replay address {addr!r} (services live in the process that started them)")


def start_server(capacity, batch_size, host=None, port=None, samplers=None, cache_policy=None, *,
                 device=None, seed=0, widen_u8=False):
    """reth_buffer.start_server (__init__.py:11-27) -> (service, address)."""
    if cache_policy is not None and type(cache_policy).__name__ != "FIFOPolicy":
        raise NotImplementedError("only the FIFO cache policy is implemented (fifo_policy.py)")
    if samplers is None:
        samplers = [{"sampler_cls": "PERSampler", "num_procs": 1, "sample_start": 1000}]
    if len(samplers) != 1:
        raise NotImplementedError("one sampler topic per shard")
    s = samplers[0]
    name = s["sampler_cls"] if isinstance(s["sampler_cls"], str) else s["sampler_cls"].__name__
    kinds = {"PERSampler": "per", "UniformSampler": "uniform", "FIFOSampler": "fifo"}
    if name not in kinds:
        raise NotImplementedError(f"sampler {name} (PERSampler, UniformSampler, FIFOSampler are implemented)")
    svc = ReplayService(capacity, batch_size, s, device, seed, widen_u8, kind=kinds[name])
    addr = f"hbm://{svc.device.index}/{next(_ids)}"
    _SERVICES[addr] = svc
    svc.hbm_addr = addr
    if host is not None or port is not None:
        # the reference's network-facing service (__init__.py:14-17): remote Clients reach this
        # shard over ZMTP; in-process Clients / loaders resolve the same tcp address
        addr = svc.listen("0.0.0.0" if host is None else host, 0 if port is None else port)
        _SERVICES[addr] = svc
    return svc, addr


def start_per(capacity, batch_size, alpha=0.6, beta=0.4, sample_start=1000, num_sampler_procs=1, host=None,
              port=None, cache_policy=None, *, device=None, seed=0, widen_u8=False):
    """reth_buffer.start_per (__init__.py:30-49) -> (service, address)."""
    samplers = [{"sampler_cls": "PERSampler", "num_procs": num_sampler_procs, "sample_start": sample_start,
                 "kwargs": {"alpha": alpha, "beta": beta}}]
    return start_server(capacity, batch_size, host, port, samplers, cache_policy, device=device, seed=seed,
                        widen_u8=widen_u8)


class Client:
    """client/client.py:8-39."""

    def __init__(self, meta_addr):
        self.remote = None
        if isinstance(meta_addr, ReplayService):
            self.svc = meta_addr
        elif meta_addr in _SERVICES or not str(meta_addr).startswith("tcp://"):
            self.svc = _lookup(meta_addr)
        else:  # a service in another process / on another node: the reference's wire path
            self.svc = None
            self.remote = _RemoteClient(meta_addr)

    def append(self, data, weights, compress=False):
        if self.remote is not None:
            return self.remote.append(data, weights, compress)
        assert isinstance(data, (list, tuple))
        n = len(weights)
        for col in data:
            assert isinstance(col, np.ndarray) or torch.is_tensor(col)
            assert len(col) == n
        rep = self.svc.ensure(data)
        dev = rep.device
        cols = [as_device(c, col.dtype, dev) for c, col in zip(data, rep.columns)]
        rep.append(cols, weights)

    def append_message(self, message):
        """append_loop (server/main_loop.py:21-61) for one wire-format message as
        Client.append sends it (utils/pack.py): the rows go from the message body to HBM
        through one host->device copy (reth_amd/pack.py)"""
        from . import pack

        if self.svc.replay is None:
            rows, _ = pack.deserialize(message)
            first = pack.deserialize(rows[0])
            self.svc.ensure([np.asarray(x)[None] for x in first], row_shapes=[np.shape(x) for x in first])
        return pack.ingest_append(self.svc.replay, message)

    def update_priorities(self, indices, weights, step=True):
        assert len(indices) == len(weights)
        if self.remote is not None:
            return self.remote.update_priorities(indices, weights, step)
        if self.svc.replay is None:
            raise RuntimeError("update_priorities before any append")
        self.svc.replay.update_priorities(indices, weights, step=step)


class _RemoteClient:
    """client/client.py:8-39 over ZMTP (reth_amd.zmtp): REQ the meta address for the config
    (utils/__init__.py:51-59), PUSH appends / priority updates to its append / update
    addresses, the message bytes identical to the reference's (reth_amd.pack)"""

    def __init__(self, meta_addr):
        import json

        from . import zmtp

        req = zmtp.Peer(b"REQ", meta_addr)
        try:
            self.meta = json.loads(bytes(req.request(b"")[0]))
        finally:
            req.close()
        self.append_sock = zmtp.Peer(b"PUSH", self.meta["append_addr"])
        self.update_sock = zmtp.Peer(b"PUSH", self.meta["update_addr"])

    def append(self, data, weights, compress=False):
        from . import pack

        assert isinstance(data, (list, tuple))
        for col in data:
            assert isinstance(col, np.ndarray)
            assert len(col) == len(weights)
        rows = [pack.serialize([col[i, ...] for col in data]) for i in range(len(weights))]
        self.append_sock.send(pack.serialize([rows, weights], compress=compress))

    def update_priorities(self, indices, weights, step=True):
        from . import pack

        self.update_sock.send(pack.serialize([indices, weights, step]))


class NumpyLoader:
    """client/numpy_loader.py:8-56: (list of np columns, np.int64 indices, np.float64 weights)."""

    def __init__(self, meta_addr, topic="default", timeout=None):
        self.svc = _lookup(meta_addr)
        self.timeout = timeout  # seconds a sample() waits for the sampler (None: forever)

    def __iter__(self):
        return self

    def __next__(self):
        return self.sample()

    def sample(self):
        self.svc.wait_ready(self.timeout)
        cols, idx, isw = self.svc.replay.sample(self.svc.batch_size)
        return [c.cpu().numpy() for c in cols], idx.cpu().numpy(), self.svc.weights_out(isw).cpu().numpy()


class TorchCudaLoader:
    """client/torch_cuda_loader.py:69-163: a ring of `buffer_size` pre-allocated device slots;
    sample() returns views into one slot, valid until the next call (the reference recycles a
    slot on the next sample(), :153-155).  sample() waits until the sampler can serve a
    batch (up to `timeout` seconds; None: forever, as the reference's res_queue.get())."""

    def __init__(self, meta_addr, topic="default", buffer_size=8, num_procs=6, prefetch=1, timeout=None):
        self.svc = _lookup(meta_addr)
        self.timeout = timeout
        self.prefetch = int(prefetch)
        self.buffer_size = max(self.prefetch + 1, int(buffer_size))
        self._slots = None
        self._next = 0
        self._pending = []  # slot ids already sampled, oldest first
        self.gather_timer = None  # bench hook: events around the gather launch

    def pending(self):
        return len(self._pending)

    def take(self):
        """the oldest already-sampled batch (no replay operation is enqueued)"""
        k = self._pending.pop(0)
        return self._slots[k]

    def issue(self):
        """enqueue the PER sample + gather of the next batch into a free slot"""
        self.svc.wait_ready(self.timeout)
        self._issue()

    def _issue(self):
        rep = self.svc.replay
        if self._slots is None:
            self._slots = [rep.new_batch(self.svc.batch_size) for _ in range(self.buffer_size)]
        k = self._next
        self._next = (self._next + 1) % self.buffer_size
        cols, idx, isw = self._slots[k]
        rep.sample_into(self.svc.batch_size, cols, idx, isw, gather_timer=self.gather_timer)
        self._pending.append(k)

    def sample_device(self):
        """(data, device int64 indices, device f64 weights) without any host sync (once the
        sampler is ready; before that it waits, draining the remote ingest)."""
        if not self._pending:
            self.svc.wait_ready(self.timeout)
            self._issue()
        k = self._pending.pop(0)
        # sample-ahead: batch k+1 is drawn before batch k's priority update is enqueued (when
        # the sampler can serve it now; a FIFO sampler may have to wait for more rows)
        while len(self._pending) < self.prefetch and self.svc.ready():
            self._issue()
        cols, idx, isw = self._slots[k]
        return cols, idx, self.svc.weights_out(isw)

    def sample(self):
        cols, idx, isw = self.sample_device()
        return cols, idx.cpu().numpy(), isw

    def __iter__(self):
        return self

    def __next__(self):
        return self.sample()

    def close(self):
        self._slots = None
