"""HBM-resident sum-tree, PER sampler and replay shard (host side of libreth_hip.so).

    SumTree     <- reth_buffer/reth_buffer/utils/sumtree.py:82-113     (NumbaSumTree)
    PERSampler  <- reth_buffer/reth_buffer/sampler/per_sampler.py:5-35
    HbmReplay   <- the reth_buffer service: append_loop (server/main_loop.py:21-61),
                   FIFOPolicy (cache_policy/fifo_policy.py:11-18), sampler_loop
                   (server/sampler_loop.py:6-42) and the loaders' gather
                   (client/torch_cuda_loader.py:20-66, numpy_loader.py:27-51)

Everything runs on the device through the C ABI; results stay in HBM unless a caller asks
for host copies (the numpy-facing reth_buffer API does).  Argument checking mirrors the
reference's asserts and raises on the host.
"""
import ctypes

import numpy as np
import torch

from . import _lib
from ._lib import ColDesc, Src, c_i64, c_vp, call, ptr, stream_ptr
from .schedule import Schedule

_TORCH_TO_RTH = {torch.uint8: _lib.RTH_U8, torch.int32: _lib.RTH_I32, torch.int64: _lib.RTH_I64,
                 torch.float32: _lib.RTH_F32, torch.float64: _lib.RTH_F64}
_RTH_TO_TORCH = {v: k for k, v in _TORCH_TO_RTH.items()}
_TORCH_TO_RTH[torch.bool] = _lib.RTH_U8  # bool columns (gym's `done`) are stored as bytes


def _device(device):
    dev = torch.device(device if device is not None else "cuda")
    if dev.type != "cuda":
        raise ValueError(f"reth_amd runs on the GPU only (got device {dev})")
    return torch.device("cuda", dev.index if dev.index is not None else torch.cuda.current_device())


def as_device(x, dtype, device):
    """numpy / list / tensor -> contiguous device tensor of `dtype` (no copy if already so)."""
    if torch.is_tensor(x):
        return x.to(device=device, dtype=dtype, non_blocking=True).contiguous()
    return torch.as_tensor(np.asarray(x), dtype=dtype).to(device, non_blocking=True).contiguous()


def _prio_tensor(w, device, raw=False):
    """priorities keep their precision class: float64 inputs are normalised in f64 (numpy
    on an f8 array), everything else in f32 (the apex path's `np.asarray(loss, "f4")`);
    raw: float64 priorities stored without normalisation."""
    if raw:
        return as_device(w, torch.float64, device), _lib.RTH_PRIO_RAW
    is64 = (torch.is_tensor(w) and w.dtype == torch.float64) or (
        not torch.is_tensor(w) and np.asarray(w).dtype == np.float64)
    t = as_device(w, torch.float64 if is64 else torch.float32, device)
    return t, (_lib.RTH_F64 if is64 else _lib.RTH_F32)


def tree_update_timeouts():
    """tree-update top passes whose bounded wait for their subtree workgroups timed out since
    the library was loaded (rth_tree_update_timeouts; expected 0 -- the tests assert it)"""
    v = ctypes.c_int64(0)
    call("rth_tree_update_timeouts", ctypes.byref(v))
    return int(v.value)


class SumTree:
    """Device in-order heap sum-tree with NumbaSumTree's interface (fp64, bit-exact)."""

    def __init__(self, capacity, device=None, _handle=None):
        self.capacity = int(capacity)
        self.device = _device(device)
        self._owned = _handle is None
        if _handle is None:
            h = c_vp()
            with torch.cuda.device(self.device):
                call("rth_sumtree_create", self.capacity, self.device.index, ctypes.byref(h))
            _handle = h.value
        self._h = _handle
        self._stats = torch.empty(2, dtype=torch.float64, device=self.device)

    def __del__(self):
        if getattr(self, "_owned", False) and getattr(self, "_h", None):
            try:
                _lib.lib().rth_sumtree_destroy(self._h)
            except Exception:
                pass
            self._h = None

    @property
    def handle(self):
        return self._h

    def clear(self):
        call("rth_sumtree_clear", self._h, stream_ptr())

    def update(self, indices, weights):
        idx = as_device(indices, torch.int64, self.device)
        w = as_device(weights, torch.float64, self.device)
        assert idx.numel() == w.numel()  # _numba_update assert (sumtree.py:63)
        call("rth_sumtree_update", self._h, ptr(idx), ptr(w), idx.numel(), stream_ptr())

    def find(self, targets):
        tg = as_device(targets, torch.float64, self.device)
        idx = torch.empty(tg.numel(), dtype=torch.int64, device=self.device)
        val = torch.empty(tg.numel(), dtype=torch.float64, device=self.device)
        call("rth_sumtree_find", self._h, ptr(tg), tg.numel(), ptr(idx), ptr(val), stream_ptr())
        return idx, val

    def sample(self, batch_size, uniforms=None, seed=0, counter=0):
        assert batch_size > 0
        u = None if uniforms is None else as_device(uniforms, torch.float64, self.device)
        idx = torch.empty(batch_size, dtype=torch.int64, device=self.device)
        val = torch.empty(batch_size, dtype=torch.float64, device=self.device)
        call("rth_sumtree_sample", self._h, batch_size, ptr(u), seed, counter, ptr(idx), ptr(val),
             stream_ptr())
        return idx, val

    def stats(self):
        """device tensor [sum(), min()] (no sync)"""
        call("rth_sumtree_stats", self._h, ptr(self._stats), stream_ptr())
        return self._stats

    def sum(self):
        return float(self.stats()[0])

    def min(self):
        return float(self.stats()[1])

    def export(self):
        s, m, v = (torch.empty(self.capacity, dtype=torch.float64, device=self.device) for _ in range(3))
        call("rth_sumtree_export", self._h, ptr(s), ptr(m), ptr(v), stream_ptr())
        return s, m, v

    def load(self, s, m, v):
        s, m, v = (as_device(x, torch.float64, self.device) for x in (s, m, v))
        call("rth_sumtree_import", self._h, ptr(s), ptr(m), ptr(v), stream_ptr())


class PERSampler:
    """reth_buffer/reth_buffer/sampler/per_sampler.py:5-35 on the device tree.

    `update` fuses _normalize_weights ((w + 1e-6) ** alpha) into the tree update; `sample`
    returns device tensors (indices int64, IS weights float64).  Without explicit uniforms
    the targets come from Philox(seed, call counter) on the device."""

    def __init__(self, capacity, alpha=0.6, beta=0.4, device=None, seed=0):
        self.sumtree = SumTree(capacity, device)
        self.device = self.sumtree.device
        self._alpha_str, self._beta_str = alpha, beta
        self.alpha = Schedule.from_str(alpha)
        self.beta = Schedule.from_str(beta)
        self.seed = seed
        self.calls = 0

    def ready_sample(self, batch_size):
        return True

    def clear(self):
        self.sumtree.clear()
        self.alpha = Schedule.from_str(self._alpha_str)
        self.beta = Schedule.from_str(self._beta_str)

    def on_step(self):
        self.alpha.step()
        self.beta.step()

    def update(self, indices, weights):
        idx = as_device(indices, torch.int64, self.device)
        w, wt = _prio_tensor(weights, self.device)
        assert idx.numel() == w.numel()
        call("rth_per_update", self.sumtree.handle, ptr(idx), ptr(w), wt, idx.numel(),
             float(self.alpha.value()), stream_ptr())

    def sample(self, batch_size, uniforms=None):
        u = None if uniforms is None else as_device(uniforms, torch.float64, self.device)
        idx = torch.empty(batch_size, dtype=torch.int64, device=self.device)
        isw = torch.empty(batch_size, dtype=torch.float64, device=self.device)
        call("rth_per_sample", self.sumtree.handle, batch_size, float(self.beta.value()), ptr(u), self.seed,
             self.calls, ptr(idx), ptr(isw), stream_ptr())
        self.calls += 1
        return idx, isw


class Column:
    """one replay column: per-row shape, storage dtype, sampled dtype.  channels_last (uint8
    (C,H,W) -> float32 only) makes sampled batches channels-last [B,C,H,W] tensors, the
    memory format the Q-network's NHWC convolutions consume without a transpose."""

    def __init__(self, shape, dtype, out_dtype=None, channels_last=False):
        self.shape = tuple(int(s) for s in shape)
        self.dtype = dtype
        self.out_dtype = out_dtype or dtype
        self.row_elems = int(np.prod(self.shape)) if self.shape else 1
        self.channels_last = bool(channels_last)
        if dtype not in _TORCH_TO_RTH:
            raise TypeError(f"unsupported replay column dtype {dtype}")
        if self.out_dtype != dtype and not (dtype == torch.uint8 and self.out_dtype == torch.float32):
            raise TypeError(f"unsupported column conversion {dtype} -> {self.out_dtype}")
        if self.channels_last and (len(self.shape) != 3 or self.out_dtype != torch.float32 or dtype != torch.uint8):
            raise TypeError("channels_last needs a uint8 (C,H,W) column sampled as float32")

    @property
    def out_planes(self):
        return self.shape[0] if self.channels_last else 0

    def desc(self):
        return ColDesc(self.row_elems, _TORCH_TO_RTH[self.dtype], _TORCH_TO_RTH[self.out_dtype], self.out_planes, 0)

    def empty_out(self, n, device):
        fmt = torch.channels_last if self.channels_last else torch.contiguous_format
        return torch.empty((n, *self.shape), dtype=self.out_dtype, device=device, memory_format=fmt)


class FrameColumn(Column):
    """a frame-stack column of a frame-store replay: a row stores its
    stack as `shape[0]` int32 frame ids into the replay's frame store, the sample assembles
    the uint8 stack [K, H, W] -- the bytes a full uint8 row would hold (rth_replay_frames_attach)"""

    def __init__(self, shape):
        super().__init__(shape, torch.int32, torch.int32)
        self.out_dtype = torch.uint8
        self.frames = True

    @property
    def out_planes(self):
        return self.shape[0]

    @property
    def frame_bytes(self):
        return self.row_elems // self.shape[0]

    def desc(self):
        return ColDesc(self.row_elems, _lib.RTH_FRAMES, _lib.RTH_U8, self.out_planes, 0)


class FrameStacks:
    """a batch of uint8 frame stacks [n, K, H, W] held as their int32 [n, K] frame ids into a
    replay's frame store (HbmReplay.set_frame_ids: the gather copies the ids, not the stacks);
    conv1 reads the frames in place (rth_conv1_frames_bias_relu / _relu_wgrad_ex), with
    results bit-identical to the same launches on the stacks() the gather would have written"""

    dtype = torch.uint8
    is_cuda = True

    def __init__(self, ids, store):
        self.ids, self.store = ids, store  # store: the replay's frames [F, H, W] (uint8)
        self.shape = torch.Size((ids.shape[0], ids.shape[1], *store.shape[1:]))

    @property
    def device(self):
        return self.ids.device

    def data_ptr(self):
        return self.ids.data_ptr()

    def dim(self):
        return 4

    def __len__(self):
        return self.shape[0]

    def __getitem__(self, rows):
        if not isinstance(rows, slice):
            raise TypeError("FrameStacks rows are taken by slice")
        return FrameStacks(self.ids[rows], self.store)

    def stacks(self):
        """the uint8 stacks themselves [n, K, H, W] (a torch gather; not on the hot path)"""
        return self.store[self.ids.long()]

    def cpu(self):
        """the stacks on the host (host-side consumers -- NumpyLoader, evaluation clients --
        treat a frame-id column like any other uint8 column)"""
        return self.stacks().cpu()

    @staticmethod
    def pair(a, b):
        """[a; b]: a view when b's ids sit right behind a's (HbmReplay.new_batch), else a copy"""
        if a.store is b.store and a.ids.is_contiguous() and b.ids.is_contiguous() and \
                b.ids.data_ptr() == a.ids.data_ptr() + a.ids.numel() * 4:
            return FrameStacks(torch.as_strided(a.ids, (2 * a.ids.shape[0], a.ids.shape[1]), a.ids.stride()), a.store)
        return FrameStacks(torch.cat([a.ids, b.ids]), a.store)


SAMPLERS = {"per": _lib.SAMPLER_PER, "uniform": _lib.SAMPLER_UNIFORM, "fifo": _lib.SAMPLER_FIFO}


class HbmReplay:
    """A replay shard resident in HBM (one per GPU).

    columns: list of Column.  alpha / beta: schedule specs (numbers or "start,end,steps").
    sampler: "per" (PERSampler, the Ape-X path), "uniform" (UniformSampler) or "fifo"
    (FIFOSampler) -- reth_buffer/reth_buffer/sampler/*.py; the non-PER samplers return
    their weights (ones / the pushed weights) where PER returns IS weights.
    """

    def __init__(self, capacity, columns, alpha=0.6, beta=0.4, device=None, seed=0, sampler="per", frame_store=None):
        if not 1 <= len(columns) <= _lib.MAX_COLS:
            raise ValueError(f"1..{_lib.MAX_COLS} columns supported, got {len(columns)}")
        self.capacity = int(capacity)
        self.columns = list(columns)
        self.device = _device(device)
        self._alpha_str, self._beta_str = alpha, beta
        self.alpha = Schedule.from_str(alpha)
        self.beta = Schedule.from_str(beta)
        if sampler not in SAMPLERS:
            raise ValueError(f"sampler must be one of {sorted(SAMPLERS)}, got {sampler!r}")
        self.sampler = sampler
        descs = (ColDesc * len(columns))(*[c.desc() for c in columns])
        h = c_vp()
        with torch.cuda.device(self.device):
            call("rth_replay_create", self.capacity, len(columns), descs, SAMPLERS[sampler],
                 ctypes.byref(sched_struct(self.alpha)), ctypes.byref(sched_struct(self.beta)), self.device.index,
                 int(seed), ctypes.byref(h))
        self._h = h.value
        # frame_store (int): the frame de-duplicated replay -- FrameColumn stacks as frame ids
        # into a ring of that many frames (rth_replay_frames_attach); frames / frame_head are
        # device views of the store and its head.  The ring must outlive every live row's
        # frames: frame ids are taken mod its size, so a ring smaller than the frames pushed
        # during a row's life silently hands that row newer frames (ApexDQN.frame_store_frames
        # gives the worst-case size: 2 frames per actor step)
        self.frames = self.frame_head = None
        fcols = [c for c in self.columns if getattr(c, "frames", False)]
        if frame_store is not None or fcols:
            if not fcols or frame_store is None:
                raise ValueError("a frame store needs FrameColumn columns and frame_store=<frames>, both")
            fb = fcols[0].frame_bytes
            store, head = c_vp(), c_vp()
            with torch.cuda.device(self.device):
                call("rth_replay_frames_attach", self._h, int(frame_store), fb, ctypes.byref(store), ctypes.byref(head))
            self.frames = _wrap_device(store.value, int(frame_store) * fb, torch.uint8, self.device).view(
                int(frame_store), *fcols[0].shape[1:])
            self.frame_head = _wrap_device(head.value, 1, torch.int64, self.device)
        th = _lib.lib().rth_replay_tree(self._h)
        self._tree = SumTree(self.capacity, self.device, _handle=th) if th else None
        self._pending = None  # buffers of a deferred priority update (kept alive until applied)

    @property
    def tree(self):
        """the shard's sum-tree (a deferred priority update is applied first)"""
        self.flush()
        return self._tree

    def flush(self):
        """apply a deferred update_priorities now (rth_replay_flush)"""
        if self._pending is not None:
            call("rth_replay_flush", self._h, stream_ptr())
            self._pending = None

    def __del__(self):
        if getattr(self, "_h", None):
            try:
                _lib.lib().rth_replay_destroy(self._h)
            except Exception:
                pass
            self._h = None

    # ---------------------------------------------------------------- counters
    def _info(self):
        vals = [c_i64() for _ in range(6)]
        call("rth_replay_info", self._h, *[ctypes.byref(v) for v in vals])
        return tuple(v.value for v in vals)

    def info(self):
        """host mirrors: (size, tail, cnt, sample_calls, schedule steps)"""
        return self._info()[:5]

    @property
    def sampler_len(self):
        """PER: rows stored; uniform: index-list length; FIFO: queued entries"""
        return self._info()[5]

    def ready_sample(self, batch_size):
        """BaseSampler.ready_sample: FIFOSampler needs len > batch (fifo_sampler.py:16-17)"""
        if self.sampler == "fifo":
            return self.sampler_len > batch_size
        return self.sampler_len > 0

    @property
    def size(self):
        return self.info()[0]

    @property
    def cnt(self):
        return self.info()[2]

    def column_storage(self, c):
        """device tensor view of column c's storage [capacity, *shape] ([capacity, K] frame ids
        for a FrameColumn)"""
        col = self.columns[c]
        p = _lib.lib().rth_replay_column(self._h, c)
        if getattr(col, "frames", False):
            return _wrap_device(p, self.capacity * col.shape[0], torch.int32, self.device).view(self.capacity,
                                                                                                 col.shape[0])
        n = self.capacity * col.row_elems
        return _wrap_device(p, n, col.dtype, self.device).view(self.capacity, *col.shape)

    def push_frames(self, ring, n, ring_slots, s0_h, s1_h, done, cur_slot, sid, init=False):
        """an actor step's new frames into the frame store and the stacks' frame ids into
        `sid` (rth_replay_push_frames; init: the actors' initial stacks)"""
        call("rth_replay_push_frames", self._h, ptr(ring), int(n), int(ring_slots), int(ring.shape[1]), ptr(s0_h),
             ptr(s1_h), ptr(done), ptr(cur_slot), ptr(sid), 1 if init else 0, stream_ptr())

    # ---------------------------------------------------------------- ops
    def append(self, cols, td_abs, src_rows=None, row_strides=None, idx_out=None, raw=False):
        """Client.append + append_loop: rows of `cols` (device tensors, [n, *shape] or a row
        source with src_rows) into FIFO slots; priorities (td_abs + 1e-6) ** alpha, or stored
        as given (float64) with raw=True."""
        if len(cols) != len(self.columns):
            raise ValueError(f"expected {len(self.columns)} columns, got {len(cols)}")
        w, wt = _prio_tensor(td_abs, self.device, raw)
        n = w.numel()
        assert n <= self.capacity  # fifo_policy.py:12
        srcs = (Src * len(cols))()
        keep = []
        for c, (col, t) in enumerate(zip(self.columns, cols)):
            src_dtype = 0  # as stored
            if t.dtype == torch.float32 and col.dtype == torch.uint8:
                src_dtype = _lib.RTH_F32  # float32 frames narrowed to bytes by the copy kernel
                if not t.is_cuda:
                    t = t.to(self.device)
            elif t.dtype != col.dtype or not t.is_cuda:
                t = t.to(device=self.device, dtype=col.dtype)
            t = t if t.is_contiguous() else t.contiguous()
            rows = None if src_rows is None else src_rows[c]
            if rows is None and t.shape[0] != n:
                raise ValueError(f"column {c} has {t.shape[0]} rows, priorities have {n}")
            keep.append(t)
            stride = 0 if row_strides is None else int(row_strides[c])
            srcs[c] = Src(ptr(t), ptr(rows), stride, src_dtype, 0)
        call("rth_replay_append", self._h, srcs, ptr(w), wt, n, ptr(idx_out), stream_ptr())
        self._pending = None  # a deferred update was merged into this launch
        return n

    def append_strided(self, cols, td_abs, row_strides, raw=False):
        """append from columns that live inside a device byte buffer (pack.ingest_append):
        cols[c].view starts at row 0 of column c, rows row_strides[c] bytes apart;
        cols[c].dtype is the source element type (float32 narrows into uint8 storage)."""
        w, wt = _prio_tensor(td_abs, self.device, raw)
        n = w.numel()
        assert n <= self.capacity  # fifo_policy.py:12
        srcs = (Src * len(cols))()
        for c, (col, bc) in enumerate(zip(self.columns, cols)):
            if bc.row_elems != col.row_elems:
                raise ValueError(f"column {c}: message rows hold {bc.row_elems} elements, replay rows {col.row_elems}")
            if bc.dtype != col.dtype and not (bc.dtype == torch.float32 and col.dtype == torch.uint8):
                raise TypeError(f"column {c}: {bc.dtype} rows into {col.dtype} storage")
            srcs[c] = Src(ptr(bc.view), None, int(row_strides[c]), _TORCH_TO_RTH[bc.dtype], 0)
        call("rth_replay_append", self._h, srcs, ptr(w), wt, n, None, stream_ptr())
        self._pending = None
        return n

    def sample_into(self, batch_size, out_cols, idx_out, isw_out, uniforms=None, gather_timer=None):
        """PER sample + gather into preallocated outputs.  gather_timer (optional) is a
        callable returning a (start, end) pair of torch.cuda.Event recorded around the
        gather launch alone (the bench's live roofline measurement)."""
        u = None if uniforms is None else as_device(uniforms, torch.float64, self.device)
        arr = (c_vp * len(out_cols))(*[ptr(t) for t in out_cols])
        if gather_timer is None:
            call("rth_replay_sample", self._h, batch_size, ptr(u), arr, ptr(idx_out), ptr(isw_out), stream_ptr())
            self._pending = None  # the sample applied a deferred update first
            return
        s = stream_ptr()
        call("rth_replay_sample", self._h, batch_size, ptr(u), None, ptr(idx_out), ptr(isw_out), s)
        self._pending = None
        ev0, ev1 = gather_timer()
        ev0.record()
        call("rth_replay_gather", self._h, ptr(idx_out), batch_size, arr, s)
        ev1.record()

    def set_frame_ids(self, on=True):
        """frames in place: gathers write the frame-stack columns' frame ids (FrameStacks
        batches from new_batch) instead of the assembled stacks (rth_replay_frames_ids_out)"""
        call("rth_replay_frames_ids_out", self._h, 1 if on else 0)
        self.frame_ids = bool(on)

    def new_batch(self, batch_size):
        """empty (cols, idx, isw) batch buffers.  Columns of identical row shape and sampled
        dtype share one allocation, back to back in column order (s1 directly behind s0), so
        a learner can run one forward over [s0; s1] without a copy (fused_learner._pair);
        with set_frame_ids, frame-stack columns are FrameStacks over one id allocation"""
        groups = {}
        for i, c in enumerate(self.columns):
            groups.setdefault((c.shape, c.out_dtype, c.channels_last), []).append(i)
        cols = [None] * len(self.columns)
        for members in groups.values():
            c = self.columns[members[0]]
            if getattr(self, "frame_ids", False) and getattr(c, "frames", False):
                ids = torch.empty((len(members) * batch_size, c.shape[0]), dtype=torch.int32, device=self.device)
                for k, i in enumerate(members):
                    cols[i] = FrameStacks(ids[k * batch_size:(k + 1) * batch_size], self.frames)
                continue
            buf = c.empty_out(len(members) * batch_size, self.device)
            for k, i in enumerate(members):
                cols[i] = buf[k * batch_size:(k + 1) * batch_size]
        idx = torch.empty(batch_size, dtype=torch.int64, device=self.device)
        isw = torch.empty(batch_size, dtype=torch.float64, device=self.device)
        return cols, idx, isw

    def sample(self, batch_size, uniforms=None):
        cols, idx, isw = self.new_batch(batch_size)
        self.sample_into(batch_size, cols, idx, isw, uniforms)
        return cols, idx, isw

    def gather(self, indices, out_cols=None):
        idx = as_device(indices, torch.int64, self.device)
        if out_cols is None:
            out_cols = (self.new_batch(idx.numel())[0] if getattr(self, "frame_ids", False)
                        else [c.empty_out(idx.numel(), self.device) for c in self.columns])
        arr = (c_vp * len(out_cols))(*[ptr(t) for t in out_cols])
        call("rth_replay_gather", self._h, ptr(idx), idx.numel(), arr, stream_ptr())
        return out_cols

    def update_priorities(self, indices, td_abs, step=False, raw=False, deferred=False):
        """Client.update_priorities -> sampler_loop: on_step() first when step (:32-35).
        The device owns the schedules; the host Schedules mirror them for inspection.
        deferred: applied by the next tree launch (merged into the next append's), in the
        same order the reference's sampler applies its messages."""
        if step:
            self.alpha.step()
            self.beta.step()
        idx = as_device(indices, torch.int64, self.device)
        w, wt = _prio_tensor(td_abs, self.device, raw)
        assert idx.numel() == w.numel()  # client.py:38
        fn = "rth_replay_update_priorities_deferred" if deferred else "rth_replay_update_priorities"
        call(fn, self._h, ptr(idx), ptr(w), wt, idx.numel(), int(bool(step)), stream_ptr())
        self._pending = (idx, w) if deferred and self.sampler == "per" else None


def sched_struct(s):
    """Schedule -> rth_schedule (the device evaluates it in the same operation order)"""
    from ._lib import SCHED_CONST, SCHED_EXP, SCHED_LINEAR, Sched

    if s.method == "const":
        return Sched(SCHED_CONST, 0, float(s.const), float(s.const), 1)
    return Sched(SCHED_LINEAR if s.method == "linear" else SCHED_EXP, 0, s.start, s.end, s.max_steps)


def _wrap_device(p, n, dtype, device):
    """A torch view of foreign device memory owned by a handle (kept alive by the caller)."""
    elem = torch.empty((), dtype=dtype).element_size()
    return _from_dev_ptr(p, n * elem, device).view(dtype)[:n]


def _from_dev_ptr(p, nbytes, device):
    class _Iface:
        pass

    iface = _Iface()
    iface.__cuda_array_interface__ = {"shape": (nbytes,), "typestr": "|u1", "data": (p, False), "version": 3}
    with torch.cuda.device(device):
        return torch.as_tensor(iface, device=device)
