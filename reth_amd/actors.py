"""Vectorised Ape-X actors on one GPU.

Reference actor loop: test/apex-dqn/worker.py:21-61 -- per actor process: epsilon-greedy act
(reth/reth/utils/exploration.py:26-31 -> DQNSolver.act, dqn_solver.py:126-131), env.step,
cast to f4/i8/f4/f4/f4, NStepAdder.push (reth/reth/utils/nstep_adder.py:11-28), a 64-row
staging NumpyBuffer, then calc_loss (the actor's stale copy: target == online, because
load_weights calls update_target, dqn_solver.py:133-137) and Client.append.

Here all N actors of a GPU step together, entirely in HBM:
  frames   uint8 [N, ring, 4, 84, 84]   per-actor ring of frame stacks (obs, next obs,
                                         reset obs); rows reference stacks by handle
                                         actor*ring + slot, never copy them until insert
  step():  Q-net over the acting stacks (batch N; the HIP conv torso reads the uint8 ring
           through the stack handles) -> rth_eps_greedy -> rth_synth_env_step ->
           rth_nstep_push (emits one row per actor once warm)
  prioritise(): Q-net over the emitted rows' s0/s1 stacks (batch 2N) -> rth_td_huber
           (no grad) = calc_loss
  step_fused(): the acting forward and the previous step's rows' priorities in one step: the
           rows' heads come from a per-stack cache (dedup) or one 4-way forward, then
           rth_actor_tail (eps-greedy + |td| + env step + n-step push, one launch)
  append(): rth_replay_append copies the rows' stacks from the ring into FIFO slots and
           inserts (|td| + 1e-6)^alpha into the tree.
No host synchronisation anywhere in the loop.
"""

import numpy as np
import torch

from . import _lib
from ._lib import call, ptr, stream_ptr
from .solver import td_huber_forward

OBS_SHAPE = (4, 84, 84)
STACK_ELEMS = 4 * 84 * 84


def apex_epsilons(n, offset=0, total=None):
    """eps_i = 0.4 ** (1 + 7 i / (size - 1)) (test/apex-dqn/worker.py:26), float64"""
    total = n if total is None else total
    i = np.arange(offset, offset + n, dtype=np.float64)
    if total <= 1:
        return np.full(n, 0.4)
    return 0.4 ** (1 + (i / (total - 1)) * 7)


class VecActors:
    def __init__(self, n_actors, num_actions, n_step=3, gamma=0.99, device=None, seed=0, eps=None,
                 actor_offset=0, total_actors=None, p_reward=0.02, p_done=1.0 / 2000, nstep_mode=0,
                 channels_last=False, env="synthetic"):
        self.N = int(n_actors)
        self.A = int(num_actions)
        self.n_step, self.gamma = int(n_step), float(gamma)
        self.gamma_n = float(np.float32(gamma ** n_step))
        self.device = torch.device(device if device is not None else "cuda")
        self.seed = int(seed)
        self.p_reward, self.p_done = float(p_reward), float(p_done)
        ring = 4
        while ring < 2 * (self.n_step + 3):  # live stacks span n_step + 2 env steps (+1 when the
            ring *= 2                         # rows are prioritised a step late), 2 per step
        self.ring = ring
        dev = self.device
        N = self.N
        # one extra all-zero stack at N * ring: the sink handle of unused batch slots.  Zero-filled
        # once: ring slots no step has written yet read as zeros, never as whatever the
        # allocator's block held before (graph and eager runs of one seed compare equal)
        self.frames = torch.zeros((N * ring + 1, *OBS_SHAPE), dtype=torch.uint8, device=dev)
        self.cur_slot = torch.empty(N, dtype=torch.int64, device=dev)
        e = apex_epsilons(N, actor_offset, total_actors) if eps is None else np.broadcast_to(np.asarray(eps, np.float64), (N,))
        self.eps = torch.as_tensor(np.ascontiguousarray(e), dtype=torch.float64, device=dev)
        self.channels_last = bool(channels_last)
        fmt = torch.channels_last if channels_last else torch.contiguous_format
        self._fmt = fmt
        self._f32 = {}  # f32 observation batches, only for networks that cannot read uint8 stacks
        z = lambda dt: torch.zeros(N, dtype=dt, device=dev)
        self.action, self.s0_h, self.s1_h = z(torch.int64), z(torch.int64), z(torch.int64)
        self.reward, self.done = z(torch.float32), z(torch.float32)
        self.emit = z(torch.int32)
        self.row_s0, self.row_a, self.row_s1 = z(torch.int64), z(torch.int64), z(torch.int64)
        self.row_r, self.row_done = z(torch.float32), z(torch.float32)
        self.row_handles = torch.empty(2 * N, dtype=torch.int64, device=dev)
        # step_fused: rows alternate between two sets by push parity (the rows of step t are
        # prioritised and appended at step t + 1, while step t + 1 emits into the other set)
        self._sets = [self._rowset_of_attrs(), RowSet(N, dev)]
        self.handles3 = torch.empty(3 * N, dtype=torch.int64, device=dev)
        h = _lib.c_vp()
        call("rth_nstep_create", N, self.n_step, self.gamma, int(nstep_mode), dev.index, _lib.ctypes.byref(h))
        self._nstep = h.value
        # deduplicated prioritisation (step_fused dedup mode): per frame-ring stack, the actor
        # network's heads from the last forward that covered it; the rows' s0 / s1 are looked
        # up there instead of being run through the network again.  Row N * ring is a sink for
        # the unused slots of the variable-size batch.
        self._sink = N * ring
        self.qcache = None  # [N * ring + 1, A + 1], allocated at the first forward
        # forward batch handles [acting | terminal stacks of the last step (sink-padded) |
        # previous rows' s0 | their s1]: dedup forwards the first 2N (n_ext counted), full all 4N
        self.hx = torch.full((4 * N,), self._sink, dtype=torch.int64, device=dev)
        self.n_ext = torch.full((1,), N, dtype=torch.int64, device=dev)  # acting + terminal stacks
        self._base = torch.arange(N, device=dev, dtype=torch.int64) * ring
        self.qrows = None
        # dedup forwards with the counted FC: FC1 as a GEMM over the N acting rows only, the
        # terminal stacks behind them device-counted, instead of one GEMM over all 2N rows.  Above
        # 512 actors (Breakout: 2,048 actors, the actor stream critical) 0.905 vs 0.954 ms/step
        # (r04); at Pong since the N-row FC1 runs on rth_fc_x9 (late r05: the hipBLASLt 256-row
        # GEMM took as long as the 512-row one, the x9 kernel's time follows the rows) 0.534 vs
        # 0.542-0.544 ms/step.  The second layer covers the counted rows only and writes the
        # per-stack heads cache in the same launch (rth_heads_fc2_upto).
        self.fresh = 0       # steps since the actor network's weights last changed
        self.t = 0           # env steps taken (per actor): host mirror of t_dev
        self.t_dev = torch.zeros(1, dtype=torch.int64, device=dev)  # what the kernels read
        self.pushes = 0
        call("rth_synth_env_reset", ptr(self.frames), N, ring, self.seed, ptr(self.cur_slot), stream_ptr())
        self.frame_replay = None  # attach_frame_store: the frame de-duplicated replay the steps feed
        self.sid = None
        # env: "synthetic" -- Pong-shaped uint8 frames straight from device Philox;
        # "atari" -- raw 210x160 RGB frame pairs (device Philox, the stand-in for ALE's screens)
        # through the MaxAndSkip / WarpFrame / FrameStack preprocessing (rth_atari_env_step)
        # into the frame ring; "atari-h2d" -- the raw pairs copied host -> device from pinned
        # memory every step first, as from host ALE emulators (reth/reth/env/util.py:121-209).
        # The reset screens of ended episodes come from device Philox in both modes
        if env not in ("synthetic", "atari", "atari-h2d"):
            raise ValueError(f"env {env!r}: synthetic | atari | atari-h2d")
        self.env = env
        if env != "synthetic":
            from .atari import AtariPreprocessor

            self.atari = AtariPreprocessor(device=dev)
            self.raw = torch.empty((N, 2, 210, 160, 3), dtype=torch.uint8, device=dev)
            # the reset screens (Worker.step's env.reset() after done, presets/worker.py:146-148):
            # one raw frame per actor, written / read only for the actors whose episode ended
            self.raw_reset = torch.zeros((N, 210, 160, 3), dtype=torch.uint8, device=dev)
            if env == "atari-h2d":
                g = np.random.default_rng(self.seed)
                self.raw_host = torch.from_numpy(g.integers(0, 256, tuple(self.raw.shape), dtype=np.uint8)).pin_memory()

    def attach_frame_store(self, replay):
        """feed a frame de-duplicated replay (HbmReplay with FrameColumns): every step's new
        frames enter its store once (rth_replay_push_frames) and each frame-ring stack's frame
        ids live in `sid` ([stacks, 4] int32), which the rows' appends copy instead of the stacks"""
        if replay.frames is None:
            raise ValueError("the replay has no frame store")
        self.frame_replay = replay
        self.sid = torch.zeros((self.frames.shape[0], OBS_SHAPE[0]), dtype=torch.int32, device=self.device)
        replay.push_frames(self.frames, self.N, self.ring, None, None, None, self.cur_slot, self.sid, init=True)

    def _push_frames(self):
        if self.frame_replay is not None:
            self.frame_replay.push_frames(self.frames, self.N, self.ring, self.s0_h, self.s1_h, self.done,
                                          self.cur_slot, self.sid)

    def __del__(self):
        if getattr(self, "_nstep", None):
            try:
                _lib.lib().rth_nstep_destroy(self._nstep)
            except Exception:
                pass
            self._nstep = None

    @property
    def warm(self):
        """every actor emits one n-step row per push once its deque is full"""
        return self.pushes > self.n_step

    def gather_f32(self, handles, out):
        call("rth_copy_rows", ptr(out), 0, None, ptr(self.frames), 0, ptr(handles), handles.numel(), STACK_ELEMS,
             _lib.RTH_U8, _lib.RTH_F32, OBS_SHAPE[0] if self.channels_last else 0, stream_ptr())
        return out

    def _forward_stacks(self, q_net, handles):
        """Q-net over the frame-ring stacks `handles`: the HIP torso reads the uint8 ring
        directly (rth_conv_bias_relu through the handle index, no f32 copy); other networks
        get a u8 -> f32 gather first"""
        if getattr(q_net, "hwc_features", False) and getattr(q_net, "dueling", False) and q_net.hip_conv:
            return q_net.forward_heads(self.frames, rows=handles), 1
        n = handles.numel()
        buf = self._f32.get(n)
        if buf is None:
            buf = self._f32[n] = torch.empty((n, *OBS_SHAPE), dtype=torch.float32, device=self.device,
                                             memory_format=self._fmt)
        return _q_forward(q_net, self.gather_f32(handles, buf))

    def current_obs_handles(self):
        if not hasattr(self, "_cur_h"):
            self._cur_h = torch.empty_like(self._base)
        return torch.add(self.cur_slot, self._base, out=self._cur_h)

    def _atari_frames(self, s):
        """Atari env mode, after the actor tail assigned the step's stack handles: this step's
        raw frame pairs (device Philox, or the pinned host buffer copied over PCIe) through the
        preprocessing into the ring"""
        if self.env == "atari":
            call("rth_atari_synth_raw", ptr(self.raw), self.raw.numel(), self.seed ^ 0x9E3779B97F4A7C15,
                 ptr(self.t_dev), s)
        else:
            self.raw.copy_(self.raw_host, non_blocking=True)
        # env.reset()'s screen for the actors whose episode ended (both modes: device Philox)
        call("rth_atari_synth_reset", ptr(self.raw_reset), self.N, self.raw_reset[0].numel(),
             self.seed ^ 0x7F4A7C159E3779B9, ptr(self.t_dev), ptr(self.done), s)
        call("rth_atari_env_step", self.atari._h, ptr(self.raw), self.N, ptr(self.frames), self.ring, OBS_SHAPE[0],
             ptr(self.s0_h), ptr(self.s1_h), ptr(self.done), ptr(self.cur_slot), ptr(self.raw_reset), s)

    @torch.no_grad()
    def step(self, q_net):
        """one environment step for every actor; returns True when rows were emitted"""
        if self.env != "synthetic":
            raise RuntimeError("the Atari env mode runs in step_fused with the HIP torso actor network")
        s = stream_ptr()
        self.t += 1
        call("rth_counter_add", ptr(self.t_dev), 1, s)
        # acting batch: the current stacks (Worker.step -> exploration.act -> solver.act)
        q, dueling = self._forward_stacks(q_net, self.current_obs_handles())
        call("rth_eps_greedy", ptr(q), self.N, self.A, dueling, ptr(self.eps), None, None, self.seed, 0,
             ptr(self.t_dev), ptr(self.action), s)
        call("rth_synth_env_step", ptr(self.frames), self.N, self.ring, 0, ptr(self.t_dev), ptr(self.cur_slot),
             ptr(self.action), self.seed, self.p_reward, self.p_done, ptr(self.reward), ptr(self.done), ptr(self.s0_h),
             ptr(self.s1_h), s)
        self._push_frames()
        call("rth_nstep_push", self._nstep, ptr(self.s0_h), ptr(self.action), ptr(self.reward), ptr(self.s1_h),
             ptr(self.done), ptr(self.emit), ptr(self.row_s0), ptr(self.row_a), ptr(self.row_r), ptr(self.row_s1),
             ptr(self.row_done), s)
        self.pushes += 1
        return self.warm

    def _rowset_of_attrs(self):
        rs = RowSet.__new__(RowSet)
        rs.s0, rs.a, rs.r, rs.s1, rs.done = self.row_s0, self.row_a, self.row_r, self.row_s1, self.row_done
        return rs

    def _bind_rows(self, rs):
        self.row_s0, self.row_a, self.row_r, self.row_s1, self.row_done = rs.s0, rs.a, rs.r, rs.s1, rs.done

    def weights_changed(self):
        """the actor network was reloaded: cached heads are stale until n + 2 steps passed"""
        self.fresh = 0

    @staticmethod
    def _hip_heads(q_net):
        return getattr(q_net, "hwc_features", False) and getattr(q_net, "dueling", False) and q_net.hip_conv

    def dedup_ready(self, q_net):
        """every stack a row prioritised now can reference has cached heads computed with the
        current weights: its s0 was acted at most n + 1 steps ago, its s1 was acted at most n
        steps ago or is the terminal stack of an episode that ended in the last n + 1 steps
        (each forward -- dedup or full -- covers the previous step's terminal stacks).  The
        terminal stacks' heads are needed: the reference's NStepAdder (nstep_adder.py:14-24)
        rewrites the s1 of the window's older rows to the terminal observation but leaves their
        done at 0, so those rows bootstrap from it (dropping the terminal forward was measured:
        |td| off in ~20 % of rows at p_done = 0.25, and no faster)"""
        return self.qcache is not None and self.fresh >= self.n_step + 2 and self._hip_heads(q_net)

    def _scatter_heads(self, q, handles, n):
        """qcache[handles[i]] = q[i] for i < n (the sink absorbs unused slots)"""
        A1 = q.shape[1]
        if self.qcache is None:
            self.qcache = torch.zeros((self.N * self.ring + 1, A1), dtype=torch.float32, device=self.device)
            self.qrows = torch.empty((2 * self.N, A1), dtype=torch.float32, device=self.device)
        call("rth_copy_rows", ptr(self.qcache), 0, ptr(handles), ptr(q), 0, None, n, A1, _lib.RTH_F32, _lib.RTH_F32, 0,
             stream_ptr())

    def _terminal_stacks(self):
        """behind the next acting batch: the terminal stacks of this step's finished episodes
        (the s1 a done row keeps, which the next acting batch -- reset stacks -- does not cover)"""
        N = self.N
        call("rth_compact_flagged", ptr(self.done), ptr(self.s1_h), N, ptr(self.hx[N:2 * N]), N, self._sink, N,
             ptr(self.n_ext), stream_ptr())

    @torch.no_grad()
    def step_fused(self, q_net, dedup=None, probe=None):
        """one environment step for every actor with the previous step's rows prioritised in
        the same forward pass: Q-net over [acting stacks; prev rows' s0; prev rows' s1]
        (3N) -> rth_eps_greedy on the first N -> rth_td_huber (calc_loss, target == online)
        on the rest -> env step -> n-step push into the other row set.  The reference's
        actor runs calc_loss on a 64-row batch well after the rows were emitted
        (test/apex-dqn/worker.py:55-60); here the delay is one step.
        dedup (default: whenever dedup_ready): the forward covers only the acting stacks and
        the terminal stacks of the episodes that ended in the previous step (a device-side
        count); the rows' heads come from the per-stack cache -- the same values, about a third
        of the forward work.
        probe (HIP-torso path): handed [("actor_tail", launch)] to issue itself (the bench's live
        timing of k_actor_tail, fused_learner.dueling_grads' probe convention).
        Returns (|td|, RowSet) of the previous step's rows, or (None, None) before any."""
        s = stream_ptr()
        p = self.pushes
        prev, cur = self._sets[(p - 1) % 2], self._sets[p % 2]
        if dedup is None:
            dedup = self.dedup_ready(q_net)
        elif dedup and not self.dedup_ready(q_net):
            raise RuntimeError("step_fused(dedup=True): the stack cache is not valid for the current weights")
        self.t += 1
        N = self.N
        hip = self._hip_heads(q_net)
        if hip:  # step counter + acting rows (= cur_slot + _base) in one launch
            call("rth_actor_prologue", ptr(self.t_dev), ptr(self.cur_slot), N, self.ring, ptr(self.hx), s)
            if dedup:  # acting + terminal stacks (device count); the rows' heads are in the cache
                if q_net._fc2_inplace():  # the second layer over the counted rows, the cache in its launch
                    q = q_net.forward_heads(self.frames, rows=self.hx[:2 * N], n_dev=self.n_ext, n_fixed=N,
                                            cache=(self.qcache, self.hx))
                else:
                    q = q_net.forward_heads(self.frames, rows=self.hx[:2 * N], n_dev=self.n_ext)
                    self._scatter_heads(q, self.hx, 2 * N)
            else:  # everything: acting, last step's terminal stacks, the rows' s0 and s1 -> cache
                torch.cat([prev.s0, prev.s1], out=self.hx[2 * N:])
                q = q_net.forward_heads(self.frames, rows=self.hx)
                self._scatter_heads(q, self.hx, 4 * N)
            # eps-greedy, the previous rows' |td| from the cache, env step, n-step push: one launch
            td_abs = torch.empty(N, dtype=torch.float32, device=self.device)
            args = _lib.ActorTailArgs(ptr(q), ptr(self.eps), ptr(self.t_dev), ptr(self.action), ptr(self.qcache),
                                      ptr(prev.s0), ptr(prev.a), ptr(prev.s1), ptr(prev.r), ptr(prev.done),
                                      ptr(td_abs), ptr(self.frames), ptr(self.cur_slot), ptr(self.reward),
                                      ptr(self.done), ptr(self.s0_h), ptr(self.s1_h), self.seed, N, self.gamma_n,
                                      self.p_reward, self.p_done, self.ring, self.A, int(self.env != "synthetic"))
            def tail(args=args, cur=cur):
                call("rth_actor_tail", self._nstep, _lib.ctypes.byref(args), ptr(self.emit), ptr(cur.s0), ptr(cur.a),
                     ptr(cur.r), ptr(cur.s1), ptr(cur.done), stream_ptr())

            if probe is not None:  # the launch issued by the prober (a cut in a captured graph)
                probe([("actor_tail", tail)])
            else:
                tail()
            if self.env != "synthetic":
                self._atari_frames(s)
            self._push_frames()
            self._terminal_stacks()
            self.pushes += 1
            self.fresh += 1
            self._bind_rows(cur)
            return (td_abs, prev) if p > self.n_step else (None, None)
        else:
            if self.env != "synthetic":
                raise RuntimeError("the Atari env mode runs with the HIP torso actor network (dueling, channels-last)")
            call("rth_counter_add", ptr(self.t_dev), 1, s)
            torch.cat([self.current_obs_handles(), prev.s0, prev.s1], out=self.handles3)
            q, dueling = self._forward_stacks(q_net, self.handles3)
            q0, q1 = q[N:2 * N], q[2 * N:]
        call("rth_eps_greedy", ptr(q), N, self.A, dueling, ptr(self.eps), None, None, self.seed, 0,
             ptr(self.t_dev), ptr(self.action), s)
        _, td_abs, _ = td_huber_forward(q0, q1, q1, prev.a, prev.r, prev.done, None, self.gamma_n, True,
                                        want_dq=False, dueling=bool(dueling))
        call("rth_synth_env_step", ptr(self.frames), N, self.ring, 0, ptr(self.t_dev), ptr(self.cur_slot),
             ptr(self.action), self.seed, self.p_reward, self.p_done, ptr(self.reward), ptr(self.done), ptr(self.s0_h),
             ptr(self.s1_h), s)
        self._push_frames()
        call("rth_nstep_push", self._nstep, ptr(self.s0_h), ptr(self.action), ptr(self.reward), ptr(self.s1_h),
             ptr(self.done), ptr(self.emit), ptr(cur.s0), ptr(cur.a), ptr(cur.r), ptr(cur.s1), ptr(cur.done), s)
        self._terminal_stacks()
        self.pushes += 1
        self.fresh += 1
        self._bind_rows(cur)
        return (td_abs, prev) if p > self.n_step else (None, None)

    @torch.no_grad()
    def prioritise(self, q_net):
        """calc_loss on the emitted rows with the actor's network (target == online)"""
        torch.cat([self.row_s0, self.row_s1], out=self.row_handles)
        q, dueling = self._forward_stacks(q_net, self.row_handles)
        q0, q1 = q[: self.N], q[self.N:]
        _, td_abs, _ = td_huber_forward(q0, q1, q1, self.row_a, self.row_r, self.row_done, None, self.gamma_n,
                                        True, want_dq=False, dueling=bool(dueling))
        return td_abs

    def append(self, replay, td_abs, rows=None):
        """Client.append of emitted rows (default: the latest; stacks copied from the ring
        into FIFO slots)"""
        rs = self._rowset_of_attrs() if rows is None else rows
        fr = self.frames if replay.frames is None else self.sid  # frame store: the stacks' frame ids
        replay.append([fr, rs.a, rs.r, fr, rs.done], td_abs, src_rows=[rs.s0, None, None, rs.s1, None])

    def rows(self):
        """emitted rows as (s0 u8, a, r, s1 u8, done) device tensors (tests / inspection)"""
        return (self.frames[self.row_s0], self.row_a.clone(), self.row_r.clone(), self.frames[self.row_s1],
                self.row_done.clone())


class RowSet:
    """one set of emitted n-step rows: s0/s1 stack handles, a, r, done"""

    def __init__(self, n, dev):
        z = lambda dt: torch.zeros(n, dtype=dt, device=dev)
        self.s0, self.a, self.s1 = z(torch.int64), z(torch.int64), z(torch.int64)
        self.r, self.done = z(torch.float32), z(torch.float32)


def _q_forward(q_net, x):
    """(f32 contiguous network output, dueling flag): a dueling conv net returns its raw heads
    [n, A+1] through the merged-heads path and the HIP consumer forms Q (model.py)"""
    if getattr(q_net, "dueling", False) and hasattr(q_net, "forward_heads"):
        q, dueling = q_net.forward_heads(x), 1
    else:
        q, dueling = q_net(x), 0
    if q.dtype != torch.float32 or not q.is_contiguous():
        q = q.float().contiguous()
    return q, dueling


def apex_columns(channels_last=False, frames_u8=False, frame_store=False):
    """replay columns of the apex-dqn rows [s0, a, r, s1, done] (worker.py:47-51): frames are
    stored uint8 and sampled as float32 (exact), the rest as the reference casts them.
    frames_u8: s0 / s1 are sampled as the stored uint8 stacks -- the HIP conv torso reads
    them directly (forward, and conv1's weight gradient), widening in registers (the same
    values at a quarter of the bytes)"""
    from .replay import Column, FrameColumn
    if frame_store:  # frame de-duplicated: frame ids, sampled as the uint8 stacks
        if not frames_u8:
            raise ValueError("the frame store samples uint8 stacks (frames_u8)")
        fr = lambda: FrameColumn(OBS_SHAPE)
    else:
        fr = lambda: Column(OBS_SHAPE, torch.uint8) if frames_u8 else Column(OBS_SHAPE, torch.uint8, torch.float32,
                                                                             channels_last=channels_last)
    return [fr(), Column((), torch.int64), Column((), torch.float32), fr(), Column((), torch.float32)]
