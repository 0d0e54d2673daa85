"""Ape-X DQN on one GPU (one process per GPU; N GPUs = N of these + a gradient all-reduce).

Reference wiring (test/apex-dqn/): trainer.py:19-41 (learner loop: loader.sample ->
Trainer.step -> Client.update_priorities, weights every send_weights_interval updates),
worker.py:21-61 (actor loop), config.yaml (hyper-parameters, defaults below), trainer.py:
52-61 (K replay shards of C // K).

Per GPU, everything lives in HBM: the actors' frame rings and n-step deques, the replay
shard (storage + sum-tree + its device-resident sampler state), the learner's networks and
the actors' weight copy.  One iteration = `actor_steps_per_update` vectorised actor steps
(N env steps each) + one learner update, in this order:

    actor compute (act, env, n-step, priorities)   append(t)
    learner train on batch k (forward, TD, backward, clip, Adam)
    sample + gather batch k+1                      update_priorities(k)

The replay/tree operations run in the reference's order: batch k+1 is sampled before batch
k's priorities land (the sampler's HWM-1 PUSH, server/sampler_loop.py:13-15, 36-39).

With `hip_graph` the two compute blocks are captured once (the learner's in two copies, one
per batch-slot parity) and replayed every iteration; the handful of replay-tree launches
between them stay eager, so the tree-op order, the host counters and the HIP-event timing
of the gather are exactly those of the eager schedule.  All per-step scalars the kernels
need (FIFO tail, Philox counters, beta schedule step, env step) live in device memory, so
the captured launches are valid on every replay.
"""
from dataclasses import dataclass, field
from typing import Optional

import torch

from .actors import OBS_SHAPE, VecActors, apex_columns
from .dist import GradAllReduce
from .model import DQNNetwork
from .replay import HbmReplay
from .reth_buffer import TorchCudaLoader, _SERVICES, start_per
from .solver import Box, DQNSolver, Discrete
from .trainer import Trainer
from .weights import WeightsSlot, WeightsSubscriber

# Every capture is thread-local: in the default global mode a stream-unsafe HIP call from ANY
# thread during a capture is an error, and with a process group alive the RCCL watchdog thread
# polls its collectives' end events (hipEventQuery) at any time -- a poll that lands inside one
# of the learner's captures aborted the process (test_rccl_gpu, r05).  Thread-local mode keeps
# the check for this (the capturing) thread only.
_CAPTURE_MODE = "thread_local"


def _end_part(parts, stream):
    """end the capture of parts[-1] on `stream`.  A part with nothing captured (two graph
    boundaries back to back: a probed launch right before a gradient bucket, say) is proved
    empty by the stream's capture state -- no node for the next capture to depend on
    (rth_stream_capture_deps == 0) -- and becomes None, skipped at replay, instead of an empty
    graph (torch warns "The CUDA Graph is empty" for one, the warning that also flags a capture
    on the wrong stream, which this check would not hide: that part's launches leave the
    capturing stream with no node either, but they then run eagerly right here, and the
    probe-copy test compares every result against the uncut graph's)."""
    import warnings

    from . import _lib

    empty = _lib.lib().rth_stream_capture_deps(stream.cuda_stream) == 0  # (< 0: not capturing, or an error)
    if not empty:
        parts[-1].capture_end()
        return
    with warnings.catch_warnings():
        warnings.filterwarnings("ignore", message="The CUDA Graph is empty")
        parts[-1].capture_end()
    parts[-1] = None


@dataclass
class ApexConfig:
    n_actors: int = 256            # actors on this GPU (BASELINE configs[1]: 256 vectorised actors)
    num_actions: int = 6           # Pong
    capacity: int = 1_000_000      # replay capacity of this GPU's shard
    batch_size: int = 512          # common.batch_size
    n_step: int = 3
    gamma: float = 0.99
    alpha: float = 0.5
    beta: str = "0.4,1,2000000"
    learning_rate: float = 1e-4
    adam_epsilon: float = 1.5e-4
    clip_value: float = 40.0
    update_target_interval: int = 100
    send_weights_interval: int = 10
    recv_weights_interval: int = 400
    actor_steps_per_update: int = 1
    sample_start: int = 1000
    seed: int = 0
    p_reward: float = 0.02
    p_done: float = 1.0 / 2000
    nstep_mode: int = 0            # 0 = numpy-1.19 promotion (the reference's pin)
    fused_adam: bool = True
    channels_last: bool = True     # NHWC end to end (gather writes it, MIOpen consumes it)
    conv_benchmark: bool = False   # torch.backends.cudnn.benchmark (MIOpen find)
    hip_graph: bool = False        # replay captured HIP graphs of the compute blocks
    fused_actor: bool = True       # act + previous rows' priorities in one 3N forward (VecActors.step_fused)
    overlap: bool = True           # graph mode: actor block and learner block on two streams, concurrently
    hip_conv: bool = True          # conv torso forward in rth_conv_bias_relu (actors/targets read uint8 stacks)
    dp_hook: Optional[bool] = None  # gradient all-reduce hook: None = when world > 1 (tests force it)
    tuned_gemm: bool = True        # TunableOp solution selection for the library GEMMs (reth_amd.gemm_tuning)
    env: str = "synthetic"         # actors' observations: synthetic | atari | atari-h2d (VecActors)
    frame_store: bool = False      # frame de-duplicated replay: each frame stored once, rows as frame ids
    frame_store_bound: str = "hard"  # store size: "hard" (worst case, 2 frames per actor step) | "expected" (p_done)
    frame_ids: bool = True         # frame store: batches hold frame ids, conv1 reads the frames in place (no stacks)
    extra: dict = field(default_factory=dict)


class _Quiet:
    def info(self, *a, **k):
        pass


class ApexDQN:
    def __init__(self, cfg: ApexConfig, device=None, rank=0, world=1, group=None, logger=None):
        self.cfg = cfg
        self.device = torch.device(device if device is not None else "cuda")
        self.rank, self.world = rank, world
        use_hook = world > 1 if cfg.dp_hook is None else cfg.dp_hook
        hook = GradAllReduce(group, force=bool(cfg.dp_hook)) if use_hook else None
        torch.backends.cudnn.benchmark = bool(cfg.conv_benchmark)
        if cfg.tuned_gemm:
            from . import gemm_tuning

            gemm_tuning.enable()
        fmt = torch.channels_last if cfg.channels_last else torch.contiguous_format
        torch.manual_seed(cfg.seed)  # identical initial weights on every rank
        self.solver = DQNSolver(Box(0, 255, OBS_SHAPE), Discrete(cfg.num_actions), gamma=cfg.gamma,
                                clip_value=cfg.clip_value, double_q=True, dueling=True,
                                learning_rate=cfg.learning_rate, adam_epsilon=cfg.adam_epsilon,
                                update_target_interval=cfg.update_target_interval, device=self.device,
                                n_step=cfg.n_step, fused_adam=cfg.fused_adam, grad_hook=hook,
                                channels_last=cfg.channels_last, capturable=cfg.hip_graph)
        self.trainer = Trainer(self.solver, logger=logger or _Quiet(), print_interval=1000)
        self.actor_net = DQNNetwork(OBS_SHAPE, cfg.num_actions).to(self.device, memory_format=fmt)
        self.actor_net.requires_grad_(False)
        self.actor_net.hwc_features = bool(cfg.channels_last)
        for net in (self.actor_net, self.solver.q_network, self.solver.target_q_network):
            net.hip_conv = bool(cfg.hip_conv)
        self.slot = WeightsSlot(self.solver.q_network)
        self.slot.copy_out(self.actor_net)  # the actors start from the learner's initial weights
        self.subscriber = WeightsSubscriber(self.slot, cfg.recv_weights_interval)
        self.actors = VecActors(cfg.n_actors, cfg.num_actions, cfg.n_step, cfg.gamma, self.device,
                                seed=cfg.seed * 1000003 + rank, actor_offset=rank * cfg.n_actors,
                                total_actors=cfg.n_actors * world, p_reward=cfg.p_reward, p_done=cfg.p_done,
                                nstep_mode=cfg.nstep_mode, channels_last=cfg.channels_last, env=cfg.env)
        self.svc, self.addr = start_per(cfg.capacity, cfg.batch_size, alpha=cfg.alpha, beta=cfg.beta,
                                        sample_start=cfg.sample_start, device=self.device, seed=cfg.seed + 7919 * rank)
        u8 = bool(cfg.hip_conv and cfg.channels_last)
        self.svc.replay = HbmReplay(cfg.capacity, apex_columns(cfg.channels_last, frames_u8=u8,
                                                               frame_store=cfg.frame_store),
                                    cfg.alpha, cfg.beta, self.device, seed=cfg.seed + 7919 * rank,
                                    frame_store=self.frame_store_frames(cfg) if cfg.frame_store else None)
        self.replay = self.svc.replay
        if cfg.frame_store:
            self.actors.attach_frame_store(self.replay)
            if cfg.frame_ids and u8:  # the sampled batches are FrameStacks (fused_learner reads them in place)
                self.replay.set_frame_ids(True)
        self.loader = TorchCudaLoader(self.addr, buffer_size=2, prefetch=1)
        self.env_steps = 0
        self.updates = 0
        self._graphs = None
        self._ev_acquired = None
        self.actor_modes = {}  # graph mode: actor steps replayed per mode ("dedup" / "full")
        self.conv_probe = None  # extra["probe_conv2"]: callable(tag) between the learner graph's parts

    @staticmethod
    def frame_store_frames(cfg):
        """frames the store must hold (rth_replay_frames_attach): every frame a live row
        references.  A row lives capacity / N actor steps after its append and its oldest
        frame is at most n + 4 steps older than the append.  Each step adds N frames plus one
        per ended episode, so at most 2 N: "hard" sizes for that worst case -- 2 capacity +
        2 (n + 16 + 2 a) N with a = actor_steps_per_update, no frame a live row references is
        ever overwritten, whatever the episode lengths (Pong 1 M rows: 14.1 GB of frames;
        Breakout 4 M: 56.5 GB).  With frame ids (cfg.frame_ids) the learner reads a sampled
        row's frames at learner time, not at gather time: the batch is sampled one iteration
        ahead (sample-ahead), so up to 2 a actor steps run between a row's sampling -- when it is
        still live, possibly the oldest -- and conv1's read of its frames, and the 2 a term keeps
        those frames in the store over that window (12 steps of slack beyond it, the n + 16 vs
        n + 4).  "expected" sizes for
        the i.i.d. episode-end rate p_done instead -- capacity (1 + 2 p_done), at least
        capacity / 64 of headroom, + (n + 16) N: half the bytes, but a burst of episode ends
        beyond that rate would overwrite frames that old rows still name."""
        if cfg.frame_store_bound == "hard":
            return 2 * cfg.capacity + 2 * (cfg.n_step + 16 + 2 * cfg.actor_steps_per_update) * cfg.n_actors + 16
        if cfg.frame_store_bound != "expected":
            raise ValueError(f"frame_store_bound {cfg.frame_store_bound!r}: 'hard' or 'expected'")
        reset = max(cfg.capacity // 64, int(2 * cfg.capacity * cfg.p_done) + 1)
        # + 8 N: the actors' initial stacks, pushed at construction and again behind a prefill
        return cfg.capacity + reset + (cfg.n_step + 16) * cfg.n_actors + 16

    def close(self):
        _SERVICES.pop(self.addr, None)
        self._graphs = None
        if self.cfg.tuned_gemm:
            from . import gemm_tuning

            gemm_tuning.restore()

    # ------------------------------------------------------------------ replay prefill
    @torch.no_grad()
    def prefill(self, n_rows, chunk=16384):
        """bulk-fill the shard with synthetic rows (uniform uint8 frames, |td| ~ U(0,1]) through
        the real append path -- the state of a replay that has run for a while"""
        g = torch.Generator(device=self.device)
        g.manual_seed(self.cfg.seed + 17 * self.rank)
        done = 0
        if self.replay.frames is not None:
            return self._prefill_frames(n_rows, g, chunk)
        while done < n_rows:
            m = min(chunk, n_rows - done)
            s0 = torch.randint(0, 256, (m, *OBS_SHAPE), dtype=torch.uint8, device=self.device, generator=g)
            s1 = torch.randint(0, 256, (m, *OBS_SHAPE), dtype=torch.uint8, device=self.device, generator=g)
            a = torch.randint(0, self.cfg.num_actions, (m,), dtype=torch.int64, device=self.device, generator=g)
            r = (torch.rand(m, device=self.device, generator=g) < self.cfg.p_reward).float()
            d = (torch.rand(m, device=self.device, generator=g) < self.cfg.p_done).float()
            td = 1.0 - torch.rand(m, device=self.device, generator=g)  # (0, 1]
            self.replay.append([s0, a, r, s1, d], td)
            done += m

    @torch.no_grad()
    def _prefill_frames(self, n_rows, g, chunk):
        """the frame store's prefill: one long synthetic trajectory -- n_rows + 7 uniform uint8
        frames behind the store's head, row j's s0 = frames j .. j+3 and s1 = frames j+3 .. j+6
        of it (an n = 3 step apart, as the actors' rows are) -- then the head moves past them,
        so the actors' frames overwrite them in the order the FIFO overwrites their rows"""
        store, K = self.replay.frames, OBS_SHAPE[0]
        F = store.shape[0]
        base = int(self.replay.frame_head)  # behind the frames already pushed (the actors' stacks)
        nf = n_rows + 2 * K - 1
        if base + nf > F:
            raise ValueError(f"prefill of {n_rows} rows needs {nf} frames behind {base}, the store holds {F}")
        for f0 in range(0, nf, chunk):
            m = min(chunk, nf - f0)
            store[base + f0:base + f0 + m] = torch.randint(0, 256, (m, *store.shape[1:]), dtype=torch.uint8,
                                                           device=self.device, generator=g)
        self.replay.frame_head.fill_(base + nf)
        done = 0
        while done < n_rows:
            m = min(chunk, n_rows - done)
            j = torch.arange(base + done, base + done + m, dtype=torch.int32, device=self.device)[:, None]
            ks = torch.arange(K, dtype=torch.int32, device=self.device)[None, :]
            s0, s1 = (j + ks).contiguous(), (j + K - 1 + ks).contiguous()
            a = torch.randint(0, self.cfg.num_actions, (m,), dtype=torch.int64, device=self.device, generator=g)
            r = (torch.rand(m, device=self.device, generator=g) < self.cfg.p_reward).float()
            d = (torch.rand(m, device=self.device, generator=g) < self.cfg.p_done).float()
            td = 1.0 - torch.rand(m, device=self.device, generator=g)  # (0, 1]
            self.replay.append([s0, a, r, s1, d], td)
            done += m
        # the actors' current stacks enter again, behind the prefill: frames are overwritten in
        # push order, and the first rows the actors append reference these
        if self.actors.pushes:
            raise RuntimeError("prefill a frame-store replay before the actors step")
        self.actors.attach_frame_store(self.replay)

    # ------------------------------------------------------------------ the blocks
    def _actor_compute(self):
        """act + env + n-step (+ priorities once rows flow); returns (|td|, rows) of the rows
        to append (the previous step's with fused_actor, this step's otherwise) or (None, None)"""
        if self.cfg.fused_actor:
            return self.actors.step_fused(self.actor_net)
        if self.actors.step(self.actor_net):
            return self.actors.prioritise(self.actor_net), None
        return None, None

    def _learner_train(self, slot):
        data, idx, isw = slot
        return self.trainer.train(data, weights=isw)

    def _actor_host(self):
        """host-side actor bookkeeping between steps (weights reload: perwez RecvSocket)"""
        if self.subscriber.maybe_load(self.actor_net, self.actors.t):
            self.actors.weights_changed()
            # the learner's next publish (another stream in overlapped graph mode) must not
            # overwrite the slot before this copy out of it has run
            self._ev_acquired = torch.cuda.Event()
            self._ev_acquired.record()

    def _learner_host(self):
        """host-side learner bookkeeping after an update (Trainer / Interval / weights send)"""
        self.trainer.account()
        self.updates += 1
        if self.solver._update_target_interval is not None and not self.solver.auto_target_update:
            self.solver._update_target_interval()
        if self.updates % self.cfg.send_weights_interval == 0:
            if self._ev_acquired is not None:
                torch.cuda.current_stream(self.device).wait_event(self._ev_acquired)
            self.slot.publish(self.solver.q_network)

    # ------------------------------------------------------------------ iteration
    def iteration(self):
        """one Ape-X iteration, enqueued on this object's own stream (the stream the graphs
        are captured from); callers synchronise with torch.cuda.synchronize()"""
        if not hasattr(self, "_stream"):
            self._stream = torch.cuda.Stream(self.device, priority=self.cfg.extra.get("actor_priority", 0))
            self._stream.wait_stream(torch.cuda.current_stream(self.device))  # init + prefill
        with torch.cuda.stream(self._stream):
            self._iteration()

    def _iteration(self):
        if self._graphs is None and self.cfg.hip_graph and self._graph_ready():
            self._capture()
        if self._graphs is not None:
            return self._iteration_graph()
        for _ in range(self.cfg.actor_steps_per_update):
            self._actor_host()
            td, rows = self._actor_compute()
            if td is not None:
                self.actors.append(self.replay, td, rows)
            self.env_steps += self.actors.N
        if not self.svc.ready():
            return
        if not self.loader.pending():
            self.loader.issue()
        slot = self.loader.take()
        td = self._learner_train(slot)
        self.loader.issue()  # sample-ahead: batch k+1 before batch k's priorities land
        self.replay.update_priorities(slot[1], td, step=True, deferred=True)  # merged into the next append
        self._learner_host()

    # ------------------------------------------------------------------ graph replay
    def _graph_ready(self):
        # capture once the actors emit rows every step, the learner has run eagerly (optimizer
        # state exists, MIOpen has chosen its kernels) and a batch is pending
        return self.actors.warm and self.updates >= 2 and self.loader.pending() == 1

    def _capture(self):
        """Capture the actor block and the learner block (one per batch-slot parity).  With a
        process group the learner is captured in parts cut at each final gradient bucket, and
        the RCCL all-reduces run eagerly between them (_learner_replay)."""
        solver = self.solver
        solver.auto_target_update = False
        slots = self.loader._slots
        tun = torch.cuda.tunable
        tuning = tun.is_enabled() and tun.tuning_is_enabled()
        if tuning:  # a GEMM shape first seen inside the capture must not be benchmarked there
            tun.tuning_enable(False)
        try:
            self._capture_graphs(solver, slots)
        finally:
            if tuning:
                tun.tuning_enable(True)

    def _capture_graphs(self, solver, slots):
        host = (self.actors.t, self.actors.pushes)
        side = torch.cuda.Stream(self.device)
        side.wait_stream(torch.cuda.current_stream(self.device))
        split = solver.grad_hook is not None
        G = dict(act=[], act_out=[], tgt=[], q1t=[], learn={}, learn_td={}, buckets={}, grads={})
        # probe sets (extra["probe_conv2"]): a second copy of the actor and learner graphs, cut
        # at the launches the bench times live (conv2 / conv3, the TD/heads backward, clip+Adam,
        # the actor tail) -- replayed only while conv_probe is set, so the headline window
        # replays the uncut graphs
        psets = [False, True] if self.cfg.extra.get("probe_conv2") else [False]
        with torch.cuda.stream(side):
            # the actor block by (mode, push parity): fused_actor alternates row sets; mode
            # "dedup" takes the rows' heads from the per-stack cache (VecActors.step_fused),
            # "full" runs them through the network (after a weights reload)
            act = self.actors
            fresh = act.fresh
            modes = ["full"] + (["dedup"] if self.cfg.fused_actor and act._hip_heads(self.actor_net) else [])
            G["act"], G["act_out"] = {}, {}
            for pr in psets:
                for mode in modes:
                    for _ in range(2):
                        k = act.pushes % 2
                        act.fresh = act.n_step + 2 if mode == "dedup" else 0
                        key = ("probe", mode, k) if pr else (mode, k)
                        if pr and self.cfg.fused_actor:
                            parts, bounds = [torch.cuda.CUDAGraph()], []
                            pool = parts[0]

                            def cut(item, parts=parts, bounds=bounds, pool=pool):
                                _end_part(parts, side)
                                bounds.append(("probe", item))
                                parts.append(torch.cuda.CUDAGraph())
                                parts[-1].capture_begin(pool=pool.pool(), capture_error_mode=_CAPTURE_MODE)

                            parts[0].capture_begin(capture_error_mode=_CAPTURE_MODE)
                            out = act.step_fused(self.actor_net, dedup=mode == "dedup", probe=cut)
                            _end_part(parts, side)
                            G["act"][key] = (parts, bounds)
                        else:
                            g = torch.cuda.CUDAGraph()
                            with torch.cuda.graph(g, stream=side, capture_error_mode=_CAPTURE_MODE):
                                out = (act.step_fused(self.actor_net, dedup=mode == "dedup") if self.cfg.fused_actor
                                       else self._actor_compute())
                            G["act"][key] = g
                        G["act_out"][key] = out
            act.fresh = fresh
            # the target network's output on each slot's s1, computed on the actor stream ahead
            # of the update (target_heads); "pre" learner graphs consume it, "full" ones
            # compute it themselves (after a target sync, and before any was precomputed).
            # Captured from a stream of its own: FC1's split-K workspace is keyed by the
            # capturing stream (model._fc_workspace), and the learner's "full" variant runs the
            # same target pass concurrently on the learner stream -- one shared workspace would
            # mix the two launches' partials
            side_tgt = torch.cuda.Stream(self.device)
            side_tgt.wait_stream(side)
            for p in range(2):
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g, stream=side_tgt, capture_error_mode=_CAPTURE_MODE):
                    q1t = solver.target_heads(slots[p][0][3])
                G["tgt"].append(g)
                G["q1t"].append(q1t)
            side.wait_stream(side_tgt)
            for pr, variant, p in [(pr, variant, p) for pr in psets for variant in ("full", "pre") for p in range(2)]:
                    v = ("probe", variant, p) if pr else (variant, p)
                    parts, bounds = [torch.cuda.CUDAGraph()], []
                    pool = parts[0]

                    ended = []

                    def cut(item, last=False, parts=parts, bounds=bounds, ended=ended, pool=pool):
                        # end this part of the learner graph at a boundary: ("bucket", a final
                        # gradient bucket -- its all-reduce runs between the parts, overlapping
                        # the next one) or ("probe", [(tag, launch), ...]) -- launches issued eagerly
                        # between the parts at every replay, each bracketed by the bench's HIP events).
                        # last: nothing is captured after this boundary, so no (empty) part follows;
                        # a part with nothing in it becomes None (_end_part)
                        _end_part(parts, side)
                        bounds.append(item)
                        if last:
                            ended.append(True)
                            return
                        parts.append(torch.cuda.CUDAGraph())
                        parts[-1].capture_begin(pool=pool.pool(), capture_error_mode=_CAPTURE_MODE)

                    parts[0].capture_begin(capture_error_mode=_CAPTURE_MODE)
                    data, idx, isw = slots[p]
                    probe = (lambda items, last=False: cut(("probe", items), last=last)) if pr else None
                    td = solver.compute_grads(data, isw, q1t=G["q1t"][p] if variant == "pre" else None,
                                              mid=(lambda b: cut(("bucket", b))) if split else None, probe=probe,
                                              prenorm=not split)
                    self.trainer._track(td)
                    if split and not any(k == "bucket" for k, _ in bounds):  # autograd path: one bucket
                        cut(("bucket", [q.grad for q in solver._params]))
                    solver.apply_grads(probe=probe)
                    if not ended:
                        _end_part(parts, side)
                    G["learn"][v], G["buckets"][v], G["learn_td"][v] = parts, bounds, td
                    G["grads"][v] = [q.grad for q in solver._params]  # what apply_grads consumed
        torch.cuda.current_stream(self.device).wait_stream(side)
        self.actors.t, self.actors.pushes = host  # capture recorded, did not run, the steps
        self._graphs = G

    def _iteration_graph(self):
        if self.cfg.overlap:
            return self._iteration_graph_overlap()
        G = self._graphs
        act = self.actors
        self._actor_block_graph()
        k = self.loader._pending.pop(0)
        v = self._learner_key(("full", k))
        self._learner_replay(v)
        self.loader.issue()  # sample-ahead into the other slot
        self.replay.update_priorities(self.loader._slots[k][1], G["learn_td"][v], step=True, deferred=True)
        self._learner_host()

    def upload_graphs(self):
        """hipGraphUpload every captured graph (actor blocks, target passes, learner parts, the
        probe copies) on this object's stream, then wait: returns the number uploaded"""
        from . import _lib

        G = self._graphs
        if G is None:
            return 0
        graphs = list(G["tgt"])
        for g in G["act"].values():
            graphs += g[0] if isinstance(g, tuple) else [g]
        for parts in G["learn"].values():
            graphs += list(parts)
        graphs = [g for g in graphs if g is not None]  # (empty parts: _end_part)
        st = self._stream if hasattr(self, "_stream") else torch.cuda.current_stream(self.device)
        for g in graphs:
            _lib.call("rth_graph_upload", g.raw_cuda_graph_exec(), st.cuda_stream)
        st.synchronize()
        return len(graphs)

    def _probing(self):
        return self.conv_probe is not None and self.cfg.extra.get("probe_conv2")

    def _learner_key(self, v):
        """the learner graph to replay for variant v: its probe copy while the bench probes"""
        return ("probe", *v) if self._probing() and ("probe", *v) in self._graphs["learn"] else v

    def _replay_parts(self, parts, bounds):
        """replay a graph captured in parts; between them the probed launches, each bracketed
        by conv_probe(tag) / conv_probe(tag + "_end")"""
        for i, g in enumerate(parts):
            if g is not None:
                g.replay()
            if i < len(bounds):
                for tag, fn in bounds[i][1]:
                    self.conv_probe(tag)
                    fn()
                    self.conv_probe(tag + "_end")

    def _learner_replay(self, v):
        """replay learner graph v on the current stream.  Its parts are cut at boundaries:
        gradient buckets (data-parallel learner: every bucket but the last is all-reduced on a
        side stream while the following part runs -- the merged heads' gradients, 95 % of the
        bytes, under the conv backward; the last one on this stream; the final part (heads
        split + clip + Adam) waits for all of them) and probes (launches issued eagerly between
        the parts, each bracketed by conv_probe(tag) / conv_probe(tag + "_end"): the bench
        records HIP events there on this stream for its live per-launch timing)."""
        G = self._graphs
        parts, bounds = G["learn"][v], G["buckets"][v]
        if any(kind == "probe" for kind, _ in bounds):
            # a launch issued between the parts (clip + Adam) reads the parameters' .grad when it
            # runs: point them at this variant's gradient buffers (each captured variant has its
            # own; the last capture left .grad on the last variant's)
            for q, g in zip(self.solver._params, G["grads"][v]):
                q.grad = g
        if not bounds:
            if parts[0] is not None:
                parts[0].replay()
            return
        hook = self.solver.grad_hook
        cur = torch.cuda.current_stream(self.device)
        bucket_at = [i for i, (kind, _) in enumerate(bounds) if kind == "bucket"]
        comm = None
        for i, (g, (kind, item)) in enumerate(zip(parts, bounds)):
            if g is not None:
                g.replay()
            if kind == "probe":  # launches issued between the parts, optionally between HIP events
                for tag, fn in item:
                    if self.conv_probe is not None:
                        self.conv_probe(tag)
                    fn()
                    if self.conv_probe is not None:
                        self.conv_probe(tag + "_end")
                continue
            key = ("bucket", bucket_at.index(i))
            if i != bucket_at[-1]:
                if comm is None:
                    if not hasattr(self, "_stream_comm"):
                        self._stream_comm = torch.cuda.Stream(self.device)
                    comm = self._stream_comm
                comm.wait_stream(cur)
                with torch.cuda.stream(comm):
                    hook.reduce(item, key=key)
            else:
                hook.reduce(item, key=key)
                # everything after the last bucket (heads split, clip + Adam -- replayed or, in a
                # probe copy, issued eagerly between parts) reads the side stream's buckets
                if comm is not None:
                    cur.wait_stream(comm)
                    comm = None
        if comm is not None:
            cur.wait_stream(comm)
        if len(parts) > len(bounds) and parts[-1] is not None:  # (a probe copy may end at its last probed launch)
            parts[-1].replay()

    def _actor_block_graph(self):
        G, act = self._graphs, self.actors
        for _ in range(self.cfg.actor_steps_per_update):
            self._actor_host()
            k = act.pushes % 2
            mode = "dedup" if ("dedup", k) in G["act"] and act.dedup_ready(self.actor_net) else "full"
            key = ("probe", mode, k) if self._probing() and ("probe", mode, k) in G["act"] else (mode, k)
            g = G["act"][key]
            if isinstance(g, tuple):  # a probe set: parts with the timed launches between them
                self._replay_parts(*g)
            else:
                g.replay()
            self.actor_modes[mode] = self.actor_modes.get(mode, 0) + 1
            act.t += 1
            act.pushes += 1
            act.fresh += 1
            td, rows = G["act_out"][key]
            if self.cfg.fused_actor:
                act._bind_rows(act._sets[k])
                if act.pushes - 1 > act.n_step:
                    act.append(self.replay, td, rows)
            else:
                act.append(self.replay, td)
            self.env_steps += act.N

    def actor_iteration(self):
        """the actor block alone (learner idle): `actor_steps_per_update` vectorised actor
        steps with their appends -- the decoupled actors' capacity (Ape-X runs actors and
        learner independently; worker.py:21-61 never waits for the trainer).  Graph mode only."""
        if self._graphs is None:
            raise RuntimeError("actor_iteration replays the captured actor graphs: run iteration() until captured")
        with torch.cuda.stream(self._stream):
            if hasattr(self, "_ev_learn"):
                self._stream.wait_event(self._ev_learn)
            self._actor_block_graph()

    def _next_learner_variant(self):
        """graph key of the next replayed learner step: (full | pre, batch slot)"""
        k = self.loader._pending[0]
        ready = getattr(self, "_q1t_ready", None)
        return ("pre" if self.cfg.overlap and ready is not None and ready[k] else "full", k)

    def _iteration_graph_overlap(self):
        """The actor block (stream A: act + env + n-step + append, then the sample of batch
        k+1) runs concurrently with the learner block of batch k (stream B: forward/backward,
        Adam, target sync, weights publish).  Cross-stream edges, all one iteration apart:
        A waits for learner k-1 (its |td| merges into this append, its batch slot is
        resampled, its weights may be loaded by the actors); B waits for sample k.  The
        replay's operations keep the single-stream order on A."""
        G = self._graphs
        A = self._stream
        if not hasattr(self, "_stream_b"):
            # both streams at normal priority: a high-priority learner stream (-1) gives the same
            # step time and a slower in-loop gather (40 vs 33-35 us)
            self._stream_b = torch.cuda.Stream(self.device, priority=self.cfg.extra.get("learner_priority", 0))
            self._ev_learn = torch.cuda.Event()
            self._ev_sample = torch.cuda.Event()
            self._ev_sample.record(A)  # batch k was sampled on A before the first overlapped step
            self._ev_learn.record(A)
            self._q1t_ready = [False, False]  # per slot: its target pass was precomputed on A
        B = self._stream_b
        A.wait_event(self._ev_learn)
        self._actor_block_graph()  # on A (the caller's stream)
        k = self.loader._pending.pop(0)
        v = self._learner_key(("pre" if self._q1t_ready[k] else "full", k))
        self._q1t_ready[k] = False
        syncs = self.solver._target_syncs
        with torch.cuda.stream(B):
            B.wait_event(self._ev_sample)
            self._learner_replay(v)  # on B
            self._learner_host()  # target sync / weights publish copies: on B
            self._ev_learn.record(B)
        self.loader.issue()  # sample-ahead into the other slot (on A, after this step's append)
        if self.solver._target_syncs == syncs:
            # no target sync in this step: the next batch's target pass runs here on A,
            # concurrently with the learner (the target weights do not change before it is used)
            kn = self.loader._pending[-1]
            G["tgt"][kn].replay()
            self._q1t_ready[kn] = True
        self._ev_sample.record(A)
        self.replay.update_priorities(self.loader._slots[k][1], G["learn_td"][v], step=True, deferred=True)
