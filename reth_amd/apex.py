"""Ape-X DQN on one GPU (one process per GPU; N GPUs = N of these + a gradient all-reduce).

Reference wiring (test/apex-dqn/): trainer.py:19-41 (learner loop: loader.sample ->
Trainer.step -> Client.update_priorities, weights every send_weights_interval updates),
worker.py:21-61 (actor loop), config.yaml (hyper-parameters, defaults below), trainer.py:
52-61 (K replay shards of C // K).

Per GPU, everything lives in HBM: the actors' frame rings and n-step deques, the replay
shard (storage + sum-tree), the learner's networks and the actors' weight copy.  One
iteration = `actor_steps_per_update` vectorised actor steps (N env steps each) + one
learner update.  The stream order reproduces the reference's sampler semantics: the next
batch is sampled before the current batch's priorities are written back (HWM-1 PUSH).
"""
from dataclasses import dataclass, field

import torch

from .actors import OBS_SHAPE, VecActors, apex_columns
from .dist import GradAllReduce
from .model import DQNNetwork
from .replay import HbmReplay
from .reth_buffer import TorchCudaLoader, start_per, _SERVICES
from .solver import Box, DQNSolver, Discrete
from .trainer import Trainer
from .weights import WeightsSlot, WeightsSubscriber


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
    prefetch: int = 1
    fused_adam: bool = True
    extra: dict = field(default_factory=dict)


class _Quiet:
    def info(self, *a, **k):
        pass


class ApexDQN:
    def __init__(self, cfg: ApexConfig, device=None, rank=0, world=1, group=None, logger=None):
        self.cfg = cfg
        self.device = torch.device(device if device is not None else "cuda")
        self.rank, self.world = rank, world
        hook = GradAllReduce(group) if world > 1 else None
        torch.manual_seed(cfg.seed)  # identical initial weights on every rank
        self.solver = DQNSolver(Box(0, 255, OBS_SHAPE), Discrete(cfg.num_actions), gamma=cfg.gamma,
                                clip_value=cfg.clip_value, double_q=True, dueling=True,
                                learning_rate=cfg.learning_rate, adam_epsilon=cfg.adam_epsilon,
                                update_target_interval=cfg.update_target_interval, device=self.device,
                                n_step=cfg.n_step, fused_adam=cfg.fused_adam, grad_hook=hook)
        self.trainer = Trainer(self.solver, logger=logger or _Quiet(), print_interval=1000)
        self.actor_net = DQNNetwork(OBS_SHAPE, cfg.num_actions).to(self.device).requires_grad_(False)
        self.slot = WeightsSlot(self.solver.q_network)
        self.slot.acquire(self.actor_net)
        self.subscriber = WeightsSubscriber(self.slot, cfg.recv_weights_interval)
        self.actors = VecActors(cfg.n_actors, cfg.num_actions, cfg.n_step, cfg.gamma, self.device,
                                seed=cfg.seed * 1000003 + rank, actor_offset=rank * cfg.n_actors,
                                total_actors=cfg.n_actors * world, p_reward=cfg.p_reward, p_done=cfg.p_done,
                                nstep_mode=cfg.nstep_mode)
        self.svc, self.addr = start_per(cfg.capacity, cfg.batch_size, alpha=cfg.alpha, beta=cfg.beta,
                                        sample_start=cfg.sample_start, device=self.device, seed=cfg.seed + 7919 * rank)
        self.svc.replay = HbmReplay(cfg.capacity, apex_columns(), cfg.alpha, cfg.beta, self.device,
                                    seed=cfg.seed + 7919 * rank)
        self.replay = self.svc.replay
        self.loader = TorchCudaLoader(self.addr, buffer_size=cfg.prefetch + 1, prefetch=cfg.prefetch)
        self.env_steps = 0
        self.updates = 0

    def close(self):
        _SERVICES.pop(self.addr, None)

    # ------------------------------------------------------------------ replay prefill
    @torch.no_grad()
    def prefill(self, n_rows, chunk=16384):
        """bulk-fill the shard with synthetic rows (uniform uint8 frames, |td| ~ U(0,1]) through
        the real append path -- the state of a replay that has run for a while"""
        g = torch.Generator(device=self.device)
        g.manual_seed(self.cfg.seed + 17 * self.rank)
        done = 0
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

    # ------------------------------------------------------------------ loop
    def actor_step(self):
        self.subscriber.maybe_load(self.actor_net, self.actors.t)
        if self.actors.step(self.actor_net):
            td = self.actors.prioritise(self.actor_net)
            self.actors.append(self.replay, td)
        self.env_steps += self.actors.N

    def learner_step(self):
        data, idx, isw = self.loader.sample_device()
        td = self.trainer.step(data, weights=isw, device_result=True)
        self.replay.update_priorities(idx, td, step=True)
        self.updates += 1
        if self.updates % self.cfg.send_weights_interval == 0:
            self.slot.publish(self.solver.q_network)

    def iteration(self):
        for _ in range(self.cfg.actor_steps_per_update):
            self.actor_step()
        if self.svc.ready():
            self.learner_step()
