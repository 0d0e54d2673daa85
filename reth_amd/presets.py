"""reth.presets on top of the HIP path: Worker, exploration and the YAML factories.

Reference: reth/reth/presets/worker.py:12-163 (Worker), reth/reth/utils/exploration.py:16-31
(RandomExploration), reth/reth/presets/config.py:12-73 (get_env / get_solver / get_worker /
get_trainer / get_replay_buffer).  The worker steps a host environment (the reference's
examples run one gym env per process); the solver, buffers and trainer are the device
ones (DQNSolver, reth_amd.buffer, Trainer).
"""
import io
import os
import time

import numpy as np
import yaml

from . import envs
from .buffer import DynamicSizeBuffer, NumpyBuffer, PrioritizedBuffer
from .schedule import Interval, Schedule
from .solver import get_solver as _get_solver
from .trainer import Trainer, getLogger


class RandomExploration:
    """exploration.py:16-31: epsilon from a Schedule stepped per act"""

    def __init__(self, solver, action_space, epsilon=0):
        self.solver, self.action_space = solver, action_space
        self.schedule = Schedule.from_str(epsilon)

    def act(self, state):
        eps = self.schedule.step()
        if np.random.rand() < eps:
            return int(np.random.randint(self.action_space.n))
        return self.solver.act(state)


class Worker:
    """worker.py:12-163 (exploration given as a number / schedule string or an object)"""

    def __init__(self, env, solver, logger=None, exploration=None, print_interval=500, device=None):
        self.env, self.solver = env, solver
        self.logger = logger if logger is not None else getLogger("worker")
        self.device = device if device is not None else getattr(solver, "device", None)
        self.s0 = self.env.reset()
        self.cur_step, self.cur_episode = 0, 1
        self._start_time = None
        self.recent_rewards, self._ep_reward = [], 0.0
        self.on_episode_end, self.on_step_end = [], []
        if print_interval is not None:
            self.add_callback(self.print, print_interval)
        if exploration is None or hasattr(exploration, "act"):
            self.exploration = exploration
        else:
            self.exploration = RandomExploration(solver, env.action_space, epsilon=exploration)

    @property
    def cur_time(self):
        return 0 if self._start_time is None else time.monotonic() - self._start_time

    def add_callback(self, cb, interval):
        if isinstance(interval, int):
            num, unit = interval, "ts"
        elif isinstance(interval, str) and interval.endswith("ts"):
            num, unit = int(interval[:-2]), "ts"
        elif isinstance(interval, str) and interval.endswith("e"):
            num, unit = int(interval[:-1]), "e"
        else:
            raise ValueError(f"Invalid interval input {interval}, valid units: ts (timestep), e (episode)")
        (self.on_step_end if unit == "ts" else self.on_episode_end).append(Interval(cb, num))

    def print(self):
        if self.logger and self.recent_rewards:
            self.logger.info(f"ts: {self.cur_step}, episode: {self.cur_episode}, "
                             f"mean_reward: {np.mean(self.recent_rewards):.3f}, time: {self.cur_time:.2f}")
        self.recent_rewards = []

    def load_weights(self, stream):
        self.solver.load_weights(stream)

    def save_weights(self, stream=None):
        return self.solver.save_weights(stream)

    def step(self, action=None):
        if self._start_time is None:
            self._start_time = time.monotonic()
        self.cur_step += 1
        if action is None:
            action = self.solver.act(self.s0) if self.exploration is None else self.exploration.act(self.s0)
        s1, r, done, info = self.env.step(action)
        result = (self.s0, action, r, s1, done)
        self.s0 = s1
        self._ep_reward += r
        if done:
            self.s0 = self.env.reset()
            self.recent_rewards.append(info.get("episode", {}).get("r", self._ep_reward))
            self._ep_reward = 0.0
            for cb in self.on_episode_end:
                cb()
            self.cur_episode += 1
        for cb in self.on_step_end:
            cb()
        return result

    def step_batch(self, batch_size):
        """worker.py:157-163: a non-circular staging buffer of batch_size transitions"""
        buf = NumpyBuffer(batch_size, circular=False, device=self.device)
        for _ in range(batch_size):
            buf.append(self.step())
        return buf.data

    def step_episode(self):
        buf = DynamicSizeBuffer(64, device=self.device)
        while True:
            res = self.step()
            buf.append(res)
            if res[-1]:
                return buf.data


def _parse_input(f):
    if isinstance(f, dict):
        return f
    if isinstance(f, str):
        if os.path.exists(f):
            with open(f) as fh:
                return yaml.safe_load(fh)
        return yaml.safe_load(f)
    if isinstance(f, io.IOBase):
        return yaml.safe_load(f)
    raise ValueError(f"Invalid config input {f!r}")


def get_env(f, **kwargs):
    return envs.make(**{**_parse_input(f)["env"], **kwargs})


def get_solver(f, env=None, **kwargs):
    config = _parse_input(f)
    env = env if env is not None else get_env(config)
    return _get_solver(observation_space=env.observation_space, action_space=env.action_space,
                       **{**config["solver"], **kwargs})


def get_worker(f, solver=None, env=None, **kwargs):
    config = _parse_input(f)
    env = env if env is not None else get_env(config)
    solver = solver if solver is not None else get_solver(config, env)
    return Worker(env, solver, **{**config.get("worker", {}), **kwargs})


def get_trainer(f, solver=None, env=None, **kwargs):
    config = _parse_input(f)
    if solver is None:
        solver = get_solver(config, env if env is not None else get_env(config))
    return Trainer(solver, **{**config.get("trainer", {}), **kwargs})


def get_replay_buffer(f, **kwargs):
    cfg = dict(_parse_input(f)["replay_buffer"])
    prioritized = cfg.pop("prioritized")
    return PrioritizedBuffer(**{**cfg, **kwargs}) if prioritized else NumpyBuffer(**{**cfg, **kwargs})
