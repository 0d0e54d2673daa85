"""Host environments -- gym and ALE are not part of this image.

CartPole restates gym's classic-control CartPole-v0/v1 dynamics (the reference's
examples/dqn/config.yaml names CartPole-v0; gym 0.17.3 is its pinned dependency): Euler
integration of the cart-pole ODE, terminal when |x| > 2.4 or |theta| > 12 degrees, reward
1 per step, TimeLimit 200 (v0) / 500 (v1).  Trajectories are not a parity claim (SURVEY
§8c: env dynamics are outside the path); the spaces and the step/reset contract are.

Atari names (`<Game>NoFrameskip-v4`, the apex configs) give `SyntheticAtari`: the spaces of
the reference's wrapped env (env/util.py:281-297, wrap_deepmind + 4-frame stack: uint8
observations [4, 84, 84], the game's minimal action set) over synthetic frames with the
bench's reward / episode-end rates -- a stand-in so the reference's scripts build their
solver, trainer and workers; ALE emulation itself is out of scope.
"""
import math

import numpy as np

from .solver import Box, Discrete


class CartPole:
    gravity, masscart, masspole, length, force_mag, tau = 9.8, 1.0, 0.1, 0.5, 10.0, 0.02
    theta_threshold = 12 * 2 * math.pi / 360
    x_threshold = 2.4

    def __init__(self, max_episode_steps=200, seed=None):
        high = np.array([self.x_threshold * 2, np.finfo(np.float32).max, self.theta_threshold * 2,
                         np.finfo(np.float32).max], dtype=np.float32)
        self.observation_space = Box(-high, high, (4,), np.float32)
        self.action_space = Discrete(2)
        self.max_episode_steps = max_episode_steps
        self.np_random = np.random.RandomState(seed)
        self.state = None
        self._t = 0

    def reset(self):
        self.state = self.np_random.uniform(low=-0.05, high=0.05, size=(4,))
        self._t = 0
        return np.array(self.state)

    def step(self, action):
        assert action in (0, 1), action
        x, x_dot, theta, theta_dot = self.state
        force = self.force_mag if action == 1 else -self.force_mag
        costheta, sintheta = math.cos(theta), math.sin(theta)
        total_mass = self.masspole + self.masscart
        polemass_length = self.masspole * self.length
        temp = (force + polemass_length * theta_dot ** 2 * sintheta) / total_mass
        thetaacc = (self.gravity * sintheta - costheta * temp) / (
            self.length * (4.0 / 3.0 - self.masspole * costheta ** 2 / total_mass))
        xacc = temp - polemass_length * thetaacc * costheta / total_mass
        x = x + self.tau * x_dot
        x_dot = x_dot + self.tau * xacc
        theta = theta + self.tau * theta_dot
        theta_dot = theta_dot + self.tau * thetaacc
        self.state = (x, x_dot, theta, theta_dot)
        self._t += 1
        done = bool(x < -self.x_threshold or x > self.x_threshold or theta < -self.theta_threshold
                    or theta > self.theta_threshold or self._t >= self.max_episode_steps)
        return np.array(self.state), 1.0, done, {}


# ALE minimal action-set sizes of the games the configs name (and a few common ones)
ATARI_ACTIONS = {"Pong": 6, "Breakout": 4, "BeamRider": 9, "Seaquest": 18, "SpaceInvaders": 6, "Qbert": 6,
                 "Enduro": 9, "MsPacman": 9, "Asterix": 9, "Boxing": 18, "Freeway": 3}


class SyntheticAtari:
    """the wrapped Atari env's interface (frame-stacked uint8 [4, 84, 84] observations, the
    minimal action set) over synthetic frames: each step shifts the stack and draws a new
    uniform frame; reward +-1 with probability p_reward, episode end with probability p_done"""

    def __init__(self, game, seed=None, p_reward=0.02, p_done=1.0 / 2000, frame_stack=4):
        self.game = game
        self.observation_space = Box(0, 255, (frame_stack, 84, 84), np.uint8)
        self.action_space = Discrete(ATARI_ACTIONS[game])
        self.p_reward, self.p_done = p_reward, p_done
        self.np_random = np.random.RandomState(seed)
        self._stack = None

    def _frame(self):
        return self.np_random.randint(0, 256, (84, 84), dtype=np.uint8)

    def reset(self):
        self._stack = np.stack([self._frame() for _ in range(self.observation_space.shape[0])])
        return self._stack.copy()

    def step(self, action):
        assert 0 <= int(action) < self.action_space.n, action
        self._stack = np.concatenate([self._stack[1:], self._frame()[None]])
        u = self.np_random.rand(2)
        r = float(np.sign(u[0] - 0.5)) if u[0] < self.p_reward or u[0] > 1 - self.p_reward else 0.0
        return self._stack.copy(), r, bool(u[1] < self.p_done), {}


def make(name, **kwargs):
    """reth.env.make (env/util.py:305-316) for the environments this build carries"""
    if name == "CartPole-v0":
        return CartPole(200, **kwargs)
    if name == "CartPole-v1":
        return CartPole(500, **kwargs)
    name = name.strip()
    if name.endswith("NoFrameskip-v4") and name[: -len("NoFrameskip-v4")] in ATARI_ACTIONS:
        return SyntheticAtari(name[: -len("NoFrameskip-v4")], **kwargs)
    raise NotImplementedError(f"environment {name!r}: gym/ALE are not part of this build (CartPole-v0/v1 are "
                              "restated, Atari names get SyntheticAtari; Atari observations: "
                              "reth_amd.atari.AtariPreprocessor)")
