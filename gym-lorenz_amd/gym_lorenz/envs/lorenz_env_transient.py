"""Drop-in for lorenz_env_transient.py:247-376 `lorenzEnv_transient` (4-state
master/slave Lorenz-like system, Euler dt=0.001, 8-D observation, classic gym API)
-- the env behind the historical id `lorenz_transient-v0` used by code/gym_run.py.

Reference semantics kept: the action is clipped to [-2, 2] and stored but never
enters the dynamics (:316-318); every step draws np.random.normal(0, 0.5, 3) and
discards it (:343); done = (t == 5) on a float accumulator (never) or
reward < -1e6 (:364-372).  float64 by default: bit-identical to the reference.
"""
import numpy as np

from .. import _native as nat
from ..compat import Box, GymEnv
from ._single import SingleEnvCore


class lorenzEnv_transient(GymEnv):  # noqa: N801 (reference name)
    metadata = {"render.modes": ["human", "rgb_array"]}

    def __init__(self, dtype="float64", device=None):
        self.input_min = -2
        self.input_max = 2
        self.state_dim = 8
        self.action_dim = self.input_max - self.input_min
        self.observation_space = Box(-np.inf, np.inf, shape=(self.state_dim,), dtype=np.float32)
        self.action_space = Box(self.input_min, self.input_max, shape=(3,), dtype=np.float32)
        self.state = None
        self.state0 = None
        self.dis = 0
        self.u1 = self.u2 = self.u3 = 0
        self.t = 0
        self.a = 10
        self.b = 8 / 3
        self.c = 28
        self.r = -1
        self._core = SingleEnvCore(nat.LORENZ4, dtype, device)

    def reset(self):
        """:275-297 -- state1, state2 ~ U(0, 5)^4 from the global RNG."""
        state1 = np.random.uniform(low=0, high=5, size=(4,))
        state2 = np.random.uniform(low=0, high=5, size=(4,))
        obs = self._core.reset(np.concatenate([state1, state2]))
        self.state = obs
        self.t = 0
        return obs

    @property
    def state1(self):
        return self._core.planes(nat.L4_M1, 4)

    @state1.setter
    def state1(self, v):
        self._core.set_planes(nat.L4_M1, v)

    @property
    def state2(self):
        return self._core.planes(nat.L4_S1, 4)

    @state2.setter
    def state2(self, v):
        self._core.set_planes(nat.L4_S1, np.asarray(v)[:4])

    def _get_observation(self):
        return self.state

    def get_current(self):
        return [self.state1[0], self.state2[0]]

    def get_current1(self):
        return [self.state1[1], self.state2[1]]

    def get_current2(self):
        return [self.state1[2], self.state2[2]]

    def get_current3(self):
        return [self.state1[3], self.state2[3]]

    def step(self, action):
        """:314-373 (kernel: lz_step on LORENZ4)."""
        self.u1 = np.clip(action[0], self.input_min, self.input_max)
        self.u2 = np.clip(action[1], self.input_min, self.input_max)
        self.u3 = np.clip(action[2], self.input_min, self.input_max)
        self.target_system_noise = np.random.normal(loc=0, scale=0.5, size=(3,))  # :343
        obs, reward, done = self._core.step(action)
        self.state = obs
        self.t = self.t + 0.001
        return obs, reward, bool(done & nat.DONE_TERMINATED), {}

    def render(self, mode="human"):
        pass

    def close(self):
        self._core.close()
