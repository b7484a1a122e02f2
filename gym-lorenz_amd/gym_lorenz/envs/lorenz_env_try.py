"""Drop-in for lorenz_env_try.py:7-179 `HRSyncEnv` (Hindmarsh-Rose neuron
master/slave synchronisation, RK4 dt=0.001), the env behind `lorenz_try-v0`
(code/train.py).

Host RNG use is the reference's: reset() draws master, slave ~ U(-10, 20)^3 and,
with add_noise and not eval_mode, sigma ~ U(0, 2) from the GLOBAL np.random
(:55-67; the seed argument only seeds self.np_random, which HR never uses); each
step with add_noise draws np.random.normal(0, sigma, 3) (:136), which the kernel
adds to the master after the RK4 update.  float64 by default.
"""
import numpy as np

from .. import _native as nat
from ..compat import Box, GymnasiumEnv
from ._single import SingleEnvCore


def hr_derivatives(state, a1, a2, a, b, c, d, r, s, I_bias, x_rest):  # noqa: N803
    """:7-12 -- the reference's public helper (host NumPy; the kernel has its own)."""
    x1, x2, x3 = state
    dx1 = x2 - a * (x1 ** 3) + b * (x1 ** 2) - x3 + I_bias
    dx2 = c - d * (x1 ** 2) - x2 + a1
    dx3 = r * (s * (x1 - x_rest) - x3) + a2
    return np.array([dx1, dx2, dx3])


class HRSyncEnv(GymnasiumEnv):
    """Hindmarsh-Rose sync env: master runs free, the slave is driven by the agent."""

    def __init__(self, add_noise=False, eval_mode=False, add_filter=False, dtype="float64",
                 device=None):
        super().__init__()
        self.add_noise = add_noise
        self.eval_mode = eval_mode
        self.add_filter = add_filter
        self.action_space = Box(low=-1.0, high=1.0, shape=(2,), dtype=np.float32)
        self.observation_space = Box(low=-1.0, high=1.0, shape=(6,), dtype=np.float32)
        self.scale_factor = 50.0
        self.a, self.b, self.c, self.d = 1.0, 3.0, 1.0, 5.0
        self.r, self.s, self.I_bias, self.x_rest = 0.006, 4.0, 3.2, -1.6
        self.dt = 0.001
        self.sigma = 0.0
        self.action_alpha = 0.95
        self._core = SingleEnvCore(nat.HR, dtype, device, add_noise=bool(add_noise),
                                   eval_mode=bool(eval_mode), add_filter=bool(add_filter))

    @property
    def state_master(self):
        return self._core.planes(nat.HR_M, 3).astype(np.float64)

    @state_master.setter
    def state_master(self, v):
        self._core.set_planes(nat.HR_M, v)

    @property
    def state_slave(self):
        return self._core.planes(nat.HR_S, 3).astype(np.float64)

    @state_slave.setter
    def state_slave(self, v):
        self._core.set_planes(nat.HR_S, v)

    @property
    def filtered_action(self):
        return self._core.planes(nat.HR_FA, 2).astype(np.float32)

    def reset(self, seed=None, options=None):
        """:49-78"""
        super().reset(seed=seed)
        m = np.random.uniform(-10, 20, 3)
        s = np.random.uniform(-10, 20, 3)
        if self.add_noise:
            self.sigma = 2.0 if self.eval_mode else np.random.uniform(0, 2)
        else:
            self.sigma = 0.0
        obs = self._core.reset(np.concatenate([m, s, [self.sigma]]))
        return obs.astype(np.float32), {}

    def step(self, action):
        """:80-179 (kernel: lz_step on HR)."""
        noise = np.random.normal(0, self.sigma, 3) if self.add_noise else None  # :136
        obs, reward, done = self._core.step(action, noise)
        return obs.astype(np.float32), float(reward), bool(done & nat.DONE_TERMINATED), False, {}

    def close(self):
        self._core.close()
