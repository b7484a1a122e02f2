"""Drop-in for lorenz_env_try_pmsm.py:7-187 `PMSM_Sync_Env` (permanent-magnet
synchronous motor chaos sync, float32, Adam-driven dual variable lambda), the env
behind `lorenz_pmsm-v0`.

Host RNG use is the reference's: reset(seed) seeds self.np_random (PCG64) and
draws state1, state2 ~ U(-30, 30)^3 (:64-65); every step draws
self.np_random.normal(0, 3, 3) (:80), which the kernel adds to the slave
derivatives when add_noise=True.  Adam m/v/step and lambda persist across
resets, as in the reference.
"""
import numpy as np

from .. import _native as nat
from ..compat import Box, GymnasiumEnv
from ._single import SingleEnvCore


class PMSM_Sync_Env(GymnasiumEnv):  # noqa: N801 (reference name)
    """pmsm motor sync environment"""

    def __init__(self, alpha=0.5, add_noise=False, device=None):
        super().__init__()
        self.sigma = 5.46
        self.gamma = 20.0
        self.dt = 0.001
        self.lambda_lr = 0.001
        self.beta1 = 0.9
        self.beta2 = 0.999
        self.epsilon = 1e-8
        self.input_min = -1.0
        self.input_max = 1.0
        self.alpha = alpha
        self.add_noise = add_noise
        self.f_max = 50
        self.action_space = Box(low=-1, high=1, shape=(2,), dtype=np.float32)
        self.observation_space = Box(low=-np.inf, high=np.inf, shape=(6,), dtype=np.float32)
        self.global_step = 0
        self.total_training_steps = 1_000_000
        self.initial_lambda_lr = 0.0001
        self.current_step = 0
        self.max_steps = 2000
        self.target_system_noise = np.zeros(3)
        self._core = SingleEnvCore(nat.PMSM, "float32", device, alpha=float(alpha),
                                   add_noise=bool(add_noise))

    # ------------------------------------------------------------ reference helpers
    def _get_derivatives(self, state, action, noise=[0, 0, 0]):  # noqa: B006 (reference API)
        """:51-58 -- host helper used by callers to rebuild observations after a
        state injection (code/lorenz_pmsm/test_evaluate.py:104-111); not on the step
        path (the kernel has its own copy)."""
        x1, x2, x3 = state
        a1, a2 = action
        dx1 = -x1 + x2 * x3 + a1 + noise[0]
        dx2 = -x2 - x1 * x3 + self.gamma * x3 + a2 + noise[1]
        dx3 = self.sigma * (x2 - x3) + noise[2]
        return np.array([dx1, dx2, dx3], dtype=np.float32)

    # ------------------------------------------------------------ device-backed state
    @property
    def state1(self):
        return self._core.planes(nat.PMSM_S1, 3).astype(np.float32)

    @state1.setter
    def state1(self, v):
        self._core.set_planes(nat.PMSM_S1, np.asarray(v, dtype=np.float32))

    @property
    def state2(self):
        return self._core.planes(nat.PMSM_S2, 3).astype(np.float32)

    @state2.setter
    def state2(self, v):
        self._core.set_planes(nat.PMSM_S2, np.asarray(v, dtype=np.float32))

    @property
    def lambda_coef(self):
        return np.float32(self._core.plane(nat.PMSM_LAMBDA))

    @property
    def m_t(self):
        return np.float32(self._core.plane(nat.PMSM_M))

    @property
    def v_t(self):
        return np.float32(self._core.plane(nat.PMSM_V))

    @property
    def adam_step(self):
        return int(self._core.plane(nat.PMSM_ADAM_STEP))

    # ------------------------------------------------------------ API
    def reset(self, seed=None, options=None):
        """:59-75"""
        super().reset(seed=seed)
        self.current_step = 0
        s1 = self.np_random.uniform(low=-30, high=30, size=(3,)).astype(np.float32)
        s2 = self.np_random.uniform(low=-30, high=30, size=(3,)).astype(np.float32)
        obs = self._core.reset(np.concatenate([s1, s2]))
        return obs, {}

    def step(self, action):
        """:76-184 (kernel: lz_step on PMSM)."""
        self.current_step += 1
        self.target_system_noise = self.np_random.normal(loc=0, scale=3, size=(3,))  # :80
        obs, reward, done = self._core.step(
            action, self.target_system_noise if self.add_noise else None)
        terminated = bool(done & nat.DONE_TERMINATED)
        truncated = bool(done & nat.DONE_TRUNCATED)
        return obs, float(reward), terminated, truncated, {}

    def render(self):
        print(f"Step: {self.current_step}, State: {self.state1}, {self.state2}")

    def close(self):
        self._core.close()
