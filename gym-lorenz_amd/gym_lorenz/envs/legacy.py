"""Drop-ins for the reference's unregistered env modules.  In the
reference all four classes are named `lorenzEnv_transient`; they are exported here
under distinct names.  Classic gym API (4-tuple step), float64 by default
(bit-identical to the reference); the host draws from the global np.random stream in
the reference's order and the kernel does every state / observation / reward update.

  LorenzTransient1Env     lorenz_env_transient1.py:18-104   (LZ_SYS_T1)
  LorenzTransient2Env     lorenz_env_transient2.py:115-240  (LZ_SYS_T2)
  LorenzTransientPmsmEnv  lorenz_env_transient_pmsm.py:17-133 (LZ_SYS_TP)
  LorenzSingleControlEnv  lorenz_singlecontrol.py:97-172     (LZ_SYS_SC)
"""
import numpy as np

from .. import _native as nat
from ..compat import Box, GymEnv
from ._single import SingleEnvCore


class _Legacy(GymEnv):
    metadata = {"render.modes": ["human", "rgb_array"]}
    SYSTEM = None
    M_FIRST, S_FIRST, NSTATE = 0, None, 3

    def _setup(self, input_min, input_max, state_dim, act_dim, dtype, device):
        self.input_min = input_min
        self.input_max = input_max
        self.state_dim = state_dim
        self.action_dim = self.input_max - self.input_min
        self.observation_space = Box(-np.inf, np.inf, shape=(state_dim,), dtype=np.float32)
        self.action_space = Box(self.input_min, self.input_max, shape=(act_dim,), dtype=np.float32)
        self.state = None
        self.u1 = self.u2 = self.u3 = 0
        self.t = 0
        self._core = SingleEnvCore(self.SYSTEM, dtype, device)

    @property
    def state1(self):
        return self._core.planes(self.M_FIRST, self.NSTATE)

    @state1.setter
    def state1(self, v):
        self._core.set_planes(self.M_FIRST, np.asarray(v)[: self.NSTATE])

    @property
    def state2(self):
        if self.S_FIRST is None:  # an all-zero 6-vector in the single-system variants
            return np.zeros(6, np.int64)
        return self._core.planes(self.S_FIRST, self.NSTATE)

    @state2.setter
    def state2(self, v):
        if self.S_FIRST is None:
            raise AttributeError("state2 is a constant zero vector in this variant")
        self._core.set_planes(self.S_FIRST, np.asarray(v)[: self.NSTATE])

    def _get_observation(self):
        return self.state

    def _current(self, j):
        return [self.state1[j], self.state2[j]]

    def _get_current(self):
        return self._current(0)

    def _get_current1(self):
        return self._current(1)

    def _get_current2(self):
        return self._current(2)

    def render(self, mode="human"):
        pass

    def close(self):
        self._core.close()


class LorenzTransient1Env(_Legacy):
    """lorenz_env_transient1.py: one PMSM-form system (a=5.46, b=20) with additive
    actions clip(a, -10, 10) on x and y, Euler dt=0.01, reward -sum|obs[0:3]|."""
    SYSTEM = nat.T1

    def __init__(self, dtype="float64", device=None):
        self._setup(-10.0, 10.0, 6, 2, dtype, device)
        self.a, self.b = 5.46, 20

    def reset(self):
        """:41-55 -- state1 ~ U(-30, 30)^3 from the global RNG."""
        state1 = np.random.uniform(low=-30, high=30, size=(3,))
        self.state = self._core.reset(state1)
        self.t = 0
        return self.state

    def step(self, action):
        """:69-104 (kernel: lz_step on LZ_SYS_T1)."""
        self.u1 = np.clip(action[0], self.input_min, self.input_max)
        self.u2 = np.clip(action[1], self.input_min, self.input_max)
        self.target_system_noise = np.random.normal(loc=0, scale=1, size=(3,))  # :77, unused
        obs, reward, done = self._core.step(action)
        self.state = obs
        self.t = self.t + 0.01
        return obs, reward, bool(done & nat.DONE_TERMINATED), {}


class LorenzTransient2Env(_Legacy):
    """lorenz_env_transient2.py: 4-state master/slave (a=30, b=1, c=36, d=0.5,
    h=0.003), actions clip(a, -2, 2) * 100 on slave x1, x2, x4, Euler dt=0.001,
    reward -S - S**(1/3), done on reward < -1e6."""
    SYSTEM = nat.T2
    M_FIRST, S_FIRST, NSTATE = nat.T2_M1, nat.T2_S1, 4

    def __init__(self, dtype="float64", device=None):
        self._setup(-2, 2, 8, 3, dtype, device)
        self.a, self.b, self.c, self.d, self.h = 30, 1, 36, 0.5, 0.003

    def reset(self):
        """:139-163 -- state1, state2 ~ U(0, 5)^4 from the global RNG."""
        state1 = np.random.uniform(low=0, high=5, size=(4,))
        state2 = np.random.uniform(low=0, high=5, size=(4,))
        self.state = self._core.reset(np.concatenate([state1, state2]))
        self.t = 0
        return self.state

    def get_current(self):
        return self._current(0)

    def get_current1(self):
        return self._current(1)

    def get_current2(self):
        return self._current(2)

    def get_current3(self):
        return self._current(3)

    def step(self, action):
        """:180-239 (kernel: lz_step on LZ_SYS_T2)."""
        self.u1 = np.clip(action[0], self.input_min, self.input_max)
        self.u2 = np.clip(action[1], self.input_min, self.input_max)
        self.u3 = np.clip(action[2], self.input_min, self.input_max)
        self.target_system_noise = np.random.normal(loc=0, scale=0.5, size=(4,))  # :209, unused
        obs, reward, done = self._core.step(action)
        self.state = obs
        self.t = self.t + 0.001
        return obs, reward, bool(done & nat.DONE_TERMINATED), {}


class LorenzTransientPmsmEnv(_Legacy):
    """lorenz_env_transient_pmsm.py: PMSM-form master/slave, actions clip(a, -2, 2)*20
    and process noise N(0, 3) on the slave, Euler dt=0.01, reward -S - S**(1/10)."""
    SYSTEM = nat.TP
    M_FIRST, S_FIRST, NSTATE = nat.TP_M, nat.TP_S, 3

    def __init__(self, dtype="float64", device=None):
        self._setup(-2, 2, 6, 2, dtype, device)
        self.a, self.b = 5.46, 20

    def reset(self):
        """:43-62 -- state1, state2 ~ U(-10, 10)^3 from the global RNG."""
        state1 = np.random.uniform(low=-10, high=10, size=(3,))
        state2 = np.random.uniform(low=-10, high=10, size=(3,))
        self.state = self._core.reset(np.concatenate([state1, state2]))
        self.t = 0
        return self.state

    def step(self, action):
        """:76-133; the N(0, 3) draw of :86 is injected into the kernel."""
        self.u1 = np.clip(action[0], self.input_min, self.input_max)
        self.u2 = np.clip(action[1], self.input_min, self.input_max)
        self.target_system_noise = np.random.normal(loc=0, scale=3, size=(3,))
        obs, reward, done = self._core.step(action, self.target_system_noise)
        self.state = obs
        self.t = self.t + 0.01
        return obs, reward, bool(done & nat.DONE_TERMINATED), {}


class LorenzSingleControlEnv(_Legacy):
    """lorenz_singlecontrol.py: the PMSM-form system from the fixed start [25, 1, -1]
    driven by process noise N(0, 3) only; step() takes no action."""
    SYSTEM = nat.SC

    def __init__(self, dtype="float64", device=None):
        self._setup(-100, 100, 6, 2, dtype, device)
        self.a, self.b = 5.46, 20

    def reset(self):
        """:120-132 -- fixed start (the reference prints the observation here)."""
        self.state = self._core.reset(np.array([25.0, 1.0, -1.0]))
        self.t = 0
        return self.state

    def step(self, action=None):
        """:145-172; the N(0, 3) draw of :147 is injected into the kernel."""
        self.target_system_noise = np.random.normal(loc=0, scale=3, size=(3,))
        obs, reward, done = self._core.step(np.zeros(2, np.float32), self.target_system_noise)
        self.state = obs
        self.t = self.t + 0.01
        return obs, reward, bool(done & nat.DONE_TERMINATED), {}
