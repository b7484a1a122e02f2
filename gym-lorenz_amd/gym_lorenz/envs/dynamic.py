"""Drop-in for dynamic.py:5-93 `lorenzEnv_transient` (3-state Lorenz, Euler dt=0.01,
additive action, 6-D observation, classic gym 4-tuple API).

Same constructor signature, spaces, attributes and RNG consumption as the reference
(reset() draws np.random.uniform(-30, 30, 3) then np.random.normal(0.22, 3) from
the global MT19937, :62 and :70).  The step runs in the HIP kernel in float64 by
default -- bit-identical to the reference (tests/test_gpu_parity.py) -- or float32
with dtype="float32".
"""
import numpy as np

from .. import _native as nat
from ..compat import Box, GymEnv
from ._single import SingleEnvCore


class lorenzEnv_transient(GymEnv):  # noqa: N801 (reference name)
    metadata = {"render.modes": ["human", "rgb_array"]}

    def __init__(self, a=1.0, b=3.0, c=1.0, d=5.0, r=0.006, s=4, xs=-1.6, input_range=None,
                 id_range=None, noise_std=0.22, gamma=0.9, dtype="float64", device=None):
        # dynamic.py:8-33 -- unused constants kept for attribute compatibility
        self.a, self.b, self.c, self.d, self.r, self.s, self.xs = a, b, c, d, r, s, xs
        self.input_min = -500.0
        self.input_max = 500.0
        self.id_range = id_range if id_range is not None else [0, 5]
        self.noise_std = noise_std
        self.gamma = gamma
        self.state_dim = 6
        self.action_dim = self.input_max - self.input_min
        self.observation_space = Box(-np.inf, np.inf, shape=(self.state_dim,), dtype=np.float32)
        self.action_space = Box(self.input_min, self.input_max, shape=(3,), dtype=np.float32)
        self.state = None
        self.state0 = None
        self.state1 = None
        self.state2 = None
        self.input_signal = 3.2
        self.input_control = 0
        self.u1 = self.u2 = self.u3 = 0
        self.t = 0
        self.u = 10
        self.i = 28
        self.o = 8 / 3
        self._core = SingleEnvCore(nat.LORENZ3, dtype, device)

    def reset(self):
        """dynamic.py:35-47"""
        state1 = np.random.uniform(low=-30, high=30, size=(3,))
        obs = self._core.reset(state1)
        self.state1 = obs[:3].copy()
        self.state0 = list(obs)
        self.state2 = np.array([0, 0, 0, 0, 0, 0])
        self.target_system_noise = np.random.normal(scale=self.noise_std, size=(3,))
        self.t = 0
        return obs

    def _get_observation(self):
        return np.asarray(self.state0) - self.state2

    def _get_current(self):
        return [self.state1[0], self.state2[0]]

    def _get_current1(self):
        return [self.state1[1], self.state2[1]]

    def _get_current2(self):
        return [self.state1[2], self.state2[2]]

    def step(self, action):
        """dynamic.py:61-90 (kernel: lz_step on LORENZ3).  The reference's per-step
        attribute bookkeeping -- u1..u3 = np.clip(action[j]) (:63-65), state1 / state0 /
        state (:80-82) -- is kept with the same values and types, but materialised on
        first access (_lazy): three np.clip calls and the list conversion were ~40% of a
        resident-kernel step."""
        self._act = np.array(action, copy=True)
        obs, reward, done = self._core.step(action)
        self._obs = obs
        self._lz = {}
        self.t = self.t + 0.01
        return obs, reward, bool(done & nat.DONE_TERMINATED), {}

    # ---- lazily materialised step attributes (see step)
    def _lazy(self, name):
        lz = self.__dict__.get("_lz")
        if lz is None or self.__dict__.get("_obs") is None:
            return self.__dict__.get("_" + name + "_v")
        if name not in lz:
            a, o = self._act, self._obs
            if name in ("u1", "u2", "u3"):
                lz[name] = np.clip(a[int(name[1]) - 1], self.input_min, self.input_max)
            elif name == "state1":
                lz[name] = o[:3].copy()
            elif name == "state0":
                lz[name] = list(o)
            else:  # state
                lz[name] = o
        return lz[name]

    def _set_lazy(self, name, v):
        lz = self.__dict__.get("_lz")
        if lz is not None and self.__dict__.get("_obs") is not None:
            for k in ("u1", "u2", "u3", "state1", "state0", "state"):  # freeze the others
                self.__dict__["_" + k + "_v"] = self._lazy(k)
            self.__dict__["_lz"] = None
        self.__dict__["_" + name + "_v"] = v

    u1 = property(lambda s: s._lazy("u1"), lambda s, v: s._set_lazy("u1", v))
    u2 = property(lambda s: s._lazy("u2"), lambda s, v: s._set_lazy("u2", v))
    u3 = property(lambda s: s._lazy("u3"), lambda s, v: s._set_lazy("u3", v))
    state1 = property(lambda s: s._lazy("state1"), lambda s, v: s._set_lazy("state1", v))
    state0 = property(lambda s: s._lazy("state0"), lambda s, v: s._set_lazy("state0", v))
    state = property(lambda s: s._lazy("state"), lambda s, v: s._set_lazy("state", v))

    def set_state(self, state1):
        """Inject a 3-state (the reference's `env.state1 = ...`)."""
        obs = self._core.reset(np.asarray(state1, dtype=np.float64))
        self.state1 = obs[:3].copy()
        self.state0 = list(obs)
        return obs

    def render(self, mode="human"):
        pass

    def close(self):
        self._core.close()
