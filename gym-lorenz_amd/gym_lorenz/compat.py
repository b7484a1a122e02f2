"""gym / gymnasium / stable-baselines3 interop.

The reference's env classes subclass `gym.Env` (classic, 4-tuple step API) or
`gymnasium.Env` (5-tuple API) and are registered with gymnasium.  When those
packages are importable the drop-in classes subclass them and the ids are
registered with them; when they are absent (as in this image) minimal stand-ins
with the same surface are used: `Box`, an `Env` base with gymnasium's
`reset(seed)` -> `self.np_random` seeding, and a `TimeLimit` wrapper.
"""
import numpy as np

try:  # pragma: no cover - depends on the environment
    import gymnasium as _gymnasium
except Exception:  # noqa: BLE001
    _gymnasium = None
try:  # pragma: no cover
    import gym as _gym
except Exception:  # noqa: BLE001
    _gym = None
try:  # pragma: no cover
    from stable_baselines3.common.vec_env.base_vec_env import VecEnv as _SB3VecEnv
except Exception:  # noqa: BLE001
    _SB3VecEnv = None

HAVE_GYMNASIUM = _gymnasium is not None
HAVE_GYM = _gym is not None
HAVE_SB3 = _SB3VecEnv is not None


class _Box:
    """Subset of gymnasium.spaces.Box: low/high/shape/dtype, sample(), contains()."""

    def __init__(self, low, high, shape=None, dtype=np.float32, seed=None):
        self.dtype = np.dtype(dtype)
        if shape is None:
            shape = np.shape(low)
        self.shape = tuple(shape)
        self.low = np.full(self.shape, low, dtype=self.dtype) if np.isscalar(low) else \
            np.asarray(low, dtype=self.dtype)
        self.high = np.full(self.shape, high, dtype=self.dtype) if np.isscalar(high) else \
            np.asarray(high, dtype=self.dtype)
        self._rng = np.random.default_rng(seed)

    def seed(self, seed=None):
        self._rng = np.random.default_rng(seed)
        return [seed]

    def sample(self):
        lo = np.where(np.isfinite(self.low), self.low, -1.0)
        hi = np.where(np.isfinite(self.high), self.high, 1.0)
        return self._rng.uniform(lo, hi).astype(self.dtype)

    def contains(self, x):
        x = np.asarray(x)
        return x.shape == self.shape and bool(np.all(x >= self.low) and np.all(x <= self.high))

    def __repr__(self):
        return "Box(%s, %s, %s, %s)" % (self.low.min(), self.high.max(), self.shape, self.dtype)


if HAVE_GYMNASIUM:  # pragma: no cover
    Box = _gymnasium.spaces.Box
else:
    Box = _Box


class _GymnasiumEnvBase:
    """gymnasium.Env surface used by the reference envs and their callers."""

    metadata = {"render_modes": []}
    render_mode = None
    spec = None
    _np_random = None

    @property
    def np_random(self):
        if self._np_random is None:
            self._np_random = np.random.default_rng()
        return self._np_random

    @np_random.setter
    def np_random(self, value):
        self._np_random = value

    def reset(self, *, seed=None, options=None):
        # gymnasium.utils.seeding.np_random(seed) == Generator(PCG64(SeedSequence(seed)))
        if seed is not None:
            self._np_random = np.random.default_rng(seed)

    @property
    def unwrapped(self):
        return self

    def close(self):
        pass

    def render(self):
        return None


class _GymEnvBase:
    """classic gym.Env surface (4-tuple step, reset() -> obs)."""

    metadata = {"render.modes": []}
    spec = None

    @property
    def unwrapped(self):
        return self

    def close(self):
        pass

    def seed(self, seed=None):
        return [seed]


GymnasiumEnv = _gymnasium.Env if HAVE_GYMNASIUM else _GymnasiumEnvBase
GymEnv = _gym.Env if HAVE_GYM else _GymEnvBase
VecEnvBase = _SB3VecEnv if HAVE_SB3 else object


class TimeLimit:
    """gymnasium.wrappers.TimeLimit equivalent (what gymnasium.make adds for a
    registered max_episode_steps): truncated=True once max_episode_steps steps
    have elapsed.  Works for both step APIs (4-tuple: done |= truncated,
    info['TimeLimit.truncated'] as classic gym did)."""

    def __init__(self, env, max_episode_steps):
        self.env = env
        self._max = int(max_episode_steps)
        self._elapsed = None
        self.observation_space = env.observation_space
        self.action_space = env.action_space

    @property
    def unwrapped(self):
        return self.env.unwrapped

    def __getattr__(self, name):
        if name.startswith("_"):
            raise AttributeError(name)
        return getattr(self.env, name)

    def reset(self, **kwargs):
        self._elapsed = 0
        return self.env.reset(**kwargs)

    def step(self, action):
        out = self.env.step(action)
        self._elapsed += 1
        hit = self._elapsed >= self._max
        if len(out) == 5:
            obs, rew, term, trunc, info = out
            return obs, rew, term, bool(trunc or hit), info
        obs, rew, done, info = out
        if hit and not done:
            info = dict(info)
            info["TimeLimit.truncated"] = True
            done = True
        return obs, rew, done, info

    def close(self):
        self.env.close()
