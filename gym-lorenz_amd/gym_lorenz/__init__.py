"""gym_lorenz -- MI355X-native drop-in for erererq/gym-lorenz's `gym_lorenz` package.

Import it exactly like the reference (`import gym_lorenz`): the env ids are
registered with gymnasium (and classic gym) when those are installed, as the
reference's gym_lorenz/__init__.py:4-23 does.  Without them, `gym_lorenz.make(id)`
provides the same construction (env + TimeLimit) and `gym_lorenz.make_vec(id, N)`
the batched SB3 VecEnv.

Every reset()/step() runs in the HIP kernels of libgym_lorenz_amd.so (built by
`make -C gym-lorenz_amd`); there is no CPU fallback.
"""
from . import _native  # noqa: F401  (fails loudly if the native library is missing)
from .compat import HAVE_GYM, HAVE_GYMNASIUM, TimeLimit
from .core import BatchedEnv
from .envs import HRSyncEnv, LorenzDynamicEnv, PMSM_Sync_Env, lorenzEnv_transient
from .registry import SPECS, spec_for
from .vec_env import LorenzVecEnv

__version__ = "0.1.0"


def make(env_id, max_episode_steps=None, **kwargs):
    """gymnasium.make equivalent: the env class wrapped in TimeLimit when the id
    registers a max_episode_steps."""
    spec = spec_for(env_id)
    env = spec.entry_class()(**kwargs)
    steps = spec.max_episode_steps if max_episode_steps is None else max_episode_steps
    if steps:
        env = TimeLimit(env, steps)
    return env


def make_vec(env_id, num_envs, **kwargs):
    """N envs of `env_id` batched on one GPU (SB3 VecEnv)."""
    return LorenzVecEnv(env_id, num_envs, **kwargs)


def _register():  # pragma: no cover - gym / gymnasium are not installed in this image
    if HAVE_GYMNASIUM:
        import gymnasium

        for s in SPECS.values():
            if s.id not in gymnasium.registry:
                gymnasium.register(id=s.id, entry_point=s.entry_point,
                                   max_episode_steps=s.max_episode_steps,
                                   reward_threshold=s.reward_threshold)
    if HAVE_GYM:
        import gym

        for s in SPECS.values():
            try:
                gym.register(id=s.id, entry_point=s.entry_point,
                             max_episode_steps=s.max_episode_steps,
                             reward_threshold=s.reward_threshold)
            except Exception:  # noqa: BLE001 - already registered
                pass


_register()

__all__ = ["BatchedEnv", "LorenzVecEnv", "HRSyncEnv", "PMSM_Sync_Env", "lorenzEnv_transient",
           "LorenzDynamicEnv", "make", "make_vec", "SPECS", "spec_for"]
