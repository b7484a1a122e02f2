"""Env ids (reference: gym_lorenz/__init__.py:4-23).

  lorenz_try-v0        HRSyncEnv        TimeLimit 5000   (registered by the reference)
  lorenz_pmsm-v0       PMSM_Sync_Env    TimeLimit 2000   (registered by the reference)
  lorenz_transient-v0  4-state lorenzEnv_transient, TimeLimit 4000 -- commented out in
                       the reference's __init__.py:11 but still called by
                       code/gym_run.py:68; restored with its historical settings
                       (stale bytecode shows max_episode_steps=4000)
  lorenz_dynamic-v0    dynamic.py's 3-state lorenzEnv_transient (new id; no TimeLimit)
"""
import numpy as np

from . import _native as nat
from .compat import Box


class EnvSpec:
    def __init__(self, env_id, entry, system, system_name, max_episode_steps, obs_dim, act,
                 obs_bounds=(-np.inf, np.inf), reward_threshold=1e50):
        self.id = env_id
        self.entry_point = entry
        self.system = system
        self.system_name = system_name
        self.max_episode_steps = max_episode_steps
        self.obs_dim = obs_dim
        self.act = act  # (low, high, dim)
        self.obs_bounds = obs_bounds
        self.reward_threshold = reward_threshold

    def spaces(self):
        lo, hi = self.obs_bounds
        obs = Box(lo, hi, shape=(self.obs_dim,), dtype=np.float32)
        alo, ahi, adim = self.act
        act = Box(alo, ahi, shape=(adim,), dtype=np.float32)
        return obs, act

    def entry_class(self):
        mod, cls = self.entry_point.split(":")
        import importlib

        return getattr(importlib.import_module(mod), cls)


SPECS = {
    "lorenz_try-v0": EnvSpec("lorenz_try-v0", "gym_lorenz.envs:HRSyncEnv", nat.HR, "hr", 5000,
                             6, (-1.0, 1.0, 2), obs_bounds=(-1.0, 1.0)),
    "lorenz_pmsm-v0": EnvSpec("lorenz_pmsm-v0", "gym_lorenz.envs:PMSM_Sync_Env", nat.PMSM, "pmsm",
                              2000, 6, (-1.0, 1.0, 2)),
    "lorenz_transient-v0": EnvSpec("lorenz_transient-v0", "gym_lorenz.envs:lorenzEnv_transient",
                                   nat.LORENZ4, "lorenz4", 4000, 8, (-2.0, 2.0, 3)),
    "lorenz_dynamic-v0": EnvSpec("lorenz_dynamic-v0", "gym_lorenz.envs:LorenzDynamicEnv",
                                 nat.LORENZ3, "lorenz3", None, 6, (-500.0, 500.0, 3)),
}


# The reference's unregistered env modules (no gym id there; addressed here by system
# name, e.g. make_vec("transient_pmsm", N)): lorenz_env_transient1.py,
# lorenz_env_transient2.py, lorenz_env_transient_pmsm.py, lorenz_singlecontrol.py
LEGACY_SPECS = {
    "transient1": EnvSpec("transient1", "gym_lorenz.envs.legacy:LorenzTransient1Env", nat.T1,
                          "transient1", None, 6, (-10.0, 10.0, 2)),
    "transient2": EnvSpec("transient2", "gym_lorenz.envs.legacy:LorenzTransient2Env", nat.T2,
                          "transient2", None, 8, (-2.0, 2.0, 3)),
    "transient_pmsm": EnvSpec("transient_pmsm", "gym_lorenz.envs.legacy:LorenzTransientPmsmEnv",
                              nat.TP, "transient_pmsm", None, 6, (-2.0, 2.0, 2)),
    "singlecontrol": EnvSpec("singlecontrol", "gym_lorenz.envs.legacy:LorenzSingleControlEnv",
                             nat.SC, "singlecontrol", None, 6, (-100.0, 100.0, 2)),
}


def spec_for(env_id):
    if env_id in SPECS:
        return SPECS[env_id]
    if env_id in LEGACY_SPECS:
        return LEGACY_SPECS[env_id]
    for s in SPECS.values():  # also accept a system name
        if s.system_name == env_id:
            return s
    raise KeyError("unknown env id %r (known: %s)" % (env_id, ", ".join(SPECS)))
