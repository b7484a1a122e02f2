"""Per-env drop-in classes (reference: gym_lorenz/envs/__init__.py:1-3).

The reference exports HRSyncEnv and PMSM_Sync_Env here (the 4-state
lorenzEnv_transient import is commented out there); this package also exports the
two `lorenzEnv_transient` classes under distinct names because the reference has
two different classes with that name.
"""
from .dynamic import lorenzEnv_transient as LorenzDynamicEnv
from .lorenz_env_transient import lorenzEnv_transient
from .lorenz_env_try import HRSyncEnv, hr_derivatives
from .legacy import (LorenzSingleControlEnv, LorenzTransient1Env, LorenzTransient2Env,
                     LorenzTransientPmsmEnv)
from .lorenz_env_try_pmsm import PMSM_Sync_Env

__all__ = ["HRSyncEnv", "PMSM_Sync_Env", "lorenzEnv_transient", "LorenzDynamicEnv",
           "hr_derivatives", "LorenzTransient1Env", "LorenzTransient2Env",
           "LorenzTransientPmsmEnv", "LorenzSingleControlEnv"]
