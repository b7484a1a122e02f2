"""NumPy restatement of stable-baselines3's VecFrameStack / StackedObservations for a
1-D Box observation space -- TEST INFRASTRUCTURE ONLY.

Third-party dependency absent from /root/reference and from this image:
stable-baselines3 2.7.1 (pinned by the reference's saved models' system_info.txt:3),
used by the reference as VecFrameStack(env, n_stack=4) around the HR env
(code/lorenz_filter/train.py:113-115).  Restates common/vec_env/stacked_observations.py
(StackedObservations.reset / update, channels-last path: stack_dimension -1) in the
same NumPy operations, to check lz_frame_stack / LorenzVecFrameStack.  Parity
unpinned beyond this restatement (the reference's files hold no stacked observations).
"""
import numpy as np


class StackedObservations:
    def __init__(self, num_envs, n_stack, obs_dim, dtype=np.float32):
        self.n_stack = n_stack
        self.stacked_obs = np.zeros((num_envs, n_stack * obs_dim), dtype=dtype)

    def reset(self, observation):
        self.stacked_obs[...] = 0
        self.stacked_obs[..., -observation.shape[-1]:] = observation
        return self.stacked_obs

    def update(self, observations, dones, infos):
        shift = -observations.shape[-1]
        self.stacked_obs = np.roll(self.stacked_obs, shift, axis=-1)
        for env_idx, done in enumerate(dones):
            if done:
                if "terminal_observation" in infos[env_idx]:
                    old_terminal = infos[env_idx]["terminal_observation"]
                    previous_stack = self.stacked_obs[env_idx, ..., :shift]
                    new_terminal = np.concatenate((previous_stack, old_terminal), axis=-1)
                    infos[env_idx]["terminal_observation"] = new_terminal
                self.stacked_obs[env_idx] = 0
        self.stacked_obs[..., shift:] = observations
        return self.stacked_obs, infos
