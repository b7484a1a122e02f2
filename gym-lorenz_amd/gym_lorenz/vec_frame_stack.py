"""LorenzVecFrameStack: stable-baselines3 `VecFrameStack` with the stack on the GPU.

The reference stacks 4 observations of the HR env for its attention policy
(code/lorenz_filter/train.py:113-115: ``VecFrameStack(DummyVecEnv([...]), n_stack=4)``).
This wrapper keeps SB3 2.7.1's semantics (common/vec_env/vec_frame_stack.py and
stacked_observations.py, 1-D Box, channels-last):

  reset:      stacked = 0; stacked[:, -O:] = obs
  step_wait:  stacked = roll(stacked, -O); for done envs the info's
              "terminal_observation" becomes concat(stacked[i, :-O], terminal_obs)
              and the row is zeroed; stacked[:, -O:] = obs

with the stacked buffer resident on the device and updated by one kernel per step
(``lz_frame_stack``).  It wraps a LorenzVecEnv or LorenzVecNormalize; outputs follow the
wrapped env's format (torch tensors with ``return_tensors=True``, NumPy otherwise).
"""
import ctypes

import numpy as np
import torch

from . import _native as nat
from .compat import Box


def _stream(device):
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)


class LorenzVecFrameStack:
    def __init__(self, venv, n_stack=4):
        self.venv = venv
        self.n_stack = int(n_stack)
        if self.n_stack < 1:
            raise ValueError("n_stack must be >= 1")
        self.num_envs = venv.num_envs
        be = venv.backend if hasattr(venv, "backend") else venv.venv.backend
        self.device = be.device
        self.obs_dim = be.obs_dim
        space = venv.observation_space
        low = np.repeat(np.asarray(space.low, np.float32), self.n_stack, axis=-1)
        high = np.repeat(np.asarray(space.high, np.float32), self.n_stack, axis=-1)
        self.observation_space = Box(low=low, high=high, dtype=np.float32)
        self.action_space = venv.action_space
        self.stacked = torch.zeros((self.num_envs, self.n_stack * self.obs_dim), dtype=torch.float32,
                                   device=self.device)

    def _dev(self, obs):
        if isinstance(obs, torch.Tensor):
            return obs.to(self.device, torch.float32).contiguous(), True
        return torch.from_numpy(np.ascontiguousarray(obs, np.float32)).to(self.device), False

    def _update(self, obs, done, reset):
        nat.check(nat.lib.lz_frame_stack(
            ctypes.c_void_p(self.stacked.data_ptr()), ctypes.c_void_p(obs.data_ptr()),
            None if done is None else ctypes.c_void_p(done.data_ptr()), self.num_envs,
            self.n_stack, self.obs_dim, int(reset), self.device.index, _stream(self.device)))

    def reset(self):
        obs, is_t = self._dev(self.venv.reset())
        self._update(obs, None, True)
        out = self.stacked.clone()
        return out if is_t else out.cpu().numpy()

    def step_async(self, actions):
        self.venv.step_async(actions)

    def step_wait(self):
        obs, rew, dones, infos = self.venv.step_wait()
        obs_d, is_t = self._dev(obs)
        done_d = (dones.to(self.device) if isinstance(dones, torch.Tensor)
                  else torch.from_numpy(np.asarray(dones, bool))).to(self.device, torch.uint8)
        done_h = done_d.cpu().numpy()
        idx = np.nonzero(done_h)[0]
        if len(idx):
            # SB3: previous_stack = rolled[i, :-O] = the stack's newest n_stack - 1 frames
            prev = self.stacked[torch.as_tensor(idx, device=self.device), self.obs_dim:]
            for j, i in enumerate(idx):
                info = infos[int(i)]
                if "terminal_observation" in info:
                    t = info["terminal_observation"]
                    if isinstance(t, torch.Tensor):
                        info["terminal_observation"] = torch.cat([prev[j], t.to(self.device).float()])
                    else:
                        info["terminal_observation"] = np.concatenate(
                            [prev[j].cpu().numpy(), np.asarray(t, np.float32)])
        self._update(obs_d, done_d, False)
        out = self.stacked.clone()
        return (out if is_t else out.cpu().numpy()), rew, dones, infos

    def step(self, actions):
        self.step_async(actions)
        return self.step_wait()

    def close(self):
        self.venv.close()

    def __getattr__(self, name):  # env_method / get_attr / seed ... pass through
        return getattr(self.venv, name)
