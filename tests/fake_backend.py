"""Test double of gym_lorenz.core.BatchedEnv driven by the CPU oracle.

TEST INFRASTRUCTURE: lets the host-side logic above the kernel (SB3 VecEnv
adapter, infos, auto-reset bookkeeping, sharding and the gather collectives) be
tested on a machine without a GPU.  It reproduces the kernel's contract (SoA
planes, done bits, compact done list, Philox auto-reset keyed by (seed, global id,
tick)) for LORENZ3 fp32 and PMSM.  The product never uses it.
"""
import numpy as np
import torch

import oracle

DONE_TERMINATED, DONE_TRUNCATED = 1, 2


class FakeBackend:
    def __init__(self, system="lorenz3", num_envs=8, seed=0, global_env_offset=0,
                 max_episode_steps=0, alpha=0.5):
        assert system in ("lorenz3", "pmsm")
        self.system_name = system
        self.num_envs = n = num_envs
        self.seed = seed
        self.gid0 = global_env_offset
        self.max_steps = max_episode_steps
        if system == "pmsm":
            own = 2000
            self.max_steps = own if not max_episode_steps else min(own, max_episode_steps)
        self.alpha = alpha
        self.obs_dim = 6
        self.action_dim = 3 if system == "lorenz3" else 2
        self.tick = 0
        self.steps = np.zeros(n, np.int32)
        if system == "lorenz3":
            self.st = np.zeros((n, 3), np.float32)
        else:
            self.S = oracle.PmsmState(n)
        self.obs = torch.zeros((n, 6))
        self.rew = torch.zeros(n)
        self.done = torch.zeros(n, dtype=torch.uint8)
        self._done_idx = np.zeros(0, np.int64)
        self._term = np.zeros((0, 6), np.float32)

    def _draw(self, tick):
        key = "l3" if self.system_name == "lorenz3" else "pmsm"
        return oracle.reset_draw(key, np.float32, self.num_envs, self.gid0, self.seed, tick)

    def _reset_obs(self, init, rows):
        if self.system_name == "lorenz3":
            self.st[rows] = init[rows]
            return oracle.l3_reset_obs(self.st)[rows]
        self.S.st[rows] = init[rows]
        self.S.cur_step[rows] = 0
        return oracle.pmsm_reset_obs(self.S.st)[rows]

    def reset(self, mask=None, init=None):
        rows = np.ones(self.num_envs, bool) if mask is None else np.asarray(mask, bool)
        init = self._draw(self.tick) if init is None else np.asarray(init, np.float32)
        o = self.obs.numpy()
        o[rows] = self._reset_obs(init, rows)
        self.steps[rows] = 0
        self.tick += 1
        return self.obs

    def step(self, actions, noise=None):
        a = np.asarray(actions.cpu() if isinstance(actions, torch.Tensor) else actions, np.float32)
        if self.system_name == "lorenz3":
            o, r = oracle.l3_step(self.st, a)
            term = np.zeros(self.num_envs, bool)
        else:
            o, r, term, _ = oracle.pmsm_step(self.S, a, None, False, self.alpha, oracle.DEV)
        self.steps += 1
        trunc = (self.steps >= self.max_steps) if self.max_steps > 0 else np.zeros_like(term)
        flags = (term * DONE_TERMINATED | trunc * DONE_TRUNCATED).astype(np.uint8)
        done = flags != 0
        self._done_idx = np.nonzero(done)[0]
        self._term = o[done].copy()
        if done.any():
            fresh = self._draw(self.tick)
            o[done] = self._reset_obs(fresh, done)
            self.steps[done] = 0
        self.tick += 1
        self.obs.copy_(torch.from_numpy(o))
        self.rew.copy_(torch.from_numpy(r.astype(np.float32)))
        self.done.copy_(torch.from_numpy(flags))
        return self.obs, self.rew, self.done

    def done_list(self):
        return torch.from_numpy(self._done_idx), torch.from_numpy(self._term)

    def get_state(self, plane):
        if self.system_name == "lorenz3":
            return torch.from_numpy(self.st[:, plane].copy())
        cols = {**{j: self.S.st[:, j] for j in range(6)}, 6: self.S.lam, 7: self.S.m, 8: self.S.v,
                9: self.S.adam_step, 10: self.S.cur_step}
        return torch.from_numpy(np.array(cols[plane]))

    def set_state(self, plane, values):
        v = np.asarray(values.cpu() if isinstance(values, torch.Tensor) else values)
        if self.system_name == "lorenz3":
            self.st[:, plane] = v
        else:
            self.S.st[:, plane] = v

    def set_seed(self, seed):
        self.seed = seed

    def close(self):
        pass
