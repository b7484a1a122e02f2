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
from gym_lorenz.core import rollout_io_args, step_io_args

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
        # the checked caller-buffer entry's view of the handle (BatchedEnv's lz_info fields)
        self.tdtype, self.device, self.reads_actions = torch.float32, torch.device("cpu"), True
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

    def step_into(self, actions, obs, rew, done, done_idx=None, term_obs=None, n_done=None,
                  noise=None):
        """BatchedEnv.step_into's contract: the same buffer checks (core.step_io_args),
        refused before any state changes; then the step's outputs land in the buffers."""
        step_io_args(self, actions, obs, rew, done, done_idx, term_obs, n_done, noise)
        o, r, d = self.step(actions)
        obs.view(-1).copy_(o.reshape(-1))
        rew.copy_(r)
        done.copy_(d)
        if done_idx is not None:
            k = len(self._done_idx)
            done_idx.view(-1)[:k] = torch.from_numpy(self._done_idx.astype(np.int32))
            term_obs.view(-1)[: k * 6] = torch.from_numpy(self._term.reshape(-1))
            if n_done is not None:
                n_done.fill_(k)
        return obs, rew, done

    def rollout_into(self, K, actions, obs, rew, done, done_idx=None, term_obs=None, cap=0,
                     n_done=None):
        """BatchedEnv.rollout_into's contract (checks only the buffers here, then K steps)."""
        rollout_io_args(self, K, actions, obs, rew, done, done_idx, term_obs, cap, n_done)
        for k in range(int(K)):
            o, r, d = self.step(actions[k])
            obs[k].view(-1).copy_(o.reshape(-1))
            rew[k].copy_(r)
            done[k].copy_(d)
        return obs, rew, done

    def done_list(self):
        return torch.from_numpy(self._done_idx), torch.from_numpy(self._term)

    def _col(self, plane):
        if self.system_name == "lorenz3":
            return self.st[:, plane]
        cols = {**{j: self.S.st[:, j] for j in range(6)}, 6: self.S.lam, 7: self.S.m, 8: self.S.v,
                9: self.S.adam_step, 10: self.S.cur_step}
        return cols[plane]

    def get_state(self, plane, indices=None):
        col = self._col(plane)
        return torch.from_numpy(np.array(col if indices is None else col[np.asarray(indices)]))

    def set_state(self, plane, values, indices=None):
        v = np.asarray(values.cpu() if isinstance(values, torch.Tensor) else values)
        col = self._col(plane)  # a view: writes land in the state
        if indices is None:
            col[:] = v
        else:
            col[np.asarray(indices)] = v

    def set_seed(self, seed):
        self.seed = seed

    def close(self):
        pass


class FakeSingleCore:
    """Test double of gym_lorenz.envs._single.SingleEnvCore (one env) driven by the
    oracle in mode REF (glibc pow: the reference's own arithmetic), so the drop-in
    classes' host logic -- RNG draw order, attribute bookkeeping, API shapes -- can be
    checked against the golden fixtures without a GPU."""

    PLANES = {0: 3, 1: 8, 2: 6, 3: 6, 4: 3, 5: 8, 6: 6, 7: 3}
    LEGACY = {4: "t1", 5: "t2", 6: "tp", 7: "sc"}

    def __init__(self, system, dtype, device=None, alpha=0.5, add_noise=False, eval_mode=False,
                 add_filter=False):
        self.system = system
        self.dt = np.float32 if (system == 2 or np.dtype(dtype) == np.float32) else np.float64
        self.alpha, self.add_noise, self.add_filter = alpha, add_noise, add_filter
        self.S = oracle.PmsmState(1) if system == 2 else None
        self.st = np.zeros((1, self.PLANES[system]), self.dt)
        self.fa = np.zeros((1, 2), np.float32)

    def reset(self, init):
        init = np.asarray(init, self.dt).reshape(1, -1)
        if self.system in self.LEGACY:
            self.st[:] = init
            return oracle.legacy_reset_obs(self.LEGACY[self.system], self.st)[0]
        if self.system == 0:
            self.st[:] = init
            return oracle.l3_reset_obs(self.st)[0]
        if self.system == 1:
            self.st[:] = init
            return oracle.l4_reset_obs(self.st)[0]
        if self.system == 2:
            self.S.st[:] = init
            self.S.cur_step[:] = 0
            return oracle.pmsm_reset_obs(self.S.st)[0]
        self.st[:] = init[:, :6]
        self.fa[:] = 0
        return oracle.hr_reset_obs(self.st)[0]

    def step(self, action, noise=None):
        a = np.asarray(action, np.float32).reshape(1, -1)
        with np.errstate(all="ignore"):
            if self.system in self.LEGACY:
                key = self.LEGACY[self.system]
                nz = None if noise is None else np.asarray(noise, np.float64).reshape(1, 3)
                o, r, d = oracle.legacy_step(key, self.st, None if key == "sc" else a, nz)
                return o[0], r[0], int(d[0])
            if self.system == 0:
                o, r = oracle.l3_step(self.st, a.astype(self.dt))
                return o[0], r[0], 0
            if self.system == 1:
                o, r, d = oracle.l4_step(self.st)
                return o[0], r[0], int(d[0])
            if self.system == 2:
                nz = None if noise is None else np.asarray(noise, np.float64).reshape(1, 3)
                o, r, te, tr = oracle.pmsm_step(self.S, a, nz, noise is not None, self.alpha,
                                                oracle.REF)
                return o[0], r[0], int(te[0]) | (2 * int(tr[0]))
            nz = None if noise is None else np.asarray(noise, self.dt).reshape(1, 3)
            o, r, te = oracle.hr_step(self.st, self.fa, a, nz, noise is not None, self.add_filter,
                                      oracle.REF)
            return o[0], r[0], int(te[0])

    def plane(self, p):
        if self.system == 2:
            cols = {6: self.S.lam, 7: self.S.m, 8: self.S.v, 9: self.S.adam_step}
            return cols[p][0] if p in cols else self.S.st[0, p]
        return self.st[0, p]

    def planes(self, first, count):
        return np.array([self.plane(first + j) for j in range(count)])

    def set_planes(self, first, values, dtype=None):
        v = np.asarray(values).reshape(-1)
        tgt = self.S.st if self.system == 2 else self.st
        tgt[0, first:first + len(v)] = v

    def close(self):
        pass
