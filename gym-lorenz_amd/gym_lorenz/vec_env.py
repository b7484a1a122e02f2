"""LorenzVecEnv: a stable-baselines3 `VecEnv` whose N envs step in one HIP kernel.

Replaces `DummyVecEnv([lambda: gymnasium.make(id, ...)] * N)` (the reference's
callers, e.g. code/train.py:98-100, code/lorenz_pmsm/train.py:166) with the same
step_wait contract (SB3 2.7.1 DummyVecEnv.step_wait):
  obs float32 [N, obs_dim], rewards float32 [N], dones bool [N], infos list of N
  dicts; a done env's info carries "terminal_observation" (its pre-reset obs) and
  "TimeLimit.truncated" (= truncated and not terminated), and its returned obs row
  is already the post-reset observation.
VecNormalize / VecFrameStack / VecMonitor wrap it unchanged.  With
return_tensors=True obs/rewards/dones stay on the GPU as torch tensors (no D2H).
"""
from collections.abc import Sequence

import numpy as np
import torch

from . import _native as nat
from .compat import HAVE_SB3, VecEnvBase
from .core import BatchedEnv
from .registry import spec_for

# attribute name -> (first plane, count) per system, for get_attr / set_attr
_STATE_ATTRS = {
    nat.LORENZ3: {"state1": (nat.L3_X, 3)},
    nat.LORENZ4: {"state1": (nat.L4_M1, 4), "state2": (nat.L4_S1, 4)},
    nat.PMSM: {"state1": (nat.PMSM_S1, 3), "state2": (nat.PMSM_S2, 3),
               "lambda_coef": (nat.PMSM_LAMBDA, 1), "m_t": (nat.PMSM_M, 1),
               "v_t": (nat.PMSM_V, 1), "adam_step": (nat.PMSM_ADAM_STEP, 1),
               "current_step": (nat.PMSM_STEP, 1)},
    nat.HR: {"state_master": (nat.HR_M, 3), "state_slave": (nat.HR_S, 3),
             "sigma": (nat.HR_SIGMA, 1), "filtered_action": (nat.HR_FA, 2)},
    nat.T1: {"state1": (nat.T1_X, 3)},
    nat.T2: {"state1": (nat.T2_M1, 4), "state2": (nat.T2_S1, 4)},
    nat.TP: {"state1": (nat.TP_M, 3), "state2": (nat.TP_S, 3)},
    nat.SC: {"state1": (nat.SC_X, 3)},
}


class LazyInfos(Sequence):
    """List-like infos: a dict is materialised only when an env's entry is touched
    (building N dicts per step dominates at 1M envs).  Mutations persist."""

    def __init__(self, n, done_entries):
        self._n = n
        self._d = done_entries  # env index -> dict

    def __len__(self):
        return self._n

    def __getitem__(self, i):
        if isinstance(i, slice):
            return [self[j] for j in range(*i.indices(self._n))]
        if i < 0:
            i += self._n
        if not 0 <= i < self._n:
            raise IndexError(i)
        d = self._d.get(i)
        if d is None:
            d = self._d[i] = {}
        return d

    def done_indices(self):
        return sorted(k for k, v in self._d.items() if "terminal_observation" in v)


class DeviceLazyInfos(Sequence):
    """The infos of a `return_tensors=True` step, sync-free until touched: the step's
    done bytes and compact done list stay in device tensors of their own, and the
    first access synchronises once and materialises the done envs' dicts
    ("terminal_observation" as a device tensor row, "TimeLimit.truncated")."""

    def __init__(self, n, done, done_idx, term_obs, n_done, host=False):
        self._n = n
        self._dev = (done, done_idx, term_obs, n_done)
        self._li = None
        self._host = host  # terminal observations as NumPy float32 rows

    def _mat(self):
        if self._li is None:
            done, didx, tobs, nd = self._dev
            m = int(nd.item())
            idx = didx[:m].cpu().numpy()
            flags = done.cpu().numpy()
            t = tobs[:m].float()
            if self._host:
                t = t.cpu().numpy()
            entries = {}
            for j, i in enumerate(idx):
                f = int(flags[i])
                entries[int(i)] = {
                    "terminal_observation": t[j],
                    "TimeLimit.truncated": bool(f & nat.DONE_TRUNCATED) and not bool(
                        f & nat.DONE_TERMINATED)}
            self._li = LazyInfos(self._n, entries)
            self._dev = None
        return self._li

    def __len__(self):
        return self._n

    def __getitem__(self, i):
        return self._mat()[i]

    def done_indices(self):
        return self._mat().done_indices()


class _StepInfos(DeviceLazyInfos):
    """DeviceLazyInfos over one return_tensors step's output buffer (views built on
    first access)."""

    def __init__(self, n, buf, offs, sizes, td, o):
        self._n = n
        self._buf = (buf, offs, sizes, td, o)
        self._li = None
        self._host = False

    def _mat(self):
        if self._li is None:
            buf, offs, sizes, td, o = self._buf
            n = self._n
            idx = buf[offs[3]: offs[3] + 4 * (n + 1)].view(torch.int32)
            self._dev = (buf[offs[2]: offs[2] + n], idx[:n],
                         buf[offs[4]: offs[4] + sizes[4]].view(td).view(n, o), idx[n:])
            self._buf = None
        return super()._mat()


class LorenzVecEnv(VecEnvBase):
    def __init__(self, env_id="lorenz_dynamic-v0", num_envs=1, device=None, dtype="float32",
                 seed=0, max_episode_steps=None, return_tensors=False, lazy_infos=None,
                 global_env_offset=0, backend=None, **env_kwargs):
        spec = spec_for(env_id)
        self.spec = spec
        if max_episode_steps is None:
            max_episode_steps = spec.max_episode_steps or 0
        self.system = spec.system
        obs_space, act_space = spec.spaces()
        if backend is None:
            backend = BatchedEnv(spec.system_name, num_envs, dtype=dtype, device=device, seed=seed,
                                 global_env_offset=global_env_offset,
                                 max_episode_steps=max_episode_steps, autoreset=True,
                                 **env_kwargs)
        self.backend = backend
        self.return_tensors = return_tensors
        self.lazy_infos = (num_envs > 1024) if lazy_infos is None else lazy_infos
        self._actions = None
        self._seed = seed
        if HAVE_SB3:  # pragma: no cover - SB3 not installed in this image
            super().__init__(num_envs, obs_space, act_space)
        else:
            self.num_envs = num_envs
            self.observation_space = obs_space
            self.action_space = act_space
            self.render_mode = None
            self.reset_infos = [{} for _ in range(num_envs)]
        self.metadata = {"render_modes": []}
        self._pin_act = self._pin_out = self._dev_act = None
        self._layout = None
        if not return_tensors and isinstance(backend, BatchedEnv):
            # host-buffer path: pinned staging, one copy each way
            self._pin_act = torch.empty((num_envs, backend.action_dim), dtype=torch.float32,
                                        pin_memory=True)
            self._pin_out = torch.empty(backend.packed.shape, dtype=torch.uint8, pin_memory=True)
            self._dev_act = torch.empty((num_envs, backend.action_dim), dtype=torch.float32,
                                        device=backend.device)

    # ------------------------------------------------------------------ conversions
    def _host_results(self):
        """obs float32 [N, O], rewards float32 [N], done bytes [N] as NumPy arrays: one
        pinned D2H copy of the packed obs|rew|done buffer, then one host copy each
        (SB3's DummyVecEnv also hands out copies)."""
        be = self.backend
        self._pin_out.copy_(be.packed, non_blocking=True)
        torch.cuda.current_stream(be.device).synchronize()
        raw = self._pin_out.numpy()
        n, o = self.num_envs, be.obs_dim
        dt = np.float64 if be.tdtype == torch.float64 else np.float32
        es = np.dtype(dt).itemsize
        obs = raw[: n * o * es].view(dt).reshape(n, o).astype(np.float32)
        rew = raw[n * o * es: n * (o + 1) * es].view(dt).astype(np.float32)
        done = raw[n * (o + 1) * es:].copy()
        return obs, rew, done
    def _out(self, t, np_dtype):
        if self.return_tensors:
            return t
        return t.detach().cpu().numpy().astype(np_dtype, copy=False)

    # ------------------------------------------------------------------ VecEnv API
    def reset(self):
        obs = self.backend.reset()
        self.reset_infos = [{} for _ in range(self.num_envs)] if not self.lazy_infos else \
            LazyInfos(self.num_envs, {})
        if self.return_tensors:
            return obs.float() if obs.dtype != torch.float32 else obs.clone()
        if self._pin_out is not None:
            return self._host_results()[0]
        return obs.detach().cpu().numpy().astype(np.float32)

    def step_async(self, actions):
        self._actions = actions

    def device_actions(self, acts):
        """Host actions through the pinned staging buffer (one H2D copy); device
        tensors pass through."""
        if not isinstance(acts, torch.Tensor) and self._pin_act is not None:
            np.copyto(self._pin_act.numpy(),
                      np.asarray(acts, dtype=np.float32).reshape(self.num_envs, -1))
            self._dev_act.copy_(self._pin_act, non_blocking=True)
            return self._dev_act
        if not isinstance(acts, torch.Tensor):
            return torch.from_numpy(np.asarray(acts, dtype=np.float32).reshape(self.num_envs, -1))
        return acts

    def step_wait(self):
        acts = self.device_actions(self._actions)
        if self.return_tensors and isinstance(self.backend, BatchedEnv):
            # sync-free: one fresh allocation per step for every output (the caching
            # allocator recycles it once the caller drops the views), addresses straight
            # into lz_step, views only for what is returned; the compact done list is
            # viewed lazily by DeviceLazyInfos
            be, n = self.backend, self.num_envs
            if self._layout is None:
                o, es = be.obs_dim, torch.empty((), dtype=be.tdtype).element_size()
                sizes = [n * o * es, n * es, n, 4 * (n + 1), n * o * es]  # obs rew done idx tobs
                offs = np.concatenate([[0], np.cumsum([(b + 15) // 16 * 16 for b in sizes])])
                self._layout = (int(offs[-1]), [int(x) for x in offs[:-1]], sizes, o)
            total, offs, sizes, o = self._layout
            buf = torch.empty((total,), dtype=torch.uint8, device=be.device)
            base = buf.data_ptr()
            a = be._check_dev(acts, torch.float32, (n, be.action_dim), "actions")
            nat.check(nat.lib.lz_step(be._h, a.data_ptr(), None, base + offs[0], base + offs[1],
                                      base + offs[2], base + offs[3], base + offs[4],
                                      base + offs[3] + 4 * n))
            be._last_actions = a
            td = be.tdtype
            obs = buf[offs[0]: offs[0] + sizes[0]].view(td).view(n, o)
            rew = buf[offs[1]: offs[1] + sizes[1]].view(td)
            done = buf[offs[2]: offs[2] + n]
            infos = _StepInfos(n, buf, offs, sizes, td, o)
            obs_o = obs.float() if td != torch.float32 else obs
            rew_o = rew.float() if td != torch.float32 else rew
            return obs_o, rew_o, done.bool(), infos
        obs, rew, done = self.backend.step(acts)
        if self.return_tensors:
            obs_o = obs.float() if obs.dtype != torch.float32 else obs.clone()
            rew_o = rew.float() if rew.dtype != torch.float32 else rew.clone()
            done_h = done.cpu().numpy()
            dones = done.bool()
        elif self._pin_out is not None:
            obs_o, rew_o, done_h = self._host_results()
            dones = done_h.astype(bool)
        else:  # a test double of the backend
            obs_o = obs.detach().cpu().numpy().astype(np.float32)
            rew_o = rew.detach().cpu().numpy().astype(np.float32)
            done_h = done.cpu().numpy()
            dones = done_h.astype(bool)
        entries = {}
        if done_h.any():
            idx, tobs = self.backend.done_list()
            idx = idx.cpu().numpy()
            tobs = tobs.float() if self.return_tensors else tobs.cpu().numpy().astype(np.float32)
            for j, i in enumerate(idx):
                flag = int(done_h[i])
                entries[int(i)] = {
                    "terminal_observation": tobs[j],
                    "TimeLimit.truncated": bool(flag & nat.DONE_TRUNCATED) and not bool(
                        flag & nat.DONE_TERMINATED),
                }
        if self.lazy_infos:
            infos = LazyInfos(self.num_envs, entries)
        else:
            infos = [entries.get(i, {}) for i in range(self.num_envs)]
        return obs_o, rew_o, dones, infos

    def step(self, actions):
        self.step_async(actions)
        return self.step_wait()

    def close(self):
        self.backend.close()

    def seed(self, seed=None):
        """SB3: seeds take effect at the next reset (on-device Philox key)."""
        if seed is None:
            seed = int(np.random.randint(0, 2 ** 31 - 1))
        self._seed = seed
        self.backend.set_seed(seed)
        return [seed + i for i in range(self.num_envs)]

    def _indices(self, indices):
        if indices is None:
            return list(range(self.num_envs))
        if isinstance(indices, int):
            return [indices]
        return list(indices)

    def get_attr(self, attr_name, indices=None):
        """SB3 VecEnv.get_attr: state attributes read as a device gather of the requested
        envs only (lz_get_state with indices)."""
        idx = self._indices(indices)
        attrs = _STATE_ATTRS[self.system]
        if attr_name in attrs:
            first, cnt = attrs[attr_name]
            ids = None if indices is None else idx
            cols = [self.backend.get_state(first + j, ids).cpu().numpy() for j in range(cnt)]
            vals = np.stack(cols, axis=1)
            rows = range(len(idx))
            return [vals[r] if cnt > 1 else vals[r, 0] for r in rows]
        if attr_name in ("observation_space", "action_space", "render_mode", "metadata", "spec"):
            return [getattr(self, attr_name) for _ in idx]
        raise AttributeError("LorenzVecEnv: unknown env attribute %r" % attr_name)

    def set_attr(self, attr_name, value, indices=None):
        """SB3 VecEnv.set_attr: every requested env gets `value` (the reference's
        `base_env.state1 = np.array([10, -10, 15])`, code/lorenz_pmsm/test_evaluate.py:
        100-102), written as a device scatter into those envs only (lz_set_state with
        indices) -- the other envs' state is not touched."""
        idx = self._indices(indices)
        attrs = _STATE_ATTRS[self.system]
        if attr_name not in attrs:
            raise AttributeError("LorenzVecEnv: attribute %r is not settable" % attr_name)
        first, cnt = attrs[attr_name]
        v = np.asarray(value, dtype=np.float64)
        if cnt > 1 and v.shape[-1:] != (cnt,):
            raise ValueError("%s takes %d components, got shape %s" % (attr_name, cnt, v.shape))
        for j in range(cnt):
            vj = v[..., j] if cnt > 1 else v
            self.backend.set_state(first + j, np.broadcast_to(vj, (len(idx),)).copy(), idx)

    def env_method(self, method_name, *method_args, indices=None, **method_kwargs):
        idx = self._indices(indices)
        if method_name.startswith("get_current") or method_name.startswith("_get_current"):
            k = method_name.rsplit("current", 1)[1]
            comp = int(k) if k else 0
            # (master first plane, slave first plane or None: the reference's state2
            # is an all-zero array for the single-system variants)
            pairs = {nat.LORENZ4: (nat.L4_M1, nat.L4_S1), nat.LORENZ3: (nat.L3_X, None),
                     nat.T1: (nat.T1_X, None), nat.T2: (nat.T2_M1, nat.T2_S1),
                     nat.TP: (nat.TP_M, nat.TP_S), nat.SC: (nat.SC_X, None)}
            if self.system in pairs:
                mf, sf = pairs[self.system]
                m = self.backend.get_state(mf + comp).cpu().numpy()
                if sf is None:
                    return [[m[i], 0] for i in idx]
                s = self.backend.get_state(sf + comp).cpu().numpy()
                return [[m[i], s[i]] for i in idx]
        raise AttributeError("LorenzVecEnv: unsupported env_method %r" % method_name)

    def env_is_wrapped(self, wrapper_class, indices=None):
        return [False for _ in self._indices(indices)]

    def get_images(self):
        return [None for _ in range(self.num_envs)]

    def render(self, mode=None):
        return None
