"""LorenzVecNormalize: stable-baselines3 `VecNormalize` with device-resident statistics.

The reference's PMSM callers wrap their env in SB3's VecNormalize
(code/lorenz_pmsm/train.py:118,170: norm_obs=True, norm_reward=False, clip_obs=10;
code/lorenz_pmsm/optimize.py:52).  SB3 keeps RunningMeanStd in host NumPy and touches
every observation on the host each step -- at 1M envs that dominates the step.  This
wrapper keeps the SB3 2.7.1 arithmetic (common/running_mean_std.py, common/vec_env/
vec_normalize.py) but runs it on the GPU over the LorenzVecEnv's device outputs
(lz_rms_* in libgym_lorenz_amd.so):

  step_wait:  obs_rms.update(obs) -> obs = clip((obs - mean) / sqrt(var + eps), +-clip_obs)
              returns = returns * gamma + reward; ret_rms.update(returns)
              reward = clip(reward / sqrt(ret_var + eps), +-clip_reward)
              terminal observations normalised; returns[dones] = 0
  reset:      returns = 0; obs_rms.update(obs); normalised obs

step_wait over a LorenzVecEnv runs as two launches (three above 262,144 envs) and no
host synchronisation (lz_step_vecnorm + lz_vecnorm_apply): the env step kernel also
produces float64 per-workgroup moments of the observations and of the updated
returns; they are reduced in one fixed order (by every workgroup of the normalise
kernel, or above 262,144 envs by a column-total launch), and the normalise kernel
applies the two RunningMeanStd updates and writes the normalised obs / rewards /
terminal observations and the bool dones.  infos are materialised lazily (only done envs get
dicts, on first access).

Multi-GPU: pass `group` (a torch.distributed process group): the batch moments
(count, sum, sum of squares) are all-reduced before every update, so all ranks hold
the statistics of the whole env population (one 2*obs_dim+1 double all-reduce per
statistic per step, RCCL over xGMI).

Statistics are saved / loaded as .npz (no pickle).
"""
import ctypes

import numpy as np
import torch
import torch.distributed as dist

from . import _native as nat
from .core import BatchedEnv
from .vec_env import DeviceLazyInfos, LazyInfos


class _FusedInfos(DeviceLazyInfos):
    """DeviceLazyInfos over the views of a fused step's output buffer."""

    def __init__(self, n, view, host=False):
        self._n = n
        self._view = view
        self._li = None
        self._host = host

    def _mat(self):
        if self._li is None:
            v = self._view
            idx = v(6)
            self._dev = (v(7), idx[: self._n], v(4), idx[self._n:])
            self._view = None
        return super()._mat()


def _p(t):
    return None if t is None else ctypes.c_void_p(t.data_ptr())


def _dt(t):
    return nat.F64 if t.dtype == torch.float64 else nat.F32


class DeviceRunningMeanStd:
    """SB3 RunningMeanStd(epsilon, shape) whose mean / var / count live on the GPU."""

    def __init__(self, dim, device, epsilon=1e-4, stream=None):
        self.dim = dim
        self.device = device
        h = ctypes.c_void_p()
        nat.check(nat.lib.lz_rms_create(dim, device.index, epsilon, ctypes.byref(h)))
        self._h = h
        s = stream if stream is not None else torch.cuda.current_stream(device)
        nat.check(nat.lib.lz_rms_set_stream(h, ctypes.c_void_p(s.cuda_stream)))
        self.moments = torch.zeros((1 + 2 * dim,), dtype=torch.float64, device=device)
        m, v, c = ctypes.c_void_p(), ctypes.c_void_p(), ctypes.c_void_p()
        nat.check(nat.lib.lz_rms_state(h, ctypes.byref(m), ctypes.byref(v), ctypes.byref(c)))
        # [mean..., var..., count] doubles owned by the library, viewed as a tensor
        self.state = _device_view(m.value, (2 * dim + 1,), "<f8", device)

    @property
    def mean(self):
        return self.state[: self.dim].cpu().numpy()

    @property
    def var(self):
        return self.state[self.dim: 2 * self.dim].cpu().numpy()

    @property
    def count(self):
        return float(self.state[-1].item())

    def set_state(self, mean, var, count):
        self.state.copy_(torch.as_tensor(np.concatenate([
            np.asarray(mean, np.float64).reshape(-1), np.asarray(var, np.float64).reshape(-1),
            [float(count)]])))

    def update(self, x, group=None):
        """RunningMeanStd.update(x) over the rows of x [n, dim] (device)."""
        x = x.reshape(x.shape[0], self.dim).contiguous()
        nat.check(nat.lib.lz_rms_moments(self._h, _p(x), _dt(x), x.shape[0], _p(self.moments)))
        if group is not None:
            dist.all_reduce(self.moments, group=group)
        nat.check(nat.lib.lz_rms_update(self._h, _p(self.moments)))

    def normalize(self, x, eps, clip, center=True):
        x = x.contiguous()
        n = x.numel() // self.dim
        y = torch.empty(x.shape, dtype=torch.float32, device=self.device)
        nat.check(nat.lib.lz_rms_normalize(self._h, _p(x), _dt(x), n, _p(y), int(center), eps,
                                           clip))
        return y

    def close(self):
        if getattr(self, "_h", None) is not None:
            nat.lib.lz_rms_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:  # noqa: BLE001
            pass


def _device_view(ptr, shape, typestr, device):
    """A torch view of library-owned device memory (no ownership; the library object
    must outlive it)."""
    class _Iface:
        __cuda_array_interface__ = {"shape": shape, "typestr": typestr, "data": (ptr, False),
                                    "version": 2, "strides": None}

    return torch.as_tensor(_Iface(), device=device)


class LorenzVecNormalize:
    """SB3 VecNormalize API over a LorenzVecEnv (device statistics)."""

    def __init__(self, venv, training=True, norm_obs=True, norm_reward=True, clip_obs=10.0,
                 clip_reward=10.0, gamma=0.99, epsilon=1e-8, group=None):
        self.venv = venv
        self.num_envs = venv.num_envs
        self.observation_space = venv.observation_space
        self.action_space = venv.action_space
        be = venv.backend
        self.device = be.device
        obs_dim = be.obs_dim
        self.obs_rms = DeviceRunningMeanStd(obs_dim, self.device)
        self.ret_rms = DeviceRunningMeanStd(1, self.device)
        self.clip_obs = clip_obs
        self.clip_reward = clip_reward
        self.gamma = gamma
        self.epsilon = epsilon
        self.training = training
        self.norm_obs = norm_obs
        self.norm_reward = norm_reward
        self.group = group
        self.returns = torch.zeros((self.num_envs,), dtype=torch.float64, device=self.device)
        self._moments = torch.zeros((2 * obs_dim + 4,), dtype=torch.float64, device=self.device)
        self._fused = isinstance(be, BatchedEnv) and be.compact
        self._layout = self._vn = self._last = None
        self.old_obs = None
        self.old_reward = None
        self._actions = None

    # --------------------------------------------------------------- normalisation
    def normalize_obs(self, obs):
        if not self.norm_obs:
            return obs
        t = obs if isinstance(obs, torch.Tensor) else torch.as_tensor(np.asarray(obs),
                                                                       device=self.device)
        return self.obs_rms.normalize(t.to(self.device), self.epsilon, self.clip_obs, center=True)

    def normalize_reward(self, reward):
        if not self.norm_reward:
            return reward
        t = reward if isinstance(reward, torch.Tensor) else torch.as_tensor(
            np.asarray(reward), device=self.device)
        return self.ret_rms.normalize(t.to(self.device), self.epsilon, self.clip_reward,
                                      center=False)

    def unnormalize_obs(self, obs):
        st = self.obs_rms.state
        d = self.obs_rms.dim
        t = torch.as_tensor(obs, device=self.device, dtype=torch.float64)
        return (t * torch.sqrt(st[d:2 * d] + self.epsilon) + st[:d]).float()

    def get_original_obs(self):
        if self._last is not None:  # fused step: the raw obs of the last step_wait
            t = self._last[1](0)
            return t if t.dtype == torch.float32 else t.float()
        return self.old_obs

    def get_original_reward(self):
        if self._last is not None:
            t = self._last[1](2)
            return t if t.dtype == torch.float32 else t.float()
        return self.old_reward

    # --------------------------------------------------------------- VecEnv API
    def _dev_outputs(self, actions):
        be = self.venv.backend
        acts = actions if isinstance(actions, torch.Tensor) else torch.from_numpy(
            np.asarray(actions, dtype=np.float32).reshape(self.num_envs, -1))
        return be.step(acts)

    def reset(self):
        obs = self.venv.backend.reset().float()  # SB3 sees DummyVecEnv's float32 obs
        self.old_obs = obs.clone()
        self._last = None
        self.returns.zero_()
        if self.training and self.norm_obs:
            self.obs_rms.update(obs, self.group)
        out = self.normalize_obs(obs)
        return out if self.venv.return_tensors else out.cpu().numpy()

    def step_async(self, actions):
        self._actions = actions

    def _flags(self):
        return ((nat.VN_TRAINING if self.training else 0) | (nat.VN_NORM_OBS if self.norm_obs else 0)
                | (nat.VN_NORM_REWARD if self.norm_reward else 0)
                | (nat.VN_DEFER if self.group is not None else 0))

    def _vn_args(self):
        vn = nat.LzVecNorm()
        vn.obs_rms = self.obs_rms._h.value
        vn.ret_rms = self.ret_rms._h.value
        vn.returns = self.returns.data_ptr()
        vn.moments = self._moments.data_ptr()
        vn.gamma, vn.epsilon = float(self.gamma), float(self.epsilon)
        vn.clip_obs, vn.clip_reward = float(self.clip_obs), float(self.clip_reward)
        vn.flags = self._flags()
        return vn

    def _step_wait_fused(self):
        venv, be = self.venv, self.venv.backend
        n, o, dev, td = self.num_envs, be.obs_dim, self.device, be.tdtype
        if self._layout is None:
            # every output of a step in one fresh allocation per step (the caching
            # allocator recycles it once the caller drops the views): raw obs and
            # terminal obs, raw reward (old_obs, old_reward), normalised obs /
            # terminal obs / reward, compact list + count, done bytes, 0-1 dones.
            # Views are only built for what is returned; the C calls take addresses.
            es = torch.empty((), dtype=td).element_size()
            spec = [(td, (n, o)), (td, (n, o)), (td, (n,)), (torch.float32, (n, o)),
                    (torch.float32, (n, o)), (torch.float32, (n,)), (torch.int32, (n + 1,)),
                    (torch.uint8, (n,)), (torch.uint8, (n,))]
            offs, off = [], 0
            for dt, shp in spec:
                nb = int(np.prod(shp)) * (es if dt == td else torch.empty((), dtype=dt).element_size())
                offs.append((off, nb, dt, shp))
                off += (nb + 15) // 16 * 16
            self._layout = (off, offs)
        total, offs = self._layout
        buf = torch.empty((total,), dtype=torch.uint8, device=dev)
        base = buf.data_ptr()
        p_obs, p_tobs, p_rew, p_on, p_tn, p_rn, p_idx, p_done, p_dones = [base + a for a, _, _, _ in offs]
        p_nd = p_idx + 4 * n
        key = (self._flags(), self.gamma, self.epsilon, self.clip_obs, self.clip_reward)
        if self._vn is None or self._vn[0] != key:
            self._vn = (key, self._vn_args())
        vn = self._vn[1]
        acts = be._check_dev(venv.device_actions(self._actions), torch.float32,
                             (n, be.action_dim), "actions")
        nat.check(nat.lib.lz_step_vecnorm(be._h, vn, acts.data_ptr(), p_obs, p_rew, p_done, p_idx,
                                          p_tobs, p_nd))
        be._last_actions = acts
        if self.group is not None and self.training:
            dist.all_reduce(self._moments, group=self.group)
        nat.check(nat.lib.lz_vecnorm_apply(be._h, vn, p_obs, p_rew, p_done, p_on, p_rn, p_dones,
                                           p_tobs, p_nd, p_tn))

        def view(k):
            a, nb, dt, shp = offs[k]
            return buf[a: a + nb].view(dt).view(shp)

        self._last = (buf, view)  # old_obs / old_reward are built on request
        infos = _FusedInfos(n, view, host=not venv.return_tensors)
        dones = view(8).view(torch.bool)
        if venv.return_tensors:
            return view(3), view(5), dones, infos
        obs_h, rew_h, done_h = view(3).cpu().numpy(), view(5).cpu().numpy(), dones.cpu().numpy()
        if not venv.lazy_infos:
            infos = [infos[i] for i in range(n)]
        return obs_h, rew_h, done_h, infos

    def step_wait(self):
        if self._fused:
            return self._step_wait_fused()
        be = self.venv.backend
        obs, rew, done = self._dev_outputs(self._actions)
        self.old_obs = obs.clone()
        self.old_reward = rew.clone()
        if self.training and self.norm_obs:
            self.obs_rms.update(obs, self.group)
        obs_n = self.normalize_obs(obs)
        dt = nat.F64 if rew.dtype == torch.float64 else nat.F32
        dev = self.device.index
        sp = ctypes.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)
        if self.training:
            nat.check(nat.lib.lz_returns_update(_p(self.returns), _p(rew), dt, None, self.num_envs,
                                                self.gamma, 0, dev, sp))
            self.ret_rms.update(self.returns.view(-1, 1), self.group)
        rew_n = self.normalize_reward(rew) if self.norm_reward else rew.float()
        done_h = done.cpu().numpy()
        infos = [{} for _ in range(self.num_envs)]
        if done_h.any():
            idx, tobs = be.done_list()
            tn = self.normalize_obs(tobs).cpu().numpy() if self.norm_obs else tobs.float().cpu().numpy()
            for j, i in enumerate(idx.cpu().numpy()):
                flag = int(done_h[i])
                infos[int(i)] = {
                    "terminal_observation": tn[j],
                    "TimeLimit.truncated": bool(flag & nat.DONE_TRUNCATED) and not bool(
                        flag & nat.DONE_TERMINATED)}
        nat.check(nat.lib.lz_returns_update(_p(self.returns), None, dt, _p(done), self.num_envs,
                                            self.gamma, 1, dev, sp))
        dones = done_h.astype(bool)
        if self.venv.return_tensors:
            return obs_n, rew_n, done.bool(), infos
        return obs_n.cpu().numpy(), rew_n.cpu().numpy().astype(np.float32), dones, infos

    def step(self, actions):
        self.step_async(actions)
        return self.step_wait()

    def close(self):
        self.obs_rms.close()
        self.ret_rms.close()
        self.venv.close()

    # --------------------------------------------------------------- persistence
    def save(self, path):
        """Statistics as .npz (SB3 pickles the whole wrapper; nothing is pickled here)."""
        np.savez(path, obs_mean=self.obs_rms.mean, obs_var=self.obs_rms.var,
                 obs_count=self.obs_rms.count, ret_mean=self.ret_rms.mean,
                 ret_var=self.ret_rms.var, ret_count=self.ret_rms.count,
                 clip_obs=self.clip_obs, clip_reward=self.clip_reward, gamma=self.gamma,
                 epsilon=self.epsilon)

    def load(self, path):
        with np.load(path, allow_pickle=False) as z:
            self.obs_rms.set_state(z["obs_mean"], z["obs_var"], z["obs_count"])
            self.ret_rms.set_state(z["ret_mean"], z["ret_var"], z["ret_count"])
            self.clip_obs = float(z["clip_obs"])
            self.clip_reward = float(z["clip_reward"])
            self.gamma = float(z["gamma"])
            self.epsilon = float(z["epsilon"])
