"""BatchedEnv: N independent envs of one system on one GPU, behind the C-ABI.

This is the native batched engine every public surface sits on (the SB3 VecEnv
adapter, the per-env drop-in classes, the multi-GPU shard).  Buffers are torch
CUDA tensors used only as device memory; all env arithmetic runs in the HIP
kernels of libgym_lorenz_amd.so.  There is no CPU path.
"""
import ctypes

import numpy as np
import torch

from . import _native as nat

SYSTEMS = {"lorenz3": nat.LORENZ3, "lorenz4": nat.LORENZ4, "pmsm": nat.PMSM, "hr": nat.HR,
           # legacy, unregistered variants of the reference
           "transient1": nat.T1, "transient2": nat.T2, "transient_pmsm": nat.TP,
           "singlecontrol": nat.SC}
_TDTYPE = {nat.F32: torch.float32, nat.F64: torch.float64}


def _ptr(t):
    return None if t is None else ctypes.c_void_p(t.data_ptr())


def check_buffer(t, name, dtype, numel, device, required=True, at_least=False):
    """One caller-owned buffer handed to the C-ABI as a raw pointer: the ABI has no sizes
    (include/lorenz_env.h lz_step / lz_rollout), so a buffer of the wrong element count is
    an out-of-bounds write on the device.  Refuses (LorenzEnvError LZ_ERR_INVALID) anything
    but a contiguous tensor of exactly `numel` (at_least: at least `numel`, a capacity)
    elements of `dtype` on `device`; returns its ctypes pointer (None for an absent
    optional buffer)."""
    if t is None:
        if required:
            raise nat.LorenzEnvError(nat.LZ_ERR_INVALID, "%s: required buffer is None" % name)
        return None
    if not isinstance(t, torch.Tensor):
        raise nat.LorenzEnvError(nat.LZ_ERR_INVALID, "%s: expected a torch.Tensor, got %s"
                                 % (name, type(t).__name__))
    bad = []
    if t.dtype != dtype:
        bad.append("dtype %s (need %s)" % (t.dtype, dtype))
    if t.device != device:
        bad.append("device %s (need %s)" % (t.device, device))
    if not t.is_contiguous():
        bad.append("not contiguous")
    if t.numel() < numel or (t.numel() != numel and not at_least):
        bad.append("%d elements, shape %s (need %s%d)" % (t.numel(), tuple(t.shape),
                                                          ">= " if at_least else "", numel))
    if bad:
        raise nat.LorenzEnvError(nat.LZ_ERR_INVALID, "%s: %s" % (name, "; ".join(bad)))
    return ctypes.c_void_p(t.data_ptr())


def step_io_args(spec, actions, obs, rew, done, done_idx=None, term_obs=None, n_done=None,
                 noise=None):
    """Validated lz_step arguments after the handle (actions, noise, obs, rew, done,
    done_idx, terminal_obs, n_done) for caller-owned buffers, checked against the
    handle's lz_info: `spec` carries num_envs, obs_dim, action_dim, tdtype and device (a
    BatchedEnv, or the CPU test double) and reads_actions.  actions float32 [N, A] (may
    be None for LORENZ4 / SC, which read none: lz_api.cpp lz_step needs_act); noise
    float64 [N, 3]; obs T [N, O]; rew T [N]; done uint8 [N]; the compact list int32 [>= N]
    + T [>= N, O] (capacities; both or neither) + int32 [1]."""
    n, o, a_dim, td, dev = spec.num_envs, spec.obs_dim, spec.action_dim, spec.tdtype, spec.device
    need_a = getattr(spec, "reads_actions", True)
    pa = check_buffer(actions, "actions", torch.float32, n * a_dim, dev, required=need_a)
    pz = check_buffer(noise, "noise", torch.float64, n * 3, dev, required=False)
    po = check_buffer(obs, "obs", td, n * o, dev)
    pr = check_buffer(rew, "rew", td, n, dev)
    pd = check_buffer(done, "done", torch.uint8, n, dev)
    if (done_idx is None) != (term_obs is None):
        raise nat.LorenzEnvError(nat.LZ_ERR_INVALID, "done_idx and term_obs: both or neither")
    pi = check_buffer(done_idx, "done_idx", torch.int32, n, dev, required=False, at_least=True)
    pt = check_buffer(term_obs, "term_obs", td, n * o, dev, required=False, at_least=True)
    pn = check_buffer(n_done, "n_done", torch.int32, 1, dev, required=False)
    return pa, pz, po, pr, pd, pi, pt, pn


def rollout_io_args(spec, K, actions, obs, rew, done, done_idx=None, term_obs=None, cap=0,
                    n_done=None):
    """Validated lz_rollout arguments after the handle (K, actions, obs, rew, done,
    done_idx, terminal_obs, cap, n_done): time-major actions float32 [K, N, A], obs
    T [K, N, O], rew T [K, N], done uint8 [K, N]; the optional done list int64 [cap] +
    T [cap, O] (both or neither, cap > 0) + int32 [1]."""
    K, cap = int(K), int(cap)
    if K < 1:
        raise nat.LorenzEnvError(nat.LZ_ERR_INVALID, "K must be >= 1, got %d" % K)
    n, o, a_dim, td, dev = spec.num_envs, spec.obs_dim, spec.action_dim, spec.tdtype, spec.device
    need_a = getattr(spec, "reads_actions", True)
    pa = check_buffer(actions, "actions", torch.float32, K * n * a_dim, dev, required=need_a)
    po = check_buffer(obs, "obs", td, K * n * o, dev)
    pr = check_buffer(rew, "rew", td, K * n, dev)
    pd = check_buffer(done, "done", torch.uint8, K * n, dev)
    if (done_idx is None) != (term_obs is None) or (done_idx is not None and cap < 1):
        raise nat.LorenzEnvError(nat.LZ_ERR_INVALID, "done_idx / term_obs: both or neither, "
                                 "with cap >= 1")
    pi = check_buffer(done_idx, "done_idx", torch.int64, cap, dev, required=False)
    pt = check_buffer(term_obs, "term_obs", td, cap * o, dev, required=False)
    pn = check_buffer(n_done, "n_done", torch.int32, 1, dev, required=False)
    return K, pa, po, pr, pd, pi, pt, (cap if pi is not None else 0), pn


class BatchedEnv:
    """One handle = one shard of the env axis on one device and stream.

    Arguments mirror the reference constructors (``add_noise``, ``eval_mode``,
    ``add_filter``, ``alpha``) plus the batching knobs; ``add_noise=None`` keeps the
    system's default (off, except the legacy TP / SC whose noise is unconditional).  ``dtype`` is the state /
    observation precision: "float64" reproduces the reference's fp64 arithmetic
    (LORENZ3 / LORENZ4 bit-exactly), "float32" is the fast path.  PMSM is float32.
    ``integrator``: "euler" (the reference's, default) or "rk4" -- the opt-in RK4 mode of
    lorenz3 / lorenz4 (lz_config.integrator, BASELINE north_star; no reference oracle).
    """

    def __init__(self, system, num_envs, dtype="float32", device=None, seed=0,
                 global_env_offset=0, max_episode_steps=0, autoreset=True, add_noise=None,
                 eval_mode=False, add_filter=False, alpha=None, params=None, compact=True,
                 variant=0, integrator="euler"):
        self.system = SYSTEMS[system] if isinstance(system, str) else int(system)
        self.system_name = {v: k for k, v in SYSTEMS.items()}[self.system]
        if not torch.cuda.is_available():
            raise nat.LorenzEnvError(nat.LZ_ERR_HIP, "no HIP device visible: the env kernels "
                                     "need an MI355X (no CPU fallback)")
        if device is None:
            device = torch.cuda.current_device()
        self.device = torch.device("cuda", device if isinstance(device, int) else
                                   torch.device(device).index or 0)
        cfg = nat.config_init(self.system)
        cfg.dtype = nat.F64 if np.dtype(dtype) == np.float64 else nat.F32
        cfg.num_envs = int(num_envs)
        cfg.global_env_offset = int(global_env_offset)
        cfg.seed = int(seed) & ((1 << 64) - 1)
        cfg.device = self.device.index
        cfg.max_episode_steps = int(max_episode_steps or 0)
        if add_noise is None:  # the system's default (TP / SC: always noisy, as the reference)
            add_noise = bool(cfg.flags & nat.FLAG_ADD_NOISE)
        cfg.flags = ((nat.FLAG_AUTORESET if autoreset else 0) | (nat.FLAG_ADD_NOISE if add_noise else 0)
                     | (nat.FLAG_EVAL_MODE if eval_mode else 0)
                     | (nat.FLAG_ADD_FILTER if add_filter else 0))
        if alpha is not None:
            cfg.alpha = float(alpha)
        cfg.reserved[0] = int(variant)  # step-kernel tuning variant (A/B experiments)
        if isinstance(integrator, str):
            if integrator not in nat.INTEGRATORS:
                raise ValueError("integrator must be one of %s" % sorted(nat.INTEGRATORS))
            integrator = nat.INTEGRATORS[integrator]
        cfg.integrator = int(integrator)
        self.integrator = {v: k for k, v in nat.INTEGRATORS.items()}.get(cfg.integrator, "?")
        if params:
            for k, v in (params.items() if isinstance(params, dict) else enumerate(params)):
                cfg.params[int(k)] = float(v)
        h = ctypes.c_void_p()
        nat.check(nat.lib.lz_create(ctypes.byref(cfg), ctypes.byref(h)))
        self._h = h
        self.stream = torch.cuda.current_stream(self.device)
        nat.check(nat.lib.lz_set_stream(h, ctypes.c_void_p(self.stream.cuda_stream)))
        info = nat.LzInfo()
        nat.check(nat.lib.lz_get_info(h, ctypes.byref(info)))
        self.info = info
        got = nat.LzConfig()
        nat.check(nat.lib.lz_get_config(h, ctypes.byref(got)))
        self.config = got
        self.num_envs = int(num_envs)
        self.obs_dim, self.action_dim, self.init_dim = info.obs_dim, info.action_dim, info.init_dim
        # LORENZ4 / SC read no actions (lz_api.cpp lz_step needs_act)
        self.reads_actions = self.system not in (nat.LORENZ4, nat.SC)
        self.tdtype = _TDTYPE[cfg.dtype]
        self.global_env_offset = int(global_env_offset)
        n, o, dev = self.num_envs, self.obs_dim, self.device
        es = torch.empty((), dtype=self.tdtype).element_size()
        # obs | rew | done packed in one allocation: a single D2H copy brings a small
        # batch's whole step result to the host (per-env drop-in classes)
        self.packed = torch.empty((n * (o + 1) * es + n,), dtype=torch.uint8, device=dev)
        self.obs = self.packed[: n * o * es].view(self.tdtype).view(n, o)
        self.rew = self.packed[n * o * es: n * (o + 1) * es].view(self.tdtype)
        self.done = self.packed[n * (o + 1) * es:]
        self.compact = compact
        if compact:
            self.done_idx = torch.empty((n,), dtype=torch.int32, device=dev)
            self.term_obs = torch.empty((n, o), dtype=self.tdtype, device=dev)
            self.n_done_dev = torch.zeros((1,), dtype=torch.int32, device=dev)
        else:
            self.done_idx = self.term_obs = self.n_done_dev = None

    # ------------------------------------------------------------------ lifecycle
    def close(self):
        if getattr(self, "_h", None) is not None:
            nat.lib.lz_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def bytes_per_env_step(self):
        return self.info.bytes_per_env_step

    def _check_dev(self, t, dtype, shape, name):
        if t is None:
            return None
        if not isinstance(t, torch.Tensor):
            t = torch.as_tensor(np.asarray(t), dtype=dtype)
        if t.device != self.device or t.dtype != dtype or not t.is_contiguous():
            t = t.to(device=self.device, dtype=dtype).contiguous()
        if tuple(t.shape) != tuple(shape):
            raise ValueError("%s: expected shape %s, got %s" % (name, tuple(shape), tuple(t.shape)))
        return t

    # ------------------------------------------------------------------ API
    def reset(self, mask=None, init=None, out=None):
        """Reset selected envs (all if mask is None); init injects initial states
        [N, init_dim] (see lz_reset).  Returns the obs tensor (rows of unselected
        envs keep their previous values)."""
        mask = self._check_dev(mask, torch.uint8, (self.num_envs,), "mask")
        init = self._check_dev(init, self.tdtype, (self.num_envs, self.init_dim), "init")
        if out is None:
            out = self.obs
        else:  # a caller-owned obs buffer: the checked entry's rules (check_buffer)
            check_buffer(out, "out", self.tdtype, self.num_envs * self.obs_dim, self.device)
        nat.check(nat.lib.lz_reset(self._h, _ptr(mask), _ptr(init), _ptr(out)))
        return out

    def step(self, actions, noise=None, want_n_done=True, out=None, compact_out=None):
        """One batched step.  actions: float32 [N, action_dim] (device or host).
        Returns (obs, rew, done) device tensors -- by default internal buffers reused
        by the next call; `out=(obs, rew, done)` writes into caller tensors (e.g. a
        slot of an on-device rollout buffer) instead, and `compact_out=(done_idx int32
        [N], terminal_obs [N, O], n_done int32 [1])` the compact done list."""
        a = self._check_dev(actions, torch.float32, (self.num_envs, self.action_dim), "actions")
        nz = self._check_dev(noise, torch.float64, (self.num_envs, 3), "noise")
        obs, rew, done = (self.obs, self.rew, self.done) if out is None else out
        if compact_out is not None:
            didx, tobs, ndone = compact_out
        else:
            didx, tobs = self.done_idx, self.term_obs
            ndone = self.n_done_dev if (self.compact and want_n_done) else None
        nat.check(nat.lib.lz_step(self._h, *step_io_args(self, a, obs, rew, done, didx, tobs,
                                                         ndone, noise=nz)))
        self._last_actions = a  # keep alive until the stream consumed it
        return obs, rew, done

    def step_args(self, actions, obs, rew, done, done_idx=None, term_obs=None, n_done=None,
                  noise=None):
        """The checked entry for CALLER-OWNED buffers (rollout rings, graph-captured
        loops): every buffer's dtype, device, contiguity and element count checked against
        this handle's lz_info (core.step_io_args), then the pointer tuple that follows
        the handle in lz_step.  Validate once, launch many times:
        ``nat.lib.lz_step(env._h, *env.step_args(...))``.  No conversion: a wrong buffer
        raises LorenzEnvError(LZ_ERR_INVALID) instead of reaching the kernel (an obs slot
        of [N, 3] for LORENZ3's [N, 6] obs would be written 12 B per env past its end)."""
        return step_io_args(self, actions, obs, rew, done, done_idx, term_obs, n_done, noise)

    def step_into(self, actions, obs, rew, done, done_idx=None, term_obs=None, n_done=None,
                  noise=None):
        """lz_step into caller-owned device buffers, checked as step_args."""
        nat.check(nat.lib.lz_step(self._h, *self.step_args(actions, obs, rew, done, done_idx,
                                                           term_obs, n_done, noise)))
        self._last_actions = actions
        return obs, rew, done

    def rollout_args(self, K, actions, obs, rew, done, done_idx=None, term_obs=None, cap=0,
                     n_done=None):
        """lz_rollout's arguments after the handle for caller-owned time-major buffers,
        checked as step_args (core.rollout_io_args)."""
        return rollout_io_args(self, K, actions, obs, rew, done, done_idx, term_obs, cap, n_done)

    def rollout_into(self, K, actions, obs, rew, done, done_idx=None, term_obs=None, cap=0,
                     n_done=None):
        """lz_rollout into caller-owned device buffers, checked as rollout_args."""
        nat.check(nat.lib.lz_rollout(self._h, *self.rollout_args(K, actions, obs, rew, done,
                                                                 done_idx, term_obs, cap, n_done)))
        self._last_actions = actions
        return obs, rew, done

    def step_vecnorm(self, actions, vn, out, compact_out):
        """lz_step_vecnorm: one step plus VecNormalize's statistics bookkeeping
        (`vn` an LzVecNorm).  out = (obs, rew, done) raw outputs, compact_out =
        (done_idx, terminal_obs, n_done); all caller-owned device tensors."""
        a = self._check_dev(actions, torch.float32, (self.num_envs, self.action_dim), "actions")
        obs, rew, done = out
        didx, tobs, ndone = compact_out
        nat.check(nat.lib.lz_step_vecnorm(self._h, ctypes.byref(vn), _ptr(a), _ptr(obs), _ptr(rew),
                                          _ptr(done), _ptr(didx), _ptr(tobs), _ptr(ndone)))
        self._last_actions = a
        return obs, rew, done

    def vecnorm_apply(self, vn, obs, rew, obs_n, rew_n, term=None, n_done=None, term_n=None,
                      done=None, dones=None):
        """lz_vecnorm_apply: the normalised float32 obs / reward / terminal rows and,
        with done / dones, the 0-1 done bytes (a torch.bool view)."""
        nat.check(nat.lib.lz_vecnorm_apply(self._h, ctypes.byref(vn), _ptr(obs), _ptr(rew),
                                           _ptr(done), _ptr(obs_n), _ptr(rew_n), _ptr(dones),
                                           _ptr(term), _ptr(n_done), _ptr(term_n)))

    def done_list(self):
        """(env indices, terminal observations) of envs done in the last step,
        sorted by env index. Synchronises the stream."""
        n = int(self.n_done_dev.item())
        idx = self.done_idx[:n].long()
        order = torch.argsort(idx)
        return idx[order], self.term_obs[:n][order]

    def rollout(self, actions, obs_out=None, rew_out=None, done_out=None, capture_terminal=0):
        """K fused steps in one launch. actions: float32 [K, N, action_dim]."""
        K = int(actions.shape[0])
        a = self._check_dev(actions, torch.float32, (K, self.num_envs, self.action_dim), "actions")
        n, o, dev = self.num_envs, self.obs_dim, self.device
        obs = obs_out if obs_out is not None else torch.empty((K, n, o), dtype=self.tdtype, device=dev)
        rew = rew_out if rew_out is not None else torch.empty((K, n), dtype=self.tdtype, device=dev)
        done = done_out if done_out is not None else torch.empty((K, n), dtype=torch.uint8, device=dev)
        didx = tobs = ndone = None
        if capture_terminal:
            didx = torch.empty((capture_terminal,), dtype=torch.int64, device=dev)
            tobs = torch.empty((capture_terminal, o), dtype=self.tdtype, device=dev)
            ndone = torch.zeros((1,), dtype=torch.int32, device=dev)
        nat.check(nat.lib.lz_rollout(self._h, *rollout_io_args(self, K, a, obs, rew, done, didx, tobs,
                                                                capture_terminal, ndone)))
        self._last_actions = a
        if capture_terminal:
            return obs, rew, done, (didx, tobs, ndone)
        return obs, rew, done

    def plane_dtype(self, plane):
        es = nat.lib.lz_plane_elem_size(self._h, int(plane))
        if es == 0:
            raise ValueError("invalid state plane %d" % plane)
        int_planes = {nat.LORENZ3: (nat.L3_STEP,), nat.LORENZ4: (nat.L4_STEP,),
                      nat.PMSM: (nat.PMSM_ADAM_STEP, nat.PMSM_STEP), nat.HR: (nat.HR_STEP,),
                      nat.T1: (nat.T1_STEP,), nat.T2: (nat.T2_STEP,), nat.TP: (nat.TP_STEP,),
                      nat.SC: (nat.SC_STEP,)}
        if plane in int_planes[self.system]:
            return torch.int32
        return torch.float64 if es == 8 else torch.float32

    def _env_ids(self, indices):
        """Validated device int64 env ids (lz_get_state / lz_set_state skip, not fault
        on, out-of-range ids: reject them here instead)."""
        idx = torch.as_tensor(indices, dtype=torch.int64).reshape(-1)
        if idx.numel() and (int(idx.min()) < 0 or int(idx.max()) >= self.num_envs):
            raise IndexError("env index out of range [0, %d)" % self.num_envs)
        return idx.to(self.device)

    def get_state(self, plane, indices=None):
        """The whole plane, or (indices: env ids) a device gather of those envs."""
        if indices is None:
            t = torch.empty((self.num_envs,), dtype=self.plane_dtype(plane), device=self.device)
            nat.check(nat.lib.lz_get_state(self._h, int(plane), _ptr(t), None, 0))
            return t
        idx = self._env_ids(indices)
        t = torch.empty((idx.numel(),), dtype=self.plane_dtype(plane), device=self.device)
        if idx.numel() == 0:  # (a NULL index list would mean the whole plane)
            return t
        nat.check(nat.lib.lz_get_state(self._h, int(plane), _ptr(t), _ptr(idx), idx.numel()))
        self._last_plane = idx
        return t

    def set_state(self, plane, values, indices=None):
        """The whole plane, or (indices) a device scatter of values[i] into env
        indices[i] (repeated ids: the last occurrence wins, as numpy assignment)."""
        if indices is None:
            t = self._check_dev(values, self.plane_dtype(plane), (self.num_envs,), "plane")
            nat.check(nat.lib.lz_set_state(self._h, int(plane), _ptr(t), None, 0))
            self._last_plane = t
            return
        idx = self._env_ids(indices)
        if idx.numel() == 0:
            return
        v = torch.as_tensor(values, dtype=self.plane_dtype(plane)).reshape(-1).to(self.device)
        v = torch.broadcast_to(v, idx.shape).contiguous()
        if idx.numel() > 1:  # keep the last occurrence of a repeated id, O(count log count)
            srt, perm = torch.sort(idx, stable=True)
            last = torch.ones_like(srt, dtype=torch.bool)
            last[:-1] = srt[1:] != srt[:-1]  # the last of each run of equal ids
            idx, v = srt[last].contiguous(), v[perm[last]].contiguous()
        nat.check(nat.lib.lz_set_state(self._h, int(plane), _ptr(v), _ptr(idx), idx.numel()))
        self._last_plane = (v, idx)

    def set_seed(self, seed):
        """Philox key for subsequent on-device resets and noise (VecEnv.seed)."""
        nat.check(nat.lib.lz_set_seed(self._h, int(seed) & ((1 << 64) - 1)))

    def sync(self):
        nat.check(nat.lib.lz_sync(self._h))
