"""Shared plumbing of the per-env drop-in classes: one env = a 1-lane BatchedEnv.

The reference's per-env classes draw their initial states (and, for PMSM / HR, their
per-step noise) from NumPy RNGs on the host -- the global MT19937 (`np.random`) or
the gymnasium-seeded PCG64 (`self.np_random`).  The drop-in classes make exactly
the same host draws in the same order, so a caller's RNG streams evolve as with the
reference, and inject the values into the kernel (lz_reset init / lz_step noise);
every dynamics, observation, reward and done computation runs in the HIP kernel.
"""
import ctypes
import os

import numpy as np
import torch

from .. import _native as nat
from ..core import BatchedEnv

try:  # the hot call as one CPython C function (csrc/lz_stepper.c); else through ctypes
    from .. import _stepper
except ImportError:  # pragma: no cover - the Makefile builds it next to the library
    _stepper = None


class SingleEnvCore:
    """A 1-env handle plus the host<->device marshalling of one step."""

    def __init__(self, system, dtype, device=None, **kw):
        self.be = BatchedEnv(system, 1, dtype=dtype, device=device, autoreset=False,
                             compact=False, max_episode_steps=0, **kw)
        self._np_dtype = np.float64 if self.be.tdtype == torch.float64 else np.float32
        # host-side inputs / outputs of lz_step_host (pinned staging lives in the library)
        o = self.be.obs_dim
        self._obs_h = np.zeros((1, o), self._np_dtype)
        self._rew_h = np.zeros((1,), self._np_dtype)
        self._done_h = np.zeros((1,), np.uint8)
        self._act_h = np.zeros((1, self.be.action_dim), np.float32)
        self._noise_h = np.zeros((1, 3), np.float64)
        es = np.dtype(self._np_dtype).itemsize
        self._o_end = o * es
        self._r_end = (o + 1) * es
        # lz_resident_step (a resident step server polling the handle's request line: no
        # launch or stream sync per step); LZ_RESIDENT=0 selects lz_step_host.  The hot
        # call goes through nat.lib_fast (no argtypes: the prebuilt c_void_p arguments
        # below pass without per-call conversion, ~0.6 us of a ~1.3 us ctypes call)
        name = "lz_step_host" if os.environ.get("LZ_RESIDENT", "1") == "0" else "lz_resident_step"
        self._step_fn = getattr(nat.lib, name)
        fast = getattr(nat.lib_fast, name)
        fast.restype = ctypes.c_int
        # the host buffers' addresses, looked up once (ndarray.ctypes costs ~0.5 us a call)
        self._p = (self._act_h.ctypes.data, self._noise_h.ctypes.data, self._obs_h.ctypes.data,
                   self._rew_h.ctypes.data, self._done_h.ctypes.data)
        vp = [ctypes.c_void_p(x) for x in self._p]
        h = ctypes.c_void_p(self.be._h.value)
        self._fast = fast
        self._args = (h, vp[0], None, vp[2], vp[3], vp[4])
        self._args_nz = (h, vp[0], vp[1], vp[2], vp[3], vp[4])
        # the same call from C (csrc/lz_stepper.c: no ctypes argument conversion, the obs
        # copy / reward scalar built directly): ~1 us less per env.step()
        self._stepper = None
        if _stepper is not None and os.environ.get("LZ_STEPPER", "1") != "0":
            fn = ctypes.cast(getattr(nat.lib, name), ctypes.c_void_p).value
            self._stepper = _stepper.Stepper(fn, self.be._h.value, *self._p, self._act_h.shape[1], o,
                                             int(self._np_dtype == np.float64))
        # state reads (test_evaluate.py:123-125 reads state1 / state2 several times after
        # every step): one host buffer + address per plane, and the values cached until
        # the next step / reset / write
        npdt = {torch.float64: np.float64, torch.float32: np.float32, torch.int32: np.int32}
        self._pbuf = []
        for q in range(self.be.info.n_planes):
            b = np.zeros((1,), npdt[self.be.plane_dtype(q)])
            self._pbuf.append((b, b.ctypes.data))
        self._ver = 0
        self._pcache = {}

    def _unpack(self):
        raw = self.be.packed.cpu().numpy()  # one D2H copy: obs | rew | done
        obs = raw[: self._o_end].view(self._np_dtype).copy()
        rew = raw[self._o_end: self._r_end].view(self._np_dtype)[0]
        done = int(raw[self._r_end])
        return obs, rew, done

    def reset(self, init):
        self._ver += 1
        init_t = torch.as_tensor(np.asarray(init, dtype=self._np_dtype).reshape(1, -1))
        self.be.reset(init=init_t)
        return self._unpack()[0]

    def step(self, action, noise=None):
        # lz_resident_step / lz_step_host: actions (+ injected noise) in, obs | reward |
        # done out, host memory, one synchronous library call
        sp = self._stepper
        if sp is not None:
            try:
                r = sp.step(action, noise)
            except ValueError:  # a shape numpy broadcasts (e.g. a scalar): the path below
                pass
            else:
                self._ver += 1
                if type(r) is int:
                    nat.check(r)
                return r
        try:
            self._act_h[0] = action  # float32 cast
        except ValueError:  # e.g. a [1, A] action
            self._act_h[...] = np.asarray(action, dtype=np.float32).reshape(1, -1)
        self._ver += 1
        if noise is None:
            st = self._fast(*self._args)
        else:
            try:
                self._noise_h[0] = noise  # float64 cast
            except ValueError:
                self._noise_h[...] = np.asarray(noise, dtype=np.float64).reshape(1, 3)
            st = self._fast(*self._args_nz)
        if st:
            nat.check(st)
        return self._obs_h[0].copy(), self._rew_h[0], int(self._done_h[0])

    def plane(self, p):
        # lz_resident_read_state: while the resident server serves this env, its copy of
        # the state after the last step (the server keeps running -- test_evaluate.py:
        # 123-125 reads state1 / state2 after every step); otherwise a device copy
        b, addr = self._pbuf[p]
        st = nat.lib.lz_resident_read_state(self.be._h, p, addr)
        if st:
            nat.check(st)
        return b[0]

    def planes(self, first, count):
        key = (first, count)
        hit = self._pcache.get(key)
        if hit is not None and hit[0] == self._ver:
            return hit[1].copy()
        vals = np.array([self.plane(first + j) for j in range(count)])
        self._pcache[key] = (self._ver, vals)
        return vals.copy()

    def set_planes(self, first, values, dtype=None):
        self._ver += 1
        values = np.asarray(values).reshape(-1)
        for j, v in enumerate(values):
            self.be.set_state(first + j, torch.tensor([v], dtype=self.be.plane_dtype(first + j)))

    def close(self):
        # the fast paths hold the raw handle address: drop it before lz_destroy frees the
        # handle, so a step after close() gets LZ_ERR_INVALID (a NULL handle), not freed memory
        if self._stepper is not None:
            self._stepper.close()
            self._stepper = None
        self._args = (None,) + self._args[1:]
        self._args_nz = (None,) + self._args_nz[1:]
        self.be.close()


DONE_TERMINATED = nat.DONE_TERMINATED
DONE_TRUNCATED = nat.DONE_TRUNCATED
