"""Shared plumbing of the per-env drop-in classes: one env = a 1-lane BatchedEnv.

The reference's per-env classes draw their initial states (and, for PMSM / HR, their
per-step noise) from NumPy RNGs on the host -- the global MT19937 (`np.random`) or
the gymnasium-seeded PCG64 (`self.np_random`).  The drop-in classes make exactly
the same host draws in the same order, so a caller's RNG streams evolve as with the
reference, and inject the values into the kernel (lz_reset init / lz_step noise);
every dynamics, observation, reward and done computation runs in the HIP kernel.
"""
import numpy as np
import torch

from .. import _native as nat
from ..core import BatchedEnv


class SingleEnvCore:
    """A 1-env handle plus the host<->device marshalling of one step."""

    def __init__(self, system, dtype, device=None, **kw):
        self.be = BatchedEnv(system, 1, dtype=dtype, device=device, autoreset=False,
                             compact=False, max_episode_steps=0, **kw)
        self._np_dtype = np.float64 if self.be.tdtype == torch.float64 else np.float32
        self._act = torch.zeros((1, self.be.action_dim), dtype=torch.float32,
                                device=self.be.device)
        self._noise = torch.zeros((1, 3), dtype=torch.float64, device=self.be.device)
        o = self.be.obs_dim
        es = np.dtype(self._np_dtype).itemsize
        self._o_end = o * es
        self._r_end = (o + 1) * es

    def _unpack(self):
        raw = self.be.packed.cpu().numpy()  # one D2H copy: obs | rew | done
        obs = raw[: self._o_end].view(self._np_dtype).copy()
        rew = raw[self._o_end: self._r_end].view(self._np_dtype)[0]
        done = int(raw[self._r_end])
        return obs, rew, done

    def reset(self, init):
        init_t = torch.as_tensor(np.asarray(init, dtype=self._np_dtype).reshape(1, -1))
        self.be.reset(init=init_t)
        return self._unpack()[0]

    def step(self, action, noise=None):
        a = np.asarray(action, dtype=np.float32).reshape(1, -1)
        self._act.copy_(torch.from_numpy(a))
        nz = None
        if noise is not None:
            self._noise.copy_(torch.from_numpy(np.asarray(noise, dtype=np.float64).reshape(1, 3)))
            nz = self._noise
        self.be.step(self._act, nz, want_n_done=False)
        return self._unpack()

    def plane(self, p):
        return self.be.get_state(p).cpu().numpy()[0]

    def planes(self, first, count):
        return np.array([self.plane(first + j) for j in range(count)])

    def set_planes(self, first, values, dtype=None):
        values = np.asarray(values).reshape(-1)
        for j, v in enumerate(values):
            self.be.set_state(first + j, torch.tensor([v], dtype=self.be.plane_dtype(first + j)))

    def close(self):
        self.be.close()


DONE_TERMINATED = nat.DONE_TERMINATED
DONE_TRUNCATED = nat.DONE_TRUNCATED
