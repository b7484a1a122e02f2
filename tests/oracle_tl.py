"""Test helper (not a test module): the oracle env batch with gymnasium TimeLimit + SB3
DummyVecEnv auto-reset semantics, as the kernels run them (lz_body.h step_body):

  * step k after a reset uses RNG tick k + 1 (the reset launch took tick 0);
  * an env whose step counter reaches L is truncated (done bit 2), one whose own
    termination fires is terminated (bit 1: LORENZ4's reward < -1e6,
    lorenz_env_transient.py:369);
  * a done env keeps its pre-reset observation as the terminal observation and is reset
    in place from the Philox draws keyed by (seed, global env id, tick).

Drives oracle.l3_step / l4_step (Euler, the reference) or their RK4 mode
(l3_step_rk4 / l4_step_rk4)."""
import numpy as np


class OracleTL:
    def __init__(self, orc, system, dtype, n, seed, L, steps0=None, rk4=False, gids=None):
        """gids: the global env ids of the n rows (a sample of a larger batch; default
        0 .. n - 1): the Philox draws are keyed by the global id, so any subset runs alone."""
        self.orc, self.sys, self.dt, self.seed, self.L = orc, system, dtype, seed, L
        self.rk4 = rk4
        self.gids = None if gids is None else np.ascontiguousarray(gids, dtype=np.int64)
        st = (orc.reset_draw(system, dtype, n, 0, seed, 0) if gids is None
              else orc.reset_draw_idx(system, dtype, self.gids, seed, 0))
        self.st = np.ascontiguousarray(st.copy())
        self.steps = (np.zeros(n, np.int64) if steps0 is None else steps0.astype(np.int64).copy())
        self.tick = 0

    def step(self, a=None):
        orc = self.orc
        self.tick += 1
        with np.errstate(all="ignore"):
            if self.sys == "l3":
                o, r = (orc.l3_step_rk4 if self.rk4 else orc.l3_step)(self.st, a)
                te = np.zeros(len(self.steps), bool)
            else:
                o, r, te = (orc.l4_step_rk4 if self.rk4 else orc.l4_step)(self.st)
        self.steps += 1
        tr = self.steps >= self.L if self.L else np.zeros(len(self.steps), bool)
        d = te.astype(np.uint8) | (tr.astype(np.uint8) << 1)
        idx = np.nonzero(d)[0]
        term = o[idx].copy()
        if idx.size:
            gi = idx if self.gids is None else self.gids[idx]
            fresh = orc.reset_draw_idx(self.sys, self.dt, gi, self.seed, self.tick)
            self.st[idx] = fresh
            o[idx] = orc.l3_reset_obs(fresh) if self.sys == "l3" else orc.l4_reset_obs(fresh)
            self.steps[idx] = 0
        return o, r, d, idx, term
