"""GPU: cfg4's on-device process noise (PMSM add_noise=True: N(0, 3) into the slave's
Euler update, lorenz_env_try_pmsm.py:80-93) over all 262,144 envs and many steps.

Each step is teacher-forced: the oracle steps the device's own pre-step state without
noise, so (state2_device - state2_noiseless) / dt recovers the device's noise sample to
within the float32 rounding of the two updates.  Every recovered sample is checked
against the normal the Philox stream prescribes for that env and tick (oracle.
noise_normals: the exact 24-bit uniforms through Box-Muller in float64; the device uses
hardware v_log_f32 / v_sqrt_f32 / v_cos_f32 / v_sin_f32) -- so the tails (u1 -> 0, where
v_log_f32 matters) are checked sample by sample, not only in distribution -- and the
recovered samples as a whole against N(0, 3): KS, moments, kurtosis, the 1e-5 and
1 - 1e-5 quantiles, and independence across components, neighbouring envs and steps."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _planes(be, first, cnt):
    return np.stack([be.get_state(first + j).cpu().numpy() for j in range(cnt)], 1)


def test_device_noise_pmsm_262k_many_steps(orc):
    import gym_lorenz as gl
    from scipy import stats

    n, T, seed = 1 << 18, 8, 3
    dt = float(orc._params("pmsm")[2])
    be = gl.BatchedEnv("pmsm", n, seed=seed, add_noise=True, autoreset=False, compact=False)
    be.reset()
    rng = np.random.default_rng(1)
    rec = np.empty((T, n, 3))
    worst = 0.0
    for t in range(T):
        S = orc.PmsmState(n)
        S.st[:] = _planes(be, 0, 6)
        S.lam[:] = be.get_state(6).cpu().numpy()
        S.m[:] = be.get_state(7).cpu().numpy()
        S.v[:] = be.get_state(8).cpu().numpy()
        S.adam_step[:] = be.get_state(9).cpu().numpy()
        S.cur_step[:] = be.get_state(10).cpu().numpy()
        a = rng.uniform(-1.2, 1.2, (n, 2)).astype(np.float32)
        be.step(torch.from_numpy(a))
        with np.errstate(all="ignore"):
            orc.pmsm_step(S, a, None, False, 0.5, orc.DEV)
        s1 = _planes(be, 0, 3)
        assert np.array_equal(s1.view(np.int32), S.st[:, :3].view(np.int32)), t  # master noiseless
        s2d = _planes(be, 3, 3)
        s2o = S.st[:, 3:]
        r = (s2d.astype(np.float64) - s2o.astype(np.float64)) / dt
        nz = 3.0 * orc.noise_normals(seed, np.arange(n), t + 1)  # reset was tick 0
        tol = ((np.spacing(np.abs(s2d)).astype(np.float64) + np.spacing(np.abs(s2o)))
               / dt * 1.01 + 1e-3 + 1e-5 * np.abs(nz))
        err = np.abs(r - nz)
        assert (err <= tol).all(), (t, float((err / tol).max()), np.argwhere(err > tol)[:5])
        worst = max(worst, float((err / tol).max()))
        rec[t] = r
    z = (rec / 3.0).reshape(-1)
    N = z.size
    ks = stats.kstest(z, "norm")
    kurt = stats.kurtosis(z)  # excess
    q_lo, q_hi = np.quantile(z, [1e-5, 1 - 1e-5])
    qt = stats.norm.ppf(1 - 1e-5)
    tail = int((np.abs(z) > 4).sum())
    tail_exp = 2 * stats.norm.sf(4) * N
    print("device noise: %d samples, KS D %.2e (p %.3f), mean %.1e, std %.5f, excess kurtosis "
          "%.4f, q(1e-5) %.3f / q(1-1e-5) %.3f (N(0,1): -/+%.3f), |z|>4: %d (exp %.0f), "
          "worst err/tol %.3f" % (N, ks.statistic, ks.pvalue, z.mean(), z.std(), kurt, q_lo, q_hi,
                                  qt, tail, tail_exp, worst))
    assert ks.statistic < 2.3 / np.sqrt(N)
    assert abs(z.mean()) < 5 / np.sqrt(N)
    assert abs(z.std() - 1) < 5 / np.sqrt(2 * N)
    assert abs(kurt) < 5 * np.sqrt(24 / N)
    assert abs(q_lo + qt) < 0.15 and abs(q_hi - qt) < 0.15
    assert abs(tail - tail_exp) < 5 * np.sqrt(tail_exp)
    lim = 5 / np.sqrt(n * T)
    c = np.corrcoef(rec.reshape(-1, 3).T)  # across components
    assert np.abs(c - np.eye(3)).max() < lim
    for j in range(3):
        lag = np.corrcoef(rec[1:, :, j].ravel(), rec[:-1, :, j].ravel())[0, 1]  # across steps
        nb = np.corrcoef(rec[:, 1:, j].ravel(), rec[:, :-1, j].ravel())[0, 1]  # neighbour envs
        assert abs(lag) < lim and abs(nb) < lim, (j, lag, nb)
    be.close()
