"""GPU: actions at and beyond the clip bounds, and non-finite actions, through the step
kernels against the oracle -- NaN-aware bit equality.  The reference clips with np.clip
(NaN propagates); the kernels clip float32 actions with IEEE 754-2019 maximum / minimum
(v_maximum3_f32 / v_minimum3_f32, lz_systems.h clip_nz) and float64 with compares: the
same values for every finite, infinite, signed-zero and NaN input (a NaN's payload
aside, which NaN-aware equality ignores)."""
import numpy as np
import pytest
import torch

from conftest import bits_equal

pytestmark = pytest.mark.gpu

SPECIAL = np.array([np.nan, np.inf, -np.inf, 0.0, -0.0, 1.0, -1.0, 1.0000001, -1.0000001,
                    0.5, -0.5, 2.0, -2.0, 500.0, -500.0, 501.0, -501.0, 1e30, -1e30, 1e-45,
                    -1e-45, 3.4e38], np.float32)


def _actions(n, A, seed):
    rng = np.random.default_rng(seed)
    return SPECIAL[rng.integers(0, SPECIAL.size, (n, A))]


def _planes(be, first, cnt):
    return np.stack([be.get_state(first + j).cpu().numpy() for j in range(cnt)], 1)


@pytest.mark.parametrize("dtype", ["float32", "float64"])
def test_lorenz3_edge_actions(orc, dtype):
    import gym_lorenz as gl

    n = 4099
    be = gl.BatchedEnv("lorenz3", n, dtype=dtype, seed=5, autoreset=False, compact=False)
    be.reset()
    st = np.ascontiguousarray(_planes(be, 0, 3))
    for k in range(3):
        a = _actions(n, 3, k)
        o, r, _ = be.step(torch.from_numpy(a))
        with np.errstate(all="ignore"):
            oo, rr = orc.l3_step(st, a)
        assert bits_equal(o.cpu().numpy(), oo), k
        assert bits_equal(r.cpu().numpy(), rr), k
        assert bits_equal(_planes(be, 0, 3), st), k
    be.close()


def test_pmsm_edge_actions(orc):
    import gym_lorenz as gl

    n = 4099
    be = gl.BatchedEnv("pmsm", n, seed=6, autoreset=False, compact=False)
    be.reset()
    S = orc.PmsmState(n)
    S.st[:] = _planes(be, 0, 6)
    for k in range(3):
        a = _actions(n, 2, 10 + k)
        o, r, d = be.step(torch.from_numpy(a))
        with np.errstate(all="ignore"):
            oo, rr, te, tr = orc.pmsm_step(S, a, None, False, 0.5, orc.DEV)
        assert bits_equal(o.cpu().numpy(), oo), k
        assert bits_equal(r.cpu().numpy(), rr), k
        assert np.array_equal((d.cpu().numpy() & 1).astype(bool), te), k
        assert bits_equal(be.get_state(6).cpu().numpy(), S.lam), k  # the Adam dual
    be.close()


@pytest.mark.parametrize("dtype,add_filter", [("float32", False), ("float32", True),
                                              ("float64", True)])
def test_hr_edge_actions(orc, dtype, add_filter):
    import gym_lorenz as gl

    n = 4099
    be = gl.BatchedEnv("hr", n, dtype=dtype, seed=7, autoreset=False, compact=False,
                       add_filter=add_filter)
    be.reset()
    st = np.ascontiguousarray(_planes(be, 0, 6))
    fa = np.zeros((n, 2), np.float32)
    for k in range(3):
        a = _actions(n, 2, 20 + k)
        o, r, d = be.step(torch.from_numpy(a))
        with np.errstate(all="ignore"):
            oo, rr, te = orc.hr_step(st, fa, a, None, False, add_filter, orc.DEV)
        assert bits_equal(o.cpu().numpy(), oo), k
        assert bits_equal(r.cpu().numpy(), rr), k
        assert np.array_equal((d.cpu().numpy() & 1).astype(bool), te), k
    be.close()
