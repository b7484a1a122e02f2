"""The RK4 integrator mode of LORENZ3 / LORENZ4 (lz_config.integrator = LZ_INT_RK4) on
the CPU: the C oracle's restatement against an independent vectorised NumPy float64
RK4 of the reference's right-hand sides.

PARITY UNPINNED against the reference: the reference's Lorenz envs integrate with
forward Euler (code/gym-lorenz/gym_lorenz/envs/dynamic.py:70-75,
lorenz_env_transient.py:327-351); its only RK4 is the Hindmarsh-Rose env
(lorenz_env_try.py:100-113), whose stage order this mode follows.  So the pins here
are (i) a NumPy restatement written from those two reference files, vectorised and
independent of the C code, and (ii) the integrator's defining property, fourth-order
convergence.  The GPU kernels are checked against this oracle bit for bit
(tests/test_gpu_rk4.py)."""
import numpy as np
import pytest

pytestmark = pytest.mark.filterwarnings("ignore::RuntimeWarning")  # diverging envs (IEEE inf/NaN)

from conftest import bits_equal, golden

L3 = dict(sigma=10.0, rho=28.0, beta=8.0 / 3.0, dt=0.01, clip=500.0)


def np_l3_rhs(s):
    """dynamic.py:70-72 (self.u = 10, self.i = 28, self.o = 8/3), one row per env."""
    x, y, z = s[:, 0], s[:, 1], s[:, 2]
    return np.stack([L3["sigma"] * (y - x), L3["rho"] * x - y - x * z, x * y - L3["beta"] * z], 1)


def np_rk4(f, s, dt):
    """lorenz_env_try.py:101-105's stage order, with NumPy's own evaluation order."""
    k1 = f(s)
    k2 = f(s + dt / 2 * k1)
    k3 = f(s + dt / 2 * k2)
    k4 = f(s + dt * k3)
    return s + (dt / 6.0) * (k1 + 2 * k2 + 2 * k3 + k4)


def np_l3_step_rk4(s, a):
    """dynamic.py:61-84 with the Euler update replaced by RK4: clip, integrate, + u,
    obs = [s', f(s')], reward = -sum|s'|."""
    u = np.clip(a, -L3["clip"], L3["clip"]).astype(np.float64)
    s = np_rk4(np_l3_rhs, s, L3["dt"]) + u
    obs = np.concatenate([s, np_l3_rhs(s)], 1)
    rew = -(((0 + np.abs(obs[:, 0])) + np.abs(obs[:, 1])) + np.abs(obs[:, 2]))
    return s, obs, rew


L4 = dict(a=10.0, b=8.0 / 3.0, c=28.0, dt=0.001)


def np_l4_rhs(v):
    """lorenz_env_transient.py:323-326."""
    x1, x2, x3, x4 = v[:, 0], v[:, 1], v[:, 2], v[:, 3]
    return np.stack([L4["a"] * (x2 - x1) + x4, L4["c"] * x1 - x2 - x1 * x3,
                     x1 * x2 - L4["b"] * x3, -x1 * x2 - L4["b"] * x3], 1)


def test_l3_rk4_oracle_equals_numpy_restatement(orc):
    """1000 steps of the golden's 14 initial states and actions: the C oracle (fp64)
    reproduces the NumPy RK4 bit for bit (so well inside the 1e-12 relative gate), NaN-
    aware -- the same IEEE operations in the same order."""
    g = golden("l3")
    st = np.ascontiguousarray(g["x0"].copy())
    s_np = g["x0"].copy()
    worst = 0.0
    for k in range(1000):
        a = g["actions"][:, k]
        o, r = orc.l3_step_rk4(st, a)
        s_np, o_np, r_np = np_l3_step_rk4(s_np, a)
        fin = np.isfinite(o_np)
        if fin.any():
            worst = max(worst, float(np.max(np.abs(o[fin] - o_np[fin]) / np.maximum(np.abs(o_np[fin]), 1.0))))
        assert bits_equal(o, o_np), k
        assert bits_equal(r, r_np), k
        assert bits_equal(st, s_np), k
    assert worst <= 1e-12


def test_l4_rk4_oracle_equals_numpy_restatement(orc):
    g = golden("l4")
    st = np.ascontiguousarray(g["init"].copy())
    m, s = g["init"][:, :4].copy(), g["init"][:, 4:].copy()
    for k in range(1000):
        o, r, d = orc.l4_step_rk4(st)
        m = np_rk4(np_l4_rhs, m, L4["dt"])
        s = np_rk4(np_l4_rhs, s, L4["dt"])
        o_np = np.concatenate([m - s, np_l4_rhs(m) - np_l4_rhs(s)], 1)
        r_np = -((((0 + np.abs(o_np[:, 0])) + np.abs(o_np[:, 1])) + np.abs(o_np[:, 2])) + np.abs(o_np[:, 3]))
        assert bits_equal(o, o_np), k
        assert bits_equal(r, r_np), k
        assert np.array_equal(d, r_np < -1e6), k


@pytest.mark.parametrize("dtype", [np.float64, np.float32])
def test_l3_rk4_is_fourth_order(orc, dtype):
    """The mode is really RK4: with the action at 0 and dt halved, the one-step error
    against a 64-substep reference solution falls by ~2^5 (local error O(dt^5)); Euler's
    falls by ~2^2.  Checked in float64 (float32 rounding swamps the small-dt error, so
    there only: RK4's one-step error is far below Euler's)."""
    rng = np.random.default_rng(3)
    x0 = rng.uniform(-15, 15, (256, 3))

    def fine(s, dt):  # reference solution: 64 RK4 substeps (NumPy, float64)
        for _ in range(64):
            s = np_rk4(np_l3_rhs, s, dt / 64)
        return s

    def one(step_fn, dt):
        p = list(orc.PARAMS["l3"])
        old = orc.PARAMS["l3"]
        orc.PARAMS["l3"] = p[:3] + [dt] + p[4:]
        try:
            st = np.ascontiguousarray(x0.astype(dtype))
            if step_fn == "rk4":
                orc.l3_step_rk4(st, np.zeros((256, 3), np.float32))
            else:
                orc.l3_step(st, np.zeros((256, 3), np.float32))
        finally:
            orc.PARAMS["l3"] = old
        return np.max(np.abs(st.astype(np.float64) - fine(x0, dt)))

    e_rk4 = [one("rk4", dt) for dt in (0.01, 0.005)]
    e_eul = [one("euler", dt) for dt in (0.01, 0.005)]
    assert e_rk4[0] < 1e-3 * e_eul[0]
    if dtype == np.float64:
        assert 24 < e_rk4[0] / e_rk4[1] < 40, e_rk4
        assert 3 < e_eul[0] / e_eul[1] < 5, e_eul
