"""The SB3 RunningMeanStd restatement (oracle/sb3_vecnorm.py) combines batches exactly
like one pass over their concatenation (Chan et al.), and VecNormalize's reward
bookkeeping zeroes the returns of done envs."""
import numpy as np
import pytest

from oracle.sb3_vecnorm import RunningMeanStd, VecNormalizeRef


def test_running_mean_std_batch_merge():
    rng = np.random.default_rng(0)
    a, b = rng.normal(3, 2, (500, 6)), rng.normal(-1, 5, (700, 6))
    r = RunningMeanStd(epsilon=0.0, shape=(6,))
    r.count = 0.0
    r.update(a)
    r.update(b)
    both = np.concatenate([a, b])
    np.testing.assert_allclose(r.mean, both.mean(0), rtol=1e-12)
    np.testing.assert_allclose(r.var, both.var(0), rtol=1e-12)
    assert r.count == 1200


def test_vecnormalize_returns_reset_on_done():
    v = VecNormalizeRef(3, 2)
    v.reset(np.zeros((3, 2)))
    _, r, _, _ = v.step(np.ones((3, 2)), np.array([1.0, 2.0, 3.0]), np.array([False, True, False]))
    assert v.returns[1] == 0 and v.returns[0] == 1.0 and v.returns[2] == 3.0
    assert np.all(np.abs(r) <= 10)


@pytest.mark.parametrize("n", [1, 31, 32, 33, 8192 + 7, 70001])
def test_vn_tile_totals_order(orc, n):
    """The per-step collect's moment order (oracle.vn_tile_totals, restated from
    lz_internal.h PStepArgs) is a float64 sum: within a few ulp of the exact sum, for
    ragged n and n below one tile."""
    import math

    x = np.random.default_rng(n).normal(3.0, 40.0, (n, 6)).astype(np.float32)
    s, q = orc.vn_tile_totals(x)
    xd = x.astype(np.float64)
    for j in range(6):
        es = math.fsum(xd[:, j])
        eq = math.fsum(xd[:, j] * xd[:, j])
        assert abs(s[j] - es) <= 1e-14 * math.fsum(np.abs(xd[:, j])) + 1e-300
        assert abs(q[j] - eq) <= 1e-14 * eq
    # deterministic, and a NaN row propagates as in SB3's np.mean
    assert np.array_equal(orc.vn_tile_totals(x)[0], s)
    x[n // 2, 2] = np.nan
    s2, q2 = orc.vn_tile_totals(x)
    assert np.isnan(s2[2]) and np.isnan(q2[2]) and np.isfinite(s2[[0, 1, 3, 4, 5]]).all()


def test_vn_rms_update_is_update_from_moments(orc):
    """oracle.vn_rms_update == SB3 RunningMeanStd.update_from_moments on the batch mean /
    var derived from the sums (to rounding of the two var formulas)."""
    from oracle.sb3_vecnorm import RunningMeanStd

    x = np.random.default_rng(1).normal(-2.0, 7.0, (5000, 6)).astype(np.float32)
    ref = RunningMeanStd(shape=(6,))
    ref.update(x.astype(np.float64))
    s, q = orc.vn_tile_totals(x)
    m, v, c = orc.vn_rms_update(np.zeros(6), np.ones(6), 1e-4, 5000, s, q)
    np.testing.assert_allclose(m, ref.mean, rtol=1e-12, atol=1e-12)
    np.testing.assert_allclose(v, ref.var, rtol=1e-10)
    assert c == ref.count
