"""The SB3 RunningMeanStd restatement (oracle/sb3_vecnorm.py) combines batches exactly
like one pass over their concatenation (Chan et al.), and VecNormalize's reward
bookkeeping zeroes the returns of done envs."""
import numpy as np

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
