"""The lane-pair PMSM rollout (lz_kernels.hip k_rollout_pair,
SysPMSM::step_pair; variant bit 1<<27 selects it, reported as LZ_KERNEL_ROLLOUT_PAIR).

Two lanes carry each env: lane q integrates system q (master / slave) and the pair
exchanges states and derivatives by DPP; one division and two square roots per lane
instead of three and four; the slave's normals are drawn two steps at a time (lane 1 this
step's, lane 0 the next step's).  Bar: bit-for-bit equal to K lz_step calls (which draw
their own normals, one env per lane) -- obs, reward, done bytes, the compact done list and
every final state plane -- at the sizes cfg5 runs per GPU and ragged ones, noise on and
off, odd and even K, TimeLimit truncations (auto-reset inside the launch), forced
terminations, alpha = 0.5 (the split square roots) and 0.7 (the float64 pow path).

Reference: lorenz_env_try_pmsm.py:76-184 (noise drawn every step at :80)."""
import numpy as np
import pytest
import torch

from conftest import bits_equal

pytestmark = [pytest.mark.gpu, pytest.mark.filterwarnings("ignore::RuntimeWarning")]

PAIR = 1 << 27


@pytest.fixture(scope="module")
def gl():
    import gym_lorenz

    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    return gym_lorenz


def _np(t):
    return t.detach().cpu().numpy()


@pytest.mark.parametrize("n,K,noise,alpha,arange", [
    (32768, 301, True, 0.5, 1.2), (65536, 200, True, 0.5, 1.2), (4097, 101, True, 0.5, 1.2),
    (4097, 64, False, 0.5, 1.2), (2050, 77, True, 0.7, 1.2), (140001, 40, True, 0.5, 1.2),
    (4099, 60, True, 0.5, 0.0),  # term_threshold 25 (params[10]): es > 25 terminates often
])
def test_pair_rollout_equals_steps(gl, n, K, noise, alpha, arange):
    from gym_lorenz import _native as nat

    kw = {"params": {10: 25.0}} if arange == 0.0 else {}
    arange = arange or 1.2
    a_be = gl.BatchedEnv("pmsm", n, seed=9, max_episode_steps=37, add_noise=noise, alpha=alpha,
                         variant=PAIR, **kw)
    b_be = gl.BatchedEnv("pmsm", n, seed=9, max_episode_steps=37, add_noise=noise, alpha=alpha, **kw)
    sh = nat.launch_shape(a_be._h, nat.CALL_ROLLOUT)
    assert sh["kernel"] == "rollout_pair" and sh["envs_per_wave"] == 32, sh
    assert sh["grid"] == (n + 31) // 32, sh
    a_be.reset()
    b_be.reset()
    A = torch.from_numpy(np.random.default_rng(5).uniform(-arange, arange, (K, n, 2))
                         .astype(np.float32)).cuda()
    obs, rew, done, (didx, tobs, nd) = a_be.rollout(A, capture_terminal=K * n)
    want_idx, want_term = [], 0
    for k in range(K):
        o, r, d = b_be.step(A[k])
        assert bits_equal(_np(obs[k]), _np(o)), k
        assert bits_equal(_np(rew[k]), _np(r)), k
        assert np.array_equal(_np(done[k]), _np(d)), k
        want_idx.append(k * n + np.nonzero(_np(d))[0])
        want_term += int((_np(d) & 1).sum())
    m = int(nd.item())
    wi = np.concatenate(want_idx)
    assert m == wi.size and m > 0
    assert np.array_equal(np.sort(_np(didx[:m])), wi)
    if kw:
        assert want_term > 0  # the termination path ran
    for p in range(a_be.info.n_planes):
        assert bits_equal(_np(a_be.get_state(p)), _np(b_be.get_state(p))), p
    a_be.close()
    b_be.close()


def test_pair_rollout_chained_launches(gl):
    """Two launches back to back (odd K: the second starts on an odd global tick but an even
    k), against the default one-wave kernel on the same inputs."""
    n, K = 8192, 33
    outs = []
    for variant in (0, PAIR):
        be = gl.BatchedEnv("pmsm", n, seed=3, max_episode_steps=20, add_noise=True, variant=variant)
        be.reset()
        g = np.random.default_rng(1)
        res = []
        for _ in range(2):
            A = torch.from_numpy(g.uniform(-1.2, 1.2, (K, n, 2)).astype(np.float32)).cuda()
            o, r, d = be.rollout(A)
            res += [_np(o), _np(r), _np(d)]
        res += [_np(be.get_state(p)) for p in range(be.info.n_planes)]
        outs.append(res)
        be.close()
    for x, y in zip(*outs):
        assert bits_equal(x, y)
