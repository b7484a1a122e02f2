"""Edge cases and error behaviour of lz_rollout_policy / lz_gae (GPU)."""
import ctypes

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def pol():
    from gym_lorenz import policy

    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    return policy


def _sd(pol, O, A):
    net = pol.ActorCriticMlp(O, A, seed=1)
    return {k: v.detach().clone() for k, v in net.state_dict().items()}


@pytest.mark.parametrize("n,K", [(1, 1), (31, 3), (33, 2), (64, 1), (65, 4)])
def test_tiny_and_ragged_batches(pol, n, K):
    import gym_lorenz as gl

    envp = gl.BatchedEnv("pmsm", n, seed=3, add_noise=True, max_episode_steps=2)
    envr = gl.BatchedEnv("pmsm", n, seed=3, add_noise=True, max_episode_steps=2)
    col = pol.FusedRolloutCollector(envp, _sd(pol, 6, 2), bootstrap=False)
    col.reset()
    envr.reset()
    b = col.collect(K)
    obs_r, rew_r, done_r = envr.rollout(torch.clamp(b.actions, -1, 1).contiguous())
    assert torch.equal(b.observations[1:], obs_r[:-1]) and torch.equal(b.last_obs, obs_r[-1])
    assert torch.equal(b.rewards, rew_r) and torch.equal(b.dones, done_r)
    _, val = pol.reference_forward_bf16(_sd(pol, 6, 2), b.observations.reshape(-1, 6).cpu())
    np.testing.assert_allclose(b.values.reshape(-1).cpu().numpy(), val.numpy(), atol=2e-2,
                               rtol=2e-2)


def test_terminal_list_capacity(pol):
    """More done envs than the compact list holds: n_done counts all of them, only the
    first `cap` entries are written, each a valid (k*N + env) of a done step."""
    import gym_lorenz as gl

    n, K, cap = 500, 6, 37
    env = gl.BatchedEnv("pmsm", n, seed=4, max_episode_steps=2)
    col = pol.FusedRolloutCollector(env, _sd(pol, 6, 2), capture_terminal=cap)
    col.reset()
    b = col.collect(K)
    total = int((b.dones != 0).sum().item())
    assert int(b.n_done.item()) == total > cap
    idx = b.done_idx.cpu().numpy()
    d = b.dones.cpu().numpy()
    assert np.all(d[idx // n, idx % n] != 0)
    assert len(set(idx.tolist())) == cap


def test_deterministic_with_bootstrap(pol):
    import gym_lorenz as gl

    n, K = 300, 7
    env = gl.BatchedEnv("lorenz3", n, seed=5, max_episode_steps=3)
    sd = _sd(pol, 6, 3)
    col = pol.FusedRolloutCollector(env, sd, deterministic=True, bootstrap=True, gamma=0.9,
                                    capture_terminal=n * K)
    col.reset()
    b = col.collect(K)
    mean, _ = pol.reference_forward_bf16(sd, b.observations.reshape(-1, 6).cpu())
    np.testing.assert_allclose(b.actions.reshape(-1, 3).cpu().numpy(), mean.numpy(), atol=2e-2,
                               rtol=2e-2)
    assert ((b.dones & 2) != 0).any()


def test_errors(pol):
    import gym_lorenz as gl
    from gym_lorenz import _native as nat

    env = gl.BatchedEnv("lorenz3", 64, dtype="float64")
    with pytest.raises(ValueError):
        pol.FusedRolloutCollector(env, _sd(pol, 6, 3))  # float64 handle
    env32 = gl.BatchedEnv("lorenz3", 64)
    c = pol.FusedRolloutCollector(env32, _sd(pol, 6, 3))
    r = nat.LzPolicyRolloutArgs()
    r.K = 4
    assert nat.lib.lz_rollout_policy(env32._h, ctypes.byref(r)) == nat.LZ_ERR_STATE  # no reset
    env32.reset()
    assert nat.lib.lz_rollout_policy(env32._h, ctypes.byref(r)) == nat.LZ_ERR_INVALID  # NULLs
    r.K = 0
    assert nat.lib.lz_rollout_policy(env32._h, ctypes.byref(r)) == nat.LZ_ERR_INVALID
    r64 = nat.LzPolicyRolloutArgs()
    r64.K = 1
    env.reset()
    assert nat.lib.lz_rollout_policy(env._h, ctypes.byref(r64)) == nat.LZ_ERR_UNSUPPORTED
    del c
