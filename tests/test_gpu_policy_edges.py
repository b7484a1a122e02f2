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


def _col(pol, *args, **kw):
    """The bf16-MFMA kernel (this file's restatements are bf16); the float32 kernel has
    its own tests (test_gpu_policy_f32.py)."""
    kw.setdefault("precision", "bf16")
    return pol.FusedRolloutCollector(*args, **kw)


def _sd(pol, O, A):
    net = pol.ActorCriticMlp(O, A, seed=1)
    return {k: v.detach().clone() for k, v in net.state_dict().items()}


@pytest.mark.parametrize("precision", ["bf16", "fp32"])
@pytest.mark.parametrize("n,K", [(1, 1), (31, 3), (33, 2), (64, 1), (65, 4), (257, 3)])
def test_tiny_and_ragged_batches(pol, n, K, precision):
    import gym_lorenz as gl

    envp = gl.BatchedEnv("pmsm", n, seed=3, add_noise=True, max_episode_steps=2)
    envr = gl.BatchedEnv("pmsm", n, seed=3, add_noise=True, max_episode_steps=2)
    col = _col(pol, envp, _sd(pol, 6, 2), bootstrap=False, precision=precision)
    col.reset()
    envr.reset()
    b = col.collect(K)
    obs_r, rew_r, done_r = envr.rollout(torch.clamp(b.actions, -1, 1).contiguous())
    assert torch.equal(b.observations[1:], obs_r[:-1]) and torch.equal(b.last_obs, obs_r[-1])
    assert torch.equal(b.rewards, rew_r) and torch.equal(b.dones, done_r)
    if precision == "fp32":  # the float32 kernel is the oracle's operation order, bit for bit
        import oracle

        _, val = oracle.mlp_f32(_sd(pol, 6, 2), b.observations.reshape(-1, 6).cpu().numpy())
        assert np.array_equal(b.values.reshape(-1).cpu().numpy(), val)
        return
    _, val = pol.reference_forward_bf16(_sd(pol, 6, 2), b.observations.reshape(-1, 6).cpu())
    np.testing.assert_allclose(b.values.reshape(-1).cpu().numpy(), val.numpy(), atol=2e-2,
                               rtol=2e-2)


def test_terminal_list_capacity(pol):
    """More done envs than the compact list holds: n_done counts all of them, only the
    first `cap` entries are written, each a valid (k*N + env) of a done step."""
    import gym_lorenz as gl

    n, K, cap = 500, 6, 37
    env = gl.BatchedEnv("pmsm", n, seed=4, max_episode_steps=2)
    col = _col(pol, env, _sd(pol, 6, 2), capture_terminal=cap)
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
    col = _col(pol, env, sd, deterministic=True, bootstrap=True, gamma=0.9,
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
        _col(pol, env, _sd(pol, 6, 3))  # float64 handle
    env32 = gl.BatchedEnv("lorenz3", 64)
    c = _col(pol, env32, _sd(pol, 6, 3))
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


# lz_episode_starts: SB3's episode_starts buffer of one collect from the done codes,
# exact vs the torch expression it replaced; grid-stride beyond 2,097,152 elements
@pytest.mark.parametrize("n,K", [(1, 1), (5, 1), (300, 7), (4099, 16), (200003, 16)])
def test_episode_starts_exact(pol, n, K):
    from gym_lorenz import _native as nat

    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(n + K)
    done = torch.randint(0, 4, (K, n), device=dev, dtype=torch.uint8, generator=g)
    done[torch.rand((K, n), device=dev, generator=g) < 0.7] = 0
    last_in = (torch.rand(n, device=dev, generator=g) < 0.5).float()
    starts = torch.full((K, n), -7.0, device=dev)
    last_out = torch.full((n,), -7.0, device=dev)
    s = ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
    p = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
    nat.check(nat.lib.lz_episode_starts(n, K, p(done), p(last_in), p(starts), p(last_out), 0, s))
    ref = torch.empty((K, n), device=dev)
    ref[0] = last_in
    if K > 1:
        ref[1:] = (done[:-1] != 0).to(torch.float32)
    assert torch.equal(starts, ref)
    assert torch.equal(last_out, (done[-1] != 0).to(torch.float32))


def test_episode_starts_errors(pol):
    from gym_lorenz import _native as nat

    t = torch.zeros(4, device="cuda:0")
    d = torch.zeros(4, device="cuda:0", dtype=torch.uint8)
    p = lambda x: ctypes.c_void_p(x.data_ptr())  # noqa: E731
    assert nat.lib.lz_episode_starts(4, 1, p(d), p(t), p(t), p(t), 0, None) != 0  # alias
    assert nat.lib.lz_episode_starts(4, 0, p(d), p(t), p(t), None, 0, None) != 0  # K, NULL
    assert nat.lib.lz_episode_starts(0, 1, p(d), p(t), p(t), p(torch.zeros(1, device="cuda:0")),
                                     0, None) == 0  # empty batch: nothing to do
