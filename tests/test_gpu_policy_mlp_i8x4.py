"""GPU parity of the opt-in i8x4 float32 MlpPolicy rollout (lz_rollout_policy_f32 with
LZ_POLICY_I8X4: each net's 128 -> 128 layer on v_mfma_i32_32x32x32_i8, lz_policy.hip
mlp_i8_tail) against its C restatement (lz_oracle.c orc_mlp_i8x4).

Bars (bit-exact unless stated): every deterministic action and value the rollout
recorded equals oracle.mlp_f32(..., precision="i8x4") on the observation the kernel
recorded, per system, with frozen VecNormalize, in all three kernels (the split kernel
below 8 tiles per CU, the one-wave-per-tile kernel at 4 and 8 waves), 128 and 64 hidden
units; last values and truncation bootstraps likewise; the split and one-wave kernels
agree on every output; a NaN observation poisons only its env; against SB3's torch
float32 forward within 1e-5 of the output scale (as the float32 path)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def gl():
    import gym_lorenz

    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    return gym_lorenz


@pytest.fixture(scope="module")
def pol():
    from gym_lorenz import policy

    return policy


def _np(t):
    return t.detach().cpu().numpy()


def _random_policy(pol, O, A, seed, hidden=128, scale=0.4):
    net = pol.ActorCriticMlp(O, A, hidden=hidden, seed=seed)
    g = torch.Generator().manual_seed(seed + 1)
    with torch.no_grad():
        for p in net.parameters():
            p.copy_(torch.randn(p.shape, generator=g) * (scale if p.dim() > 1 else 0.3))
    return {k: v.detach().clone() for k, v in net.state_dict().items()}


def _eq(a, b):
    return np.array_equal(a, b, equal_nan=True)


def _check_forward(orc, sd, b, O, A, rows=None):
    obs = _np(b.observations).reshape(-1, O)
    act = _np(b.actions).reshape(-1, A)
    val = _np(b.values).reshape(-1)
    if rows is not None:
        obs, act, val = obs[rows], act[rows], val[rows]
    m, v = orc.mlp_f32(sd, obs, precision="i8x4")
    assert _eq(act, m), np.abs(act - m)[np.isfinite(m)].max()
    assert _eq(val, v), np.abs(val - v)[np.isfinite(v)].max()


@pytest.mark.parametrize("system,kw", [
    ("pmsm", dict(add_noise=True, max_episode_steps=5)),
    ("lorenz3", dict(max_episode_steps=4)),
    ("lorenz4", dict(max_episode_steps=3)),
    ("hr", dict(add_noise=True, add_filter=True)),
])
@pytest.mark.parametrize("variant", [0, 8192])  # split kernel / one-wave kernel (4 waves)
def test_i8x4_mlp_forward_bitexact(gl, pol, orc, system, kw, variant):
    from gym_lorenz.vec_normalize import DeviceRunningMeanStd

    n, K = 4099, 6
    env = gl.BatchedEnv(system, n, seed=5, variant=variant, **kw)
    O, A = env.obs_dim, env.action_dim
    sd = _random_policy(pol, O, A, seed=7)
    rms = DeviceRunningMeanStd(O, env.device)
    rng = np.random.default_rng(1)
    rms.set_state(rng.normal(0, 2, O), rng.uniform(0.5, 30, O), 1e4)
    col = pol.FusedRolloutCollector(env, sd, bootstrap=False, deterministic=True, obs_rms=rms,
                                    training=False, precision="i8x4")
    col.reset()
    b = col.collect(K)
    _check_forward(orc, sd, b, O, A)
    x_last = np.clip((_np(b.last_obs).astype(np.float64) - rms.mean) / np.sqrt(rms.var + 1e-8),
                     -10.0, 10.0).astype(np.float32)
    _, vl = orc.mlp_f32(sd, x_last, precision="i8x4")
    assert _eq(_np(b.last_values), vl)
    env.close()


def test_i8x4_mlp_eight_wave_kernel_narrow_net(gl, pol, orc):
    """262,147 envs: the 8-wave one-wave-per-tile kernel, grid-stride tiles, a ragged
    last tile; code/lorenz_pmsm/optimize.py's [64, 64] net zero-padded."""
    n, K = 262147, 3
    env = gl.BatchedEnv("pmsm", n, seed=2, add_noise=True)
    sd = _random_policy(pol, 6, 2, seed=11, hidden=64)
    col = pol.FusedRolloutCollector(env, sd, bootstrap=False, deterministic=True, precision="i8x4")
    col.reset()
    b = col.collect(K)
    rows = np.random.default_rng(0).choice(K * n, 6000, replace=False)
    rows = np.concatenate([rows, np.arange(K * n - 70, K * n)])
    _check_forward(orc, sd, b, 6, 2, rows)
    env.close()


@pytest.mark.parametrize("n", [3001, 40001])
def test_i8x4_mlp_split_equals_one_wave_with_bootstrap(gl, pol, orc, n):
    """Sampling, truncation bootstraps, captured terminal obs, pooled moments: the split
    and the one-wave kernel agree bit for bit, and their values are the oracle's."""
    from gym_lorenz.vec_normalize import DeviceRunningMeanStd

    K, gamma = 16, 0.95
    out = []
    for variant in (0, 8192):
        env = gl.BatchedEnv("pmsm", n, seed=41, variant=variant, add_noise=True, max_episode_steps=5)
        sd = _random_policy(pol, 6, 2, seed=9)
        rms = DeviceRunningMeanStd(6, env.device)
        rng = np.random.default_rng(3)
        rms.set_state(rng.normal(0, 2, 6), rng.uniform(0.5, 30, 6), 1e4)
        col = pol.FusedRolloutCollector(env, sd, gamma=gamma, bootstrap=True, obs_rms=rms,
                                        training=True, vecnorm_update="rollout",
                                        capture_terminal=K * n, precision="i8x4")
        col.reset()
        col.collect(K)
        b = col.collect(K)
        m = int(b.n_done.item())
        idx = _np(b.done_idx[:m])
        order = np.argsort(idx)
        res = {f: _np(getattr(b, f)) for f in ("observations", "actions", "log_probs", "values",
                                               "rewards", "dones", "last_values", "last_obs",
                                               "obs_moments")}
        res["done_idx"] = idx[order]
        res["terminal_obs"] = _np(b.terminal_obs[:m])[order]
        out.append(res)
        # the values and the bootstrap's V(terminal obs): the oracle's bits
        rows = np.random.default_rng(n).choice(K * n, 3000, replace=False)
        _, v = orc.mlp_f32(sd, res["observations"].reshape(-1, 6)[rows], precision="i8x4")
        assert _eq(res["values"].reshape(-1)[rows], v)
        d = res["dones"]
        assert ((d & 2 != 0) & (d & 1 == 0)).sum() > 0  # truncations were bootstrapped
        env.close()
    for f in out[0]:
        assert _eq(out[0][f], out[1][f]), f


def test_i8x4_mlp_vs_sb3_torch_fp32(gl, pol):
    """An SB3-initialised policy (orthogonal init) against the torch float32 forward SB3
    computes: within 1e-5 of the output scale, the float32 path's bar."""
    n = 8192
    env = gl.BatchedEnv("pmsm", n, seed=3, add_noise=True)
    net = pol.ActorCriticMlp(6, 2, seed=3)
    sd = {k: v.detach().clone() for k, v in net.state_dict().items()}
    col = pol.FusedRolloutCollector(env, sd, bootstrap=False, deterministic=True, precision="i8x4")
    col.reset()
    b = col.collect(4)
    obs = b.observations.reshape(-1, 6).cpu()
    with torch.no_grad():
        tm, tv = net(obs)
    act, val = b.actions.reshape(-1, 2).cpu(), b.values.reshape(-1).cpu()
    em = float((act - tm).abs().max() / tm.abs().max())
    ev = float((val - tv).abs().max() / tv.abs().max())
    print("i8x4 MlpPolicy vs torch fp32: mean %.2e value %.2e" % (em, ev))
    assert em < 1e-5 and ev < 1e-5
    env.close()


def test_i8x4_mlp_nan_obs_poisons_its_env_only(gl, pol, orc):
    env = gl.BatchedEnv("lorenz3", 64, seed=3)
    sd = _random_policy(pol, env.obs_dim, env.action_dim, seed=5, scale=0.2)
    col = pol.FusedRolloutCollector(env, sd, bootstrap=False, deterministic=True, precision="i8x4")
    col.reset()
    col.last_obs[9, 1] = float("nan")
    b = col.collect(1)
    act, val = _np(b.actions)[0], _np(b.values)[0]
    assert np.isnan(act[9]).all() and np.isnan(val[9])
    m, v = orc.mlp_f32(sd, _np(b.observations)[0], precision="i8x4")
    assert _eq(act, m) and _eq(val, v)
    env.close()


def test_i8x4_mlp_refusals(gl, pol):
    from gym_lorenz.vec_normalize import DeviceRunningMeanStd

    sd = _random_policy(pol, 6, 2, seed=1)
    env = gl.BatchedEnv("pmsm", 100, seed=1)
    rms = DeviceRunningMeanStd(6, env.device)
    with pytest.raises(ValueError):  # the per-step VecNormalize collect is float32 only
        pol.FusedRolloutCollector(env, sd, obs_rms=rms, training=True, precision="i8x4")
    env.close()
    env = gl.BatchedEnv("transient1", 100, seed=1)
    with pytest.raises(ValueError):  # the legacy systems have no i8x4 instantiation
        pol.FusedRolloutCollector(env, _random_policy(pol, env.obs_dim, env.action_dim, 1),
                                  precision="i8x4")
    env.close()
