"""GPU parity of the float32 policy rollout (lz_rollout_policy_f32: SURVEY §8 f3 at the
precision SB3 runs its policies in) and the f2 closed loop.

Bars (all bit-exact unless stated):
  * forward: every deterministic action (= the policy mean) and value the fused
    rollout recorded equals oracle.mlp_f32 (lz_oracle.c orc_mlp_f32, the CPU
    restatement of the kernel's operation order) applied to the observation the
    kernel recorded for that step -- per system, with and without VecNormalize, at a
    ragged batch and at 262,147 envs (grid-stride tiles), 128 and 64 hidden units;
    last_values likewise; log_prob bit for bit from the packed Normal constants;
  * env part: bit-exact vs lz_rollout fed the clipped actions
    (test_gpu_policy.py::test_policy_rollout_env_part_bitexact[fp32-*]);
  * sampling: z = (a - mean) / std ~ N(0, 1); log_prob = the kernel's float32 formula;
  * truncation bootstrap: reward = env reward + float32(gamma * V(terminal obs)), V
    from the oracle;
  * against SB3's own arithmetic (torch float32 nn.Linear / Tanh, an SB3-initialised
    policy behind VecNormalize): max |difference| <= 1e-5 of the output scale
    (measured ~1e-6; the fp32 twin of test_policy_bf16_vs_fp32_sb3_init);
  * f2 -- code/lorenz_pmsm/test_evaluate.py:61-166 with the reference's eight trained
    A2C policies and their frozen VecNormalize statistics: the fused closed loop (two
    launches, K = 1999 + 1) equals the oracle closed loop bit for bit (normalised obs,
    actions, final states), which equals the reference env + torch run within 5e-4 on
    state1 - state2 (tests/test_policy_f32_host.py; measured 8.1e-5).
"""
import numpy as np
import pytest
import torch

from test_policy_f32_host import GOLD, normalize_obs, oracle_closed_loop

pytestmark = pytest.mark.gpu

F32_LOGSTD = 2 * 73024  # lz_internal.h kF32LogStd


@pytest.fixture(scope="module")
def gl():
    import gym_lorenz

    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    return gym_lorenz


@pytest.fixture(scope="module")
def pol():
    from gym_lorenz import policy

    return policy


@pytest.fixture(scope="module")
def orc():
    import oracle

    return oracle


def _np(t):
    return t.detach().cpu().numpy()


def _random_policy(pol, O, A, seed, hidden=128, scale=0.4):
    net = pol.ActorCriticMlp(O, A, hidden=hidden, seed=seed)
    g = torch.Generator().manual_seed(seed + 1)
    with torch.no_grad():
        for p in net.parameters():
            p.copy_(torch.randn(p.shape, generator=g) * (scale if p.dim() > 1 else 0.3))
    return net, {k: v.detach().clone() for k, v in net.state_dict().items()}


def _normal_consts(col):
    f = _np(col.blob).view(np.float32)[F32_LOGSTD // 4: F32_LOGSTD // 4 + 16]
    return f[4:8], f[8:12], f[12:16]  # scale, 2 scale^2, log scale


def _logp(d, var2, lscale, A):
    """The kernel's log_prob: sum_j ((-(d*d)) / (2 s^2) - log s) - log(sqrt(2 pi))."""
    lp = None
    for j in range(A):
        dj = d[..., j].astype(np.float32)
        lpj = ((-(dj * dj)) / var2[j] - lscale[j]) - np.float32(0.91893853320467274)
        lp = lpj if lp is None else (lp + lpj).astype(np.float32)
    return lp


def _eq(a, b):
    return np.array_equal(a, b, equal_nan=True)


def _check_forward(orc, sd, b, O, A, rows=None):
    obs = _np(b.observations).reshape(-1, O)
    act = _np(b.actions).reshape(-1, A)
    val = _np(b.values).reshape(-1)
    if rows is not None:
        obs, act, val = obs[rows], act[rows], val[rows]
    m, v = orc.mlp_f32(sd, obs)
    assert _eq(act, m), np.abs(act - m)[np.isfinite(m)].max()
    assert _eq(val, v), np.abs(val - v)[np.isfinite(v)].max()


@pytest.mark.parametrize("system,kw", [
    ("pmsm", dict(add_noise=True, max_episode_steps=5)),
    ("lorenz3", dict(max_episode_steps=4)),
    ("lorenz4", dict(max_episode_steps=3)),
    ("hr", dict(add_noise=True, add_filter=True)),
])
@pytest.mark.parametrize("vecnorm", [False, True])
def test_f32_forward_bitexact_vs_oracle(gl, pol, orc, system, kw, vecnorm):
    from gym_lorenz.vec_normalize import DeviceRunningMeanStd

    n, K = 4099, 6
    env = gl.BatchedEnv(system, n, seed=5, **kw)
    O, A = env.obs_dim, env.action_dim
    _, sd = _random_policy(pol, O, A, seed=7)
    rms = None
    if vecnorm:
        rms = DeviceRunningMeanStd(O, env.device)
        rng = np.random.default_rng(1)
        rms.set_state(rng.normal(0, 2, O), rng.uniform(0.5, 30, O), 1e4)
    col = pol.FusedRolloutCollector(env, sd, bootstrap=False, deterministic=True, obs_rms=rms,
                                    training=False, precision="fp32")
    col.reset()
    b = col.collect(K)
    _check_forward(orc, sd, b, O, A)
    x_last = _np(b.last_obs)
    if vecnorm:
        x_last = np.clip((x_last.astype(np.float64) - rms.mean) / np.sqrt(rms.var + 1e-8),
                         -10.0, 10.0).astype(np.float32)
    _, vl = orc.mlp_f32(sd, x_last)
    assert _eq(_np(b.last_values), vl)
    # deterministic: a = mean, log_prob = sum_j (-log s_j) - log sqrt(2 pi)
    scale, var2, lscale = _normal_consts(col)
    lp = _logp(np.zeros((1, A), np.float32), var2, lscale, A)
    assert np.all(_np(b.log_probs) == lp[0])


def test_f32_narrow_net_and_large_batch(gl, pol, orc):
    """code/lorenz_pmsm/optimize.py's [64, 64] net (zero-padded) at 262,147 envs: many
    tiles per wave (grid-stride loop) and a ragged last tile."""
    n, K = 262147, 3
    env = gl.BatchedEnv("pmsm", n, seed=2, add_noise=True)
    _, sd = _random_policy(pol, 6, 2, seed=11, hidden=64)
    col = pol.FusedRolloutCollector(env, sd, bootstrap=False, deterministic=True, precision="fp32")
    col.reset()
    b = col.collect(K)
    rows = np.random.default_rng(0).choice(K * n, 6000, replace=False)
    rows = np.concatenate([rows, np.arange(K * n - 70, K * n)])  # the ragged last tile
    _check_forward(orc, sd, b, 6, 2, rows)


def test_f32_sampling_and_log_prob(gl, pol, orc):
    n, K = 32768, 4
    env = gl.BatchedEnv("pmsm", n, seed=9)
    _, sd = _random_policy(pol, 6, 2, seed=2)
    sd["log_std"] = torch.tensor([-0.5, 0.25])
    col = pol.FusedRolloutCollector(env, sd, bootstrap=False, precision="fp32")
    col.reset()
    b = col.collect(K)
    obs = _np(b.observations).reshape(-1, 6)
    mean, val = orc.mlp_f32(sd, obs)
    assert _eq(_np(b.values).reshape(-1), val)
    act = _np(b.actions).reshape(-1, 2)
    scale, var2, lscale = _normal_consts(col)
    z = (act - mean) / scale[:2]
    assert abs(z.mean()) < 0.01 and abs(z.std() - 1.0) < 0.01
    assert abs(np.corrcoef(z[:, 0], z[:, 1])[0, 1]) < 0.01
    d = (act - mean).astype(np.float32)
    assert np.array_equal(_np(b.log_probs).reshape(-1), _logp(d, var2, lscale, 2))
    lp_torch = torch.distributions.Normal(torch.from_numpy(mean), torch.exp(sd["log_std"])).log_prob(
        torch.from_numpy(act)).sum(-1).numpy()
    np.testing.assert_allclose(_np(b.log_probs).reshape(-1), lp_torch, rtol=1e-5, atol=1e-5)


def test_f32_truncation_bootstrap(gl, pol, orc):
    n, K, gamma = 2000, 13, 0.97
    ea = gl.BatchedEnv("pmsm", n, seed=21, max_episode_steps=5)
    eb = gl.BatchedEnv("pmsm", n, seed=21, max_episode_steps=5)
    _, sd = _random_policy(pol, 6, 2, seed=4)
    ca = pol.FusedRolloutCollector(ea, sd, gamma=gamma, bootstrap=True, capture_terminal=K * n,
                                   precision="fp32")
    cb = pol.FusedRolloutCollector(eb, sd, gamma=gamma, bootstrap=False, precision="fp32")
    ca.reset()
    cb.reset()
    ba, bb = ca.collect(K), cb.collect(K)
    assert torch.equal(ba.actions, bb.actions)
    d = _np(ba.dones)
    trunc = (d & 2 != 0) & (d & 1 == 0)
    assert trunc.sum() > 0
    ra, rb = _np(ba.rewards), _np(bb.rewards)
    assert np.array_equal(ra[~trunc], rb[~trunc])
    m = int(ba.n_done.item())
    idx = _np(ba.done_idx[:m])
    k, e = idx // n, idx % n
    sel = trunc[k, e]
    _, vt = orc.mlp_f32(sd, _np(ba.terminal_obs[:m]))
    want = (rb[k, e] + (np.float32(gamma) * vt).astype(np.float32)).astype(np.float32)
    assert _eq(ra[k, e][sel], want[sel])


@pytest.mark.parametrize("n", [3001, 40001])  # 40,001: 313 groups on 256 CUs (grid-stride repeats)
@pytest.mark.parametrize("system,kw", [("pmsm", dict(add_noise=True, max_episode_steps=5)),
                                       ("lorenz4", dict(max_episode_steps=4))])
def test_f32_split_kernel_equals_one_wave_kernel(gl, pol, system, kw, n):
    """Below 8 tiles per CU the rollout runs k_rollout_policy_f32_split (pi net + env step
    in waves 0-3, the value net in waves 4-7); lz_config reserved[0] bit 8192 keeps the
    one-wave-per-tile kernel.  Every output of both -- K = 16 with sampling, truncation
    bootstraps, captured terminal obs, VecNormalize statistics, pooled moments, final
    env state -- is bit-identical, at a ragged N (a partly dead last tile and a
    workgroup with dead tiles), and where workgroups run a second tile group (the
    hand-over across the group boundary)."""
    from gym_lorenz.vec_normalize import DeviceRunningMeanStd

    K = 16
    out = []
    for variant in (0, 8192):
        env = gl.BatchedEnv(system, n, seed=41, variant=variant, **kw)
        O, A = env.obs_dim, env.action_dim
        _, sd = _random_policy(pol, O, A, seed=9)
        rms = DeviceRunningMeanStd(O, env.device)
        rng = np.random.default_rng(3)
        rms.set_state(rng.normal(0, 2, O), rng.uniform(0.5, 30, O), 1e4)
        col = pol.FusedRolloutCollector(env, sd, gamma=0.95, bootstrap=True, obs_rms=rms,
                                        training=True, vecnorm_update="rollout",
                                        capture_terminal=K * n, precision="fp32")
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
        for j in range(64):  # every state plane (lz_plane_elem_size 0 ends the list)
            try:
                res["plane%d" % j] = _np(env.get_state(j))
            except ValueError:
                break
        out.append(res)
        env.close()
    assert out[0]["done_idx"].size > 0
    for f in out[0]:
        assert _eq(out[0][f], out[1][f]), f


def test_f32_vs_sb3_fp32_forward(gl, pol):
    """The fp32 twin of test_policy_bf16_vs_fp32_sb3_init: an SB3-initialised policy
    behind VecNormalize against the plain torch float32 forward SB3 computes."""
    from gym_lorenz.vec_normalize import DeviceRunningMeanStd

    for system in ("pmsm", "hr"):
        n, K = 8192, 4
        env = gl.BatchedEnv(system, n, seed=15)
        O, A = env.obs_dim, env.action_dim
        net = pol.ActorCriticMlp(O, A, seed=3)
        rms = DeviceRunningMeanStd(O, env.device)
        col = pol.FusedRolloutCollector(env, net.state_dict(), bootstrap=False, deterministic=True,
                                        obs_rms=rms, training=True, precision="fp32")
        col.reset()
        col.collect(K)
        b = col.collect(K)
        obs = b.observations.reshape(-1, O).cpu()
        fin = torch.isfinite(obs).all(1)
        with torch.no_grad():
            mean32, val32 = net(obs[fin])
        dv = (b.values.reshape(-1).cpu()[fin] - val32).abs().max().item()
        dm = (b.actions.reshape(-1, A).cpu()[fin] - mean32).abs().max().item()
        sv, sm = val32.abs().max().item(), mean32.abs().max().item()
        print("%s fp32 kernel vs torch fp32: value max %.3g (|V| <= %.3g), mean max %.3g "
              "(|mu| <= %.3g)" % (system, dv, sv, dm, sm))
        assert dv <= 1e-5 * max(sv, 1.0)
        assert dm <= 1e-5 * max(sm, 1.0)


def test_f32_vecnormalize_moments(gl, pol):
    """vecnorm_update="rollout" (the pooled opt-in): training statistics from the f32
    kernel's register moments, equal to float64 sums over the raw step outputs (the
    lz_rollout twin's obs) to 1e-12; the policy saw the rollout-start statistics."""
    from gym_lorenz.vec_normalize import DeviceRunningMeanStd

    n, K = 3001, 7
    envp = gl.BatchedEnv("pmsm", n, seed=31, add_noise=True, max_episode_steps=4)
    envr = gl.BatchedEnv("pmsm", n, seed=31, add_noise=True, max_episode_steps=4)
    _, sd = _random_policy(pol, 6, 2, seed=5)
    rms = DeviceRunningMeanStd(6, envp.device)
    col = pol.FusedRolloutCollector(envp, sd, bootstrap=False, obs_rms=rms, training=True,
                                    precision="fp32", vecnorm_update="rollout")
    col.reset()
    envr.reset()
    mean0, var0 = rms.mean.copy(), rms.var.copy()
    b = col.collect(K)
    lo, hi = pol.action_bounds("pmsm")
    obs_r, _, _ = envr.rollout(torch.clamp(b.actions, lo, hi).contiguous())
    raw = _np(obs_r).reshape(-1, 6).astype(np.float64)
    mom = _np(b.obs_moments)
    assert mom[0] == K * n
    np.testing.assert_allclose(mom[1:7], raw.sum(0), rtol=1e-12)
    np.testing.assert_allclose(mom[7:], (raw * raw).sum(0), rtol=1e-12)
    # the policy saw the raw obs normalised with the statistics at rollout start
    seen = np.clip((np.concatenate([_np(col._keep[1])[None], _np(obs_r[:-1])]).astype(np.float64)
                    - mean0) / np.sqrt(var0 + 1e-8), -10, 10).astype(np.float32)
    assert np.array_equal(_np(b.observations), seen)


def test_f2_pmsm_closed_loop_reference_policies(gl, pol, orc):
    """code/lorenz_pmsm/test_evaluate.py:61-166 on the GPU for the 8 trained policies."""
    from gym_lorenz import _native as nat
    from gym_lorenz.vec_normalize import DeviceRunningMeanStd

    gold = np.load(GOLD)
    for j in range(8):
        alpha = float(gold["alphas"][j])
        sd = {k: torch.from_numpy(gold["a%d/%s" % (j, k)]) for k in orc.POLICY_KEYS + ("log_std",)}
        env = gl.BatchedEnv("pmsm", 1, seed=0, alpha=alpha, add_noise=False)
        rms = DeviceRunningMeanStd(6, env.device)
        rms.set_state(gold["a%d/obs_rms.mean" % j], gold["a%d/obs_rms.var" % j],
                      float(gold["a%d/obs_rms.count" % j]))
        col = pol.FusedRolloutCollector(env, sd, obs_rms=rms, training=False, deterministic=True,
                                        bootstrap=False, clip_obs=float(gold["a%d/clip_obs" % j]),
                                        norm_eps=float(gold["a%d/epsilon" % j]), precision="fp32")
        col.reset()
        # :75-76,100-102: inject the fixed initial states
        s1, s2 = gold["init_state1"], gold["init_state2"]
        for i in range(3):
            env.set_state(nat.PMSM_S1 + i, torch.tensor([s1[i]], device=env.device))
            env.set_state(nat.PMSM_S2 + i, torch.tensor([s2[i]], device=env.device))
        # :105-108: the raw obs of the injected state, as the reference computes it on the host
        f = np.float32

        def der(s):
            x1, x2, x3 = s
            return np.array([-x1 + x2 * x3, -x2 - x1 * x3 + f(20.0) * x3, f(5.46) * (x2 - x3)], f)

        raw0 = np.concatenate([s1 - s2, der(s1) - der(s2)]).astype(f)
        col.last_obs = torch.from_numpy(raw0[None]).to(env.device)
        b1 = col.collect(1999)
        st = np.array([_np(env.get_state(p))[0] for p in range(6)], f)
        b2 = col.collect(1)
        obs = np.concatenate([_np(b1.observations), _np(b2.observations)])[:, 0]
        act = np.concatenate([_np(b1.actions), _np(b2.actions)])[:, 0]
        xs, ms, es, st_prev = oracle_closed_loop(gold, j, orc)
        assert np.array_equal(obs, xs), j
        assert np.array_equal(act, ms), j
        assert np.array_equal(st, st_prev), j
        d = np.abs(es[:1999] - gold["cpu_e"][j, :1999]).max()
        print("alpha=%.3f: GPU closed loop == oracle (2000 steps); |e - reference run| <= %.2e"
              % (alpha, d))
        assert d <= 5e-4
        env.close()
