"""GPU parity of the fused policy rollout (lz_rollout_policy) and lz_gae.

Bars:
  * env part: bit-exact.  The policy rollout's observations / rewards / dones /
    terminal observations equal those of the action-driven lz_rollout (itself
    bit-exact vs the oracle) fed with the policy's own clipped actions, same seed.
  * policy forward (bf16 MFMA, fp32 accumulate): values and deterministic actions vs
    the torch restatement with the same bf16 roundings (policy.reference_forward_bf16)
    within atol 2e-2 + rtol 2e-2 -- an activation whose fp32 pre-image sits on a bf16
    rounding boundary may round the other way under a different fp32 summation
    order (1 bf16 ulp = 2^-8 relative); the measured max error is printed.  An
    SB3-initialised policy against the plain fp32 forward (what SB3 computes): mean
    abs error < 2% of the output scale (bf16 operand precision), printed.
  * sampling: z = (a - mean) / std ~ N(0, 1) (moments), log_prob = torch
    Normal(mean, std).log_prob(a).sum(-1) within 2e-2.
  * truncation bootstrap: reward - env reward == gamma * V(terminal obs) (torch bf16
    restatement, same tolerance), zero elsewhere.
  * VecNormalize: the observations the policy saw equal lz_rms_normalize of the raw
    observations bit for bit; the moments equal lz_rms_moments (rel 1e-12).
  * lz_gae: bit-exact vs the NumPy restatement of SB3's compute_returns_and_advantage.
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

TOL_A, TOL_R = 2e-2, 2e-2


@pytest.fixture(scope="module")
def gl():
    import gym_lorenz

    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    return gym_lorenz


@pytest.fixture(scope="module")
def pol():
    from gym_lorenz import policy

    return policy


def _col(pol, *args, **kw):
    """The bf16-MFMA kernel (this file's restatements are bf16); the float32 kernel has
    its own tests (test_gpu_policy_f32.py)."""
    kw.setdefault("precision", "bf16")
    return pol.FusedRolloutCollector(*args, **kw)


def _np(t):
    return t.detach().cpu().numpy()


def _random_policy(pol, O, A, seed, scale=0.4):
    net = pol.ActorCriticMlp(O, A, seed=seed)
    g = torch.Generator().manual_seed(seed + 1)
    with torch.no_grad():
        for p in net.parameters():
            p.copy_(torch.randn(p.shape, generator=g) * (scale if p.dim() > 1 else 0.3))
    return net, {k: v.detach().clone() for k, v in net.state_dict().items()}


def _twins(gl, system, n, seed, **kw):
    a = gl.BatchedEnv(system, n, seed=seed, **kw)
    b = gl.BatchedEnv(system, n, seed=seed, **kw)
    return a, b


def _clip_actions(pol, system, act):
    lo, hi = pol.action_bounds(system)
    return torch.clamp(act, lo, hi)


@pytest.mark.parametrize("precision", ["bf16", "fp32"])
@pytest.mark.parametrize("system,n,K,kw", [
    ("pmsm", 1000, 24, dict(add_noise=True, max_episode_steps=7)),
    ("lorenz3", 2051, 12, dict(max_episode_steps=5)),
    ("hr", 640, 10, dict(add_noise=True, add_filter=True)),
    ("lorenz4", 333, 9, dict(max_episode_steps=4)),
    ("transient2", 640, 8, dict(max_episode_steps=5)),
    ("transient_pmsm", 500, 8, dict(max_episode_steps=3)),
    ("singlecontrol", 300, 6, dict(max_episode_steps=4)),
])
def test_policy_rollout_env_part_bitexact(gl, pol, system, n, K, kw, precision):
    envp, envr = _twins(gl, system, n, seed=11, **kw)
    O, A = envp.obs_dim, envp.action_dim
    _, sd = _random_policy(pol, O, A, seed=3)
    col = _col(pol, envp, sd, bootstrap=False, capture_terminal=K * n, precision=precision)
    obs0 = _np(col.reset())
    obs0r = _np(envr.reset())
    assert np.array_equal(obs0, obs0r)
    b = col.collect(K)
    acts = _clip_actions(pol, system, b.actions).contiguous()
    obs_r, rew_r, done_r, (didx, tobs, nd) = envr.rollout(acts, capture_terminal=K * n)
    assert np.array_equal(_np(b.observations[0]), obs0)  # no normalisation: raw obs
    assert np.array_equal(_np(b.observations[1:]), _np(obs_r[:-1]))
    assert np.array_equal(_np(b.last_obs), _np(obs_r[-1]))
    assert np.array_equal(_np(b.rewards), _np(rew_r))
    assert np.array_equal(_np(b.dones), _np(done_r))
    m, mr = int(b.n_done.item()), int(nd.item())
    assert m == mr
    o1 = np.argsort(_np(b.done_idx[:m]))
    o2 = np.argsort(_np(didx[:mr]))
    assert np.array_equal(_np(b.done_idx[:m])[o1], _np(didx[:mr])[o2])
    assert np.array_equal(_np(b.terminal_obs[:m])[o1], _np(tobs[:mr])[o2])
    if kw.get("max_episode_steps"):
        assert m > 0
    # state planes agree after the rollout too
    for p in range(3):
        assert np.array_equal(_np(envp.get_state(p)), _np(envr.get_state(p)))
    # episode_starts = previous step's dones
    st = _np(b.episode_starts)
    assert np.all(st[0] == 1.0)
    assert np.array_equal(st[1:], (_np(b.dones[:-1]) != 0).astype(np.float32))


@pytest.mark.parametrize("system", ["pmsm", "lorenz3"])
def test_policy_forward_vs_torch(gl, pol, system):
    n, K = 4099, 6
    env = gl.BatchedEnv(system, n, seed=5, add_noise=(system == "pmsm"))
    O, A = env.obs_dim, env.action_dim
    net, sd = _random_policy(pol, O, A, seed=7)
    col = _col(pol, env, sd, bootstrap=False, deterministic=True)
    col.reset()
    b = col.collect(K)
    obs = b.observations.reshape(-1, O).cpu()
    finite = torch.isfinite(obs).all(1)
    mean_ref, val_ref = pol.reference_forward_bf16(sd, obs)
    act = b.actions.reshape(-1, A).cpu()
    val = b.values.reshape(-1).cpu()
    f = finite.numpy()
    err_a = (act - mean_ref).abs()[finite].max().item()
    err_v = (val - val_ref).abs()[finite].max().item()
    print("max |kernel - bf16 restatement|: mean %.3g value %.3g" % (err_a, err_v))
    np.testing.assert_allclose(_np(act)[f], _np(mean_ref)[f], atol=TOL_A, rtol=TOL_R)
    np.testing.assert_allclose(_np(val)[f], _np(val_ref)[f], atol=TOL_A, rtol=TOL_R)
    # bulk agreement is far tighter than the worst case
    assert np.median(np.abs(_np(val)[f] - _np(val_ref)[f])) < 2e-3
    # deterministic log_prob = sum_j Normal(mean, std).log_prob(mean)
    ls = sd["log_std"].float()
    lp0 = (-ls - 0.5 * np.log(2 * np.pi)).sum().item()
    np.testing.assert_allclose(_np(b.log_probs), lp0, rtol=1e-6, atol=1e-6)
    # last values = V(last obs)
    _, vl = pol.reference_forward_bf16(sd, b.last_obs.cpu())
    fl = torch.isfinite(b.last_obs.cpu()).all(1).numpy()
    np.testing.assert_allclose(_np(b.last_values)[fl], _np(vl)[fl], atol=TOL_A, rtol=TOL_R)


@pytest.mark.parametrize("system", ["pmsm", "hr"])
def test_policy_bf16_vs_fp32_sb3_init(gl, pol, system):
    """SB3-initialised policy (orthogonal, gains sqrt(2) / 0.01 / 1): the bf16-MFMA
    forward against the plain fp32 torch forward (what SB3 computes on the CPU)."""
    from gym_lorenz.vec_normalize import DeviceRunningMeanStd

    n, K = 8192, 4
    env = gl.BatchedEnv(system, n, seed=15)
    O, A = env.obs_dim, env.action_dim
    net = pol.ActorCriticMlp(O, A, seed=3)
    # as the reference trains PMSM: VecNormalize(norm_obs=True, clip_obs=10) in front
    rms = DeviceRunningMeanStd(O, env.device)
    col = _col(pol, env, net.state_dict(), bootstrap=False, deterministic=True,
                                    obs_rms=rms, training=True)
    col.reset()
    col.collect(K)  # statistics warm-up
    b = col.collect(K)
    obs = b.observations.reshape(-1, O).cpu()
    fin = torch.isfinite(obs).all(1)
    with torch.no_grad():
        mean32, val32 = net(obs[fin])
    dv = (b.values.reshape(-1).cpu()[fin] - val32).abs()
    dm = (b.actions.reshape(-1, A).cpu()[fin] - mean32).abs()
    scale_v = val32.abs().mean().item()
    scale_m = mean32.abs().mean().item()
    print("%s bf16 vs fp32: value max %.3g mean %.3g (|V| ~ %.3g); action mean max %.3g "
          "mean %.3g (|mu| ~ %.3g)" % (system, dv.max(), dv.mean(), scale_v, dm.max(), dm.mean(),
                                       scale_m))
    assert dv.mean().item() < 0.02 * max(scale_v, 1e-3) + 1e-3
    assert dm.mean().item() < 0.02 * max(scale_m, 1e-3) + 1e-4
    assert dv.max().item() < 0.1 * max(scale_v, 1.0)


def test_policy_sampling_and_log_prob(gl, pol):
    n, K = 32768, 4
    env = gl.BatchedEnv("pmsm", n, seed=9)
    _, sd = _random_policy(pol, 6, 2, seed=2)
    sd["log_std"] = torch.tensor([-0.5, 0.25])
    col = _col(pol, env, sd, bootstrap=False)
    col.reset()
    b = col.collect(K)
    obs = b.observations.reshape(-1, 6).cpu()
    mean_ref, _ = pol.reference_forward_bf16(sd, obs)
    act = b.actions.reshape(-1, 2).cpu()
    std = torch.exp(sd["log_std"])
    z = ((act - mean_ref) / std).numpy()
    assert abs(z.mean()) < 0.01 and abs(z.std() - 1.0) < 0.01
    assert abs(np.corrcoef(z[:, 0], z[:, 1])[0, 1]) < 0.01
    lp_ref = torch.distributions.Normal(mean_ref, std).log_prob(act).sum(-1)
    np.testing.assert_allclose(_np(b.log_probs).reshape(-1), lp_ref.numpy(), atol=5e-2, rtol=2e-2)
    # a different call counter gives different samples; the same seed reproduces them
    env2 = gl.BatchedEnv("pmsm", n, seed=9)
    col2 = _col(pol, env2, sd, bootstrap=False)
    col2.reset()
    b2 = col2.collect(K)
    assert torch.equal(b.actions, b2.actions)
    assert not torch.equal(b.actions[0], b.actions[1])


def test_policy_truncation_bootstrap(gl, pol):
    n, K, gamma = 2000, 13, 0.97
    ea, eb = _twins(gl, "pmsm", n, seed=21, max_episode_steps=5)
    _, sd = _random_policy(pol, 6, 2, seed=4)
    ca = _col(pol, ea, sd, gamma=gamma, bootstrap=True, capture_terminal=K * n)
    cb = _col(pol, eb, sd, gamma=gamma, bootstrap=False)
    ca.reset()
    cb.reset()
    ba, bb = ca.collect(K), cb.collect(K)
    assert torch.equal(ba.actions, bb.actions)
    d = _np(ba.dones)
    trunc = (d & 2 != 0) & (d & 1 == 0)
    assert trunc.sum() > 0
    diff = _np(ba.rewards) - _np(bb.rewards)
    assert np.all(diff[~trunc] == 0)
    m = int(ba.n_done.item())
    idx = _np(ba.done_idx[:m])
    tobs = ba.terminal_obs[:m].cpu()
    _, vt = pol.reference_forward_bf16(sd, tobs)
    k, e = idx // n, idx % n
    sel = trunc[k, e]
    got = (_np(ba.rewards)[k, e] - _np(bb.rewards)[k, e])[sel]
    want = (np.float32(gamma) * _np(vt))[sel]
    fin = np.isfinite(want)
    np.testing.assert_allclose(got[fin], want[fin], atol=TOL_A, rtol=TOL_R)


def test_policy_vecnormalize(gl, pol):
    from gym_lorenz.vec_normalize import DeviceRunningMeanStd

    n, K = 3000, 8
    envp, envr = _twins(gl, "pmsm", n, seed=31, add_noise=True)
    _, sd = _random_policy(pol, 6, 2, seed=6)
    rms = DeviceRunningMeanStd(6, envp.device)
    rng = np.random.default_rng(0)
    rms.set_state(rng.normal(0, 2, 6), rng.uniform(0.5, 30, 6), 1234.0)
    ref = DeviceRunningMeanStd(6, envp.device)
    ref.set_state(rms.mean, rms.var, rms.count)
    col = _col(pol, envp, sd, obs_rms=rms, clip_obs=3.0, bootstrap=False,
                                    training=True)
    obs0 = col.last_obs = envp.reset().clone()
    b = col.collect(K)
    envr.reset()
    obs_r, _, _ = envr.rollout(_clip_actions(pol, "pmsm", b.actions).contiguous())
    raw = torch.cat([obs0[None], obs_r[:-1]], 0)
    want = ref.normalize(raw.reshape(-1, 6), 1e-8, 3.0).reshape(K, n, 6)
    assert torch.equal(b.observations, want)
    assert (b.observations.abs() <= 3.0).all()
    mom = torch.zeros(13, dtype=torch.float64, device=envp.device)
    from gym_lorenz import _native as nat
    import ctypes
    nat.check(nat.lib.lz_rms_moments(ref._h, ctypes.c_void_p(obs_r.data_ptr()), nat.F32, K * n,
                                     ctypes.c_void_p(mom.data_ptr())))
    np.testing.assert_allclose(_np(b.obs_moments), _np(mom), rtol=1e-12)
    ref.update(obs_r.reshape(-1, 6))
    np.testing.assert_allclose(rms.mean, ref.mean, rtol=1e-12)
    np.testing.assert_allclose(rms.var, ref.var, rtol=1e-12)
    assert rms.count == ref.count


# (K, n): both load schedules of k_gae (double-buffered U=4 below 262,144 envs, single
# batches of U=8 from there) with K below one batch, exactly 2 and 3 batches, and ragged tails
@pytest.mark.parametrize("K,n", [(37, 5003), (3, 70), (8, 100), (12, 64), (9, 131075),
                                 (37, 131072), (5, 262147), (37, 262147)])
def test_gae_bitexact_vs_sb3_restatement(gl, pol, K, n):
    from oracle.sb3_buffer import compute_returns_and_advantage

    rng = np.random.default_rng(1)
    rew = rng.normal(0, 3, (K, n)).astype(np.float32)
    val = rng.normal(0, 3, (K, n)).astype(np.float32)
    done = (rng.random((K, n)) < 0.05).astype(np.uint8) * rng.integers(1, 4, (K, n)).astype(np.uint8)
    last = rng.normal(0, 3, n).astype(np.float32)
    starts = np.zeros((K, n), np.float32)
    starts[0] = 1.0
    starts[1:] = (done[:-1] != 0)
    env = gl.BatchedEnv("pmsm", 8)
    col = _col(pol, env, gamma=0.99, gae_lambda=0.95)
    dev = env.device
    b = pol.RolloutBatch(None, None, None, torch.from_numpy(val).to(dev),
                         torch.from_numpy(rew).to(dev), torch.from_numpy(done).to(dev), None,
                         torch.from_numpy(last).to(dev), None)
    adv, ret = col.compute_returns_and_advantage(b)
    adv_r, ret_r = compute_returns_and_advantage(rew, val, starts, last, done[-1] != 0, 0.99, 0.95)
    assert np.array_equal(_np(adv), adv_r)
    assert np.array_equal(_np(ret), ret_r)


def test_policy_rollout_large_batch(gl, pol):
    """262,144 envs (BASELINE cfg4 size), K=16 (the reference's A2C n_steps): env part
    bit-exact vs the action-driven rollout over the whole batch."""
    n, K = 262144, 16
    envp, envr = _twins(gl, "pmsm", n, seed=41, add_noise=True)
    _, sd = _random_policy(pol, 6, 2, seed=8, scale=0.2)
    col = _col(pol, envp, sd)
    col.reset()
    envr.reset()
    b = col.collect(K)
    obs_r, rew_r, done_r = envr.rollout(_clip_actions(pol, "pmsm", b.actions).contiguous())
    assert torch.equal(b.observations[1:], obs_r[:-1])
    assert torch.equal(b.dones, done_r)
    boot = ((b.dones & 2) != 0) & ((b.dones & 1) == 0)
    assert torch.equal(b.rewards[~boot], rew_r[~boot])
    assert torch.isfinite(b.values).all() and torch.isfinite(b.log_probs).all()


@pytest.mark.parametrize("n", [70000, 262144])
def test_policy_launch_shapes_agree_bitwise(gl, pol, n):
    """The three launch shapes (64-env waves / 32-env waves x 8 / 32-env waves x 4 with
    interleaved nets, lz_internal.h policy_shape) run the same per-env arithmetic: every
    output is bit-identical across them (only the moments' summation order differs)."""
    from gym_lorenz.vec_normalize import DeviceRunningMeanStd

    K = 5
    outs = []
    for var in (0, 32, 64):
        env = gl.BatchedEnv("pmsm", n, seed=77, add_noise=True, max_episode_steps=3, variant=var)
        _, sd = _random_policy(pol, 6, 2, seed=12, scale=0.2)
        rms = DeviceRunningMeanStd(6, env.device)
        rms.set_state(np.zeros(6), np.full(6, 40.0), 10.0)
        col = _col(pol, env, sd, obs_rms=rms, training=True)
        col.last_obs = env.reset().clone()
        b = col.collect(K)
        outs.append(b)
    for b in outs[1:]:
        for f in ("observations", "actions", "log_probs", "values", "rewards", "dones",
                  "last_values", "last_obs"):
            assert torch.equal(getattr(b, f), getattr(outs[0], f)), f
        np.testing.assert_allclose(_np(b.obs_moments), _np(outs[0].obs_moments), rtol=1e-12)


def test_policy_narrow_net_optuna_setting(gl, pol):
    """code/lorenz_pmsm/optimize.py:36-52: A2C MlpPolicy net_arch [64, 64] Tanh behind
    VecNormalize(norm_obs, clip_obs=10) on PMSM -- zero-padded into the 128-unit kernel."""
    from gym_lorenz.vec_normalize import DeviceRunningMeanStd

    n, K = 4099, 8
    env = gl.BatchedEnv("pmsm", n, seed=5)
    net = pol.ActorCriticMlp(6, 2, hidden=64, seed=1)
    g = torch.Generator().manual_seed(2)
    with torch.no_grad():
        for p in net.parameters():
            p.copy_(torch.randn(p.shape, generator=g) * (0.4 if p.dim() > 1 else 0.3))
    sd = {k: v.detach().clone() for k, v in net.state_dict().items()}
    rms = DeviceRunningMeanStd(6, env.device)
    col = _col(pol, env, sd, bootstrap=False, deterministic=True, obs_rms=rms)
    col.reset()
    col.collect(K)
    b = col.collect(K)
    obs = b.observations.reshape(-1, 6).cpu()
    mean_ref, val_ref = pol.reference_forward_bf16(sd, obs)
    np.testing.assert_allclose(_np(b.actions).reshape(-1, 2), _np(mean_ref), atol=TOL_A, rtol=TOL_R)
    np.testing.assert_allclose(_np(b.values).reshape(-1), _np(val_ref), atol=TOL_A, rtol=TOL_R)
    assert np.median(np.abs(_np(b.values).reshape(-1) - _np(val_ref))) < 2e-3


def test_collect_from_a_side_stream(gl, pol):
    """collect() + GAE called under a current stream other than the env handle's: the
    follow-up kernels (episode starts, GAE, obs_rms update) see the rollout's outputs
     -- results equal a same-stream collect bit for bit."""
    n, K = 20000, 16
    _, sd = _random_policy(pol, 6, 2, seed=3, scale=0.2)
    out = []
    for side in (False, True):
        env = gl.BatchedEnv("pmsm", n, seed=12, add_noise=True)
        col = _col(pol, env, sd)
        col.reset()
        torch.cuda.synchronize()
        s = torch.cuda.Stream(device=env.device) if side else torch.cuda.current_stream(env.device)
        with torch.cuda.stream(s):
            b = col.collect(K)
            adv, ret = col.compute_returns_and_advantage(b)
            res = [t.clone() for t in (b.rewards, b.dones, b.episode_starts, adv, ret)]
        s.synchronize()
        out.append([_np(t) for t in res])
    for x, y in zip(*out):
        assert np.array_equal(x, y)
