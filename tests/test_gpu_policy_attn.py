"""GPU parity of the bf16 opt-in (precision="bf16") of the fused rollout with
code/train.py's attention actor-critic (lz_rollout_policy_attn: AttentionFeaturesExtractor
shared by pi/vf, code/train.py:52-112); the float32 default is test_gpu_policy_attn_f32.py.

Bars (as test_gpu_policy.py):
  * env part: bit-exact vs the action-driven lz_rollout fed with the policy's own
    clipped actions (observations, rewards, dones, terminal observations, state);
  * forward: deterministic actions and values vs the torch restatement with the same
    bf16 roundings (policy.reference_forward_attn_bf16) within atol 3e-2 + rtol 3e-2
    (a bf16 rounding boundary crossed under a different fp32 summation order propagates
    through three more bf16 layers than in the MlpPolicy); the median is far tighter;
  * an SB3-initialised policy vs the plain fp32 module (nn.MultiheadAttention): mean
    abs error < 2% of the output scale;
  * truncation bootstrap and log-probs against the restatement.
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

TOL_A, TOL_R = 3e-2, 3e-2


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


def _col(pol, *args, **kw):
    """The bf16 kernels (this file's restatements are bf16)."""
    kw.setdefault("precision", "bf16")
    return pol.FusedRolloutCollector(*args, **kw)


def _random_attn(pol, O, A, seed, scale=0.3):
    net = pol.ActorCriticAttn(O, A, seed=seed)
    g = torch.Generator().manual_seed(seed + 1)
    with torch.no_grad():
        for p in net.parameters():
            p.copy_(torch.randn(p.shape, generator=g) * (scale if p.dim() > 1 else 0.3))
    return net, {k: v.detach().clone() for k, v in net.state_dict().items()}


@pytest.mark.parametrize("system,n,K,kw", [
    ("hr", 1000, 12, dict(add_noise=True, add_filter=True, max_episode_steps=5)),
    ("pmsm", 777, 10, dict(add_noise=True, max_episode_steps=4)),
    ("lorenz3", 40000, 3, dict(max_episode_steps=2)),  # grid-stride: 313 groups > 256 CUs
    ("hr", 5, 6, dict(max_episode_steps=2)),            # a single partial 32-env tile
])
def test_attn_rollout_env_part_bitexact(gl, pol, system, n, K, kw):
    envp = gl.BatchedEnv(system, n, seed=11, **kw)
    envr = gl.BatchedEnv(system, n, seed=11, **kw)
    O, A = envp.obs_dim, envp.action_dim
    _, sd = _random_attn(pol, O, A, seed=3)
    col = _col(pol, envp, sd, bootstrap=False, capture_terminal=K * n)
    assert col.attention
    obs0 = _np(col.reset())
    assert np.array_equal(obs0, _np(envr.reset()))
    b = col.collect(K)
    lo, hi = pol.action_bounds(envp.system_name)
    acts = torch.clamp(b.actions, lo, hi).contiguous()
    obs_r, rew_r, done_r, (didx, tobs, nd) = envr.rollout(acts, capture_terminal=K * n)
    assert np.array_equal(_np(b.observations[1:]), _np(obs_r[:-1]))
    assert np.array_equal(_np(b.last_obs), _np(obs_r[-1]))
    assert np.array_equal(_np(b.rewards), _np(rew_r))
    assert np.array_equal(_np(b.dones), _np(done_r))
    m, mr = int(b.n_done.item()), int(nd.item())
    assert m == mr and m > 0
    o1, o2 = np.argsort(_np(b.done_idx[:m])), np.argsort(_np(didx[:mr]))
    assert np.array_equal(_np(b.done_idx[:m])[o1], _np(didx[:mr])[o2])
    assert np.array_equal(_np(b.terminal_obs[:m])[o1], _np(tobs[:mr])[o2])
    for p in range(3):
        assert np.array_equal(_np(envp.get_state(p)), _np(envr.get_state(p)))
    assert torch.isfinite(b.values).all() and torch.isfinite(b.actions).all()


@pytest.mark.parametrize("system", ["hr", "pmsm"])
def test_attn_forward_vs_torch(gl, pol, system):
    """HR as code/train.py runs it (raw obs, |obs| ~ 1); PMSM behind VecNormalize
    (clip_obs=10) as the reference's PMSM learners run it.  (Raw PMSM obs of |o| ~ 60
    under random weights drive the attention softmax to a hard argmax whose near-ties
    a one-ulp bf16 difference flips: not a meaningful comparison.)"""
    from gym_lorenz.vec_normalize import DeviceRunningMeanStd

    n, K = 4099, 5
    env = gl.BatchedEnv(system, n, seed=5, add_noise=True)
    O, A = env.obs_dim, env.action_dim
    _, sd = _random_attn(pol, O, A, seed=7)
    rms = DeviceRunningMeanStd(O, env.device) if system == "pmsm" else None
    col = _col(pol, env, sd, bootstrap=False, deterministic=True, obs_rms=rms)
    col.reset()
    if rms is not None:
        col.collect(K)  # statistics warm-up, then frozen: last_values use the same stats
        col.training = False
    b = col.collect(K)
    obs = b.observations.reshape(-1, O).cpu()
    fin = torch.isfinite(obs).all(1)
    mean_ref, val_ref = pol.reference_forward_attn_bf16(sd, obs)
    act = b.actions.reshape(-1, A).cpu()
    val = b.values.reshape(-1).cpu()
    f = fin.numpy()
    ea = (act - mean_ref).abs()[fin]
    ev = (val - val_ref).abs()[fin]
    print("max |kernel - bf16 restatement|: mean %.3g value %.3g (median %.3g / %.3g)"
          % (ea.max(), ev.max(), ea.median(), ev.median()))
    np.testing.assert_allclose(_np(act)[f], _np(mean_ref)[f], atol=TOL_A, rtol=TOL_R)
    np.testing.assert_allclose(_np(val)[f], _np(val_ref)[f], atol=TOL_A, rtol=TOL_R)
    assert ev.median().item() < 2e-3 and ea.median().item() < 2e-3
    ls = sd["log_std"].float()
    lp0 = (-ls - 0.5 * np.log(2 * np.pi)).sum().item()
    np.testing.assert_allclose(_np(b.log_probs), lp0, rtol=1e-6, atol=1e-6)
    last = b.last_obs if rms is None else rms.normalize(b.last_obs, 1e-8, 10.0)
    _, vl = pol.reference_forward_attn_bf16(sd, last.float().cpu())
    fl = torch.isfinite(last.cpu()).all(1).numpy()
    np.testing.assert_allclose(_np(b.last_values)[fl], _np(vl)[fl], atol=TOL_A, rtol=TOL_R)


def test_attn_bf16_vs_fp32_sb3_init(gl, pol):
    """code/train.py's setting: HR (lorenz_try-v0), SB3-initialised attention policy;
    the fused bf16 forward against the fp32 nn.MultiheadAttention module."""
    n, K = 8192, 4
    env = gl.BatchedEnv("hr", n, seed=15)
    O, A = env.obs_dim, env.action_dim
    net = pol.ActorCriticAttn(O, A, seed=3)
    col = _col(pol, env, net.state_dict(), bootstrap=False, deterministic=True)
    col.reset()
    b = col.collect(K)
    obs = b.observations.reshape(-1, O).cpu()
    fin = torch.isfinite(obs).all(1)
    with torch.no_grad():
        mean32, val32 = net(obs[fin])
    dv = (b.values.reshape(-1).cpu()[fin] - val32).abs()
    dm = (b.actions.reshape(-1, A).cpu()[fin] - mean32).abs()
    sv, sm = val32.abs().mean().item(), mean32.abs().mean().item()
    print("attn bf16 vs fp32: value max %.3g mean %.3g (|V| ~ %.3g); action max %.3g mean %.3g "
          "(|mu| ~ %.3g)" % (dv.max(), dv.mean(), sv, dm.max(), dm.mean(), sm))
    assert dv.mean().item() < 0.02 * max(sv, 1e-3) + 1e-3
    assert dm.mean().item() < 0.02 * max(sm, 1e-3) + 1e-4
    assert dv.max().item() < 0.1 * max(sv, 1.0)


def test_attn_bootstrap_and_log_prob(gl, pol):
    n, K, gamma = 2000, 11, 0.97
    ea = gl.BatchedEnv("hr", n, seed=21, max_episode_steps=4)
    eb = gl.BatchedEnv("hr", n, seed=21, max_episode_steps=4)
    _, sd = _random_attn(pol, 6, 2, seed=4)
    sd["log_std"] = torch.tensor([-0.5, 0.25])
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
    _, vt = pol.reference_forward_attn_bf16(sd, ba.terminal_obs[:m].cpu())
    k, e = idx // n, idx % n
    sel = trunc[k, e]
    got = (_np(ba.rewards)[k, e] - _np(bb.rewards)[k, e])[sel]
    want = (np.float32(gamma) * _np(vt))[sel]
    fin = np.isfinite(want)
    np.testing.assert_allclose(got[fin], want[fin], atol=TOL_A, rtol=TOL_R)
    # log pi(a|s) of the sampled actions under the restated Gaussian
    obs = ba.observations.reshape(-1, 6).cpu()
    mean_ref, _ = pol.reference_forward_attn_bf16(sd, obs)
    act = ba.actions.reshape(-1, 2).cpu()
    lp_ref = torch.distributions.Normal(mean_ref, torch.exp(sd["log_std"])).log_prob(act).sum(-1)
    np.testing.assert_allclose(_np(ba.log_probs).reshape(-1), lp_ref.numpy(), atol=8e-2, rtol=3e-2)


# --------------------------- code/lorenz_filter/train.py: LayerNorm extractor on VecFrameStack(4)
def _random_attn_ln(pol, I, A, seed, scale=0.3):
    net = pol.ActorCriticAttn(I, A, seed=seed, layer_norm=True)
    g = torch.Generator().manual_seed(seed + 1)
    with torch.no_grad():
        for name, p in net.named_parameters():
            if "layer_norm" in name:
                p.copy_((1.0 if name.endswith("weight") else 0.0)
                        + 0.2 * torch.randn(p.shape, generator=g))
            else:
                p.copy_(torch.randn(p.shape, generator=g) * (scale if p.dim() > 1 else 0.3))
    return net, {k: v.detach().clone() for k, v in net.state_dict().items()}


def _sb3_stacks(obs0, obs_r, done_r, didx, tobs, n, n_stack):
    """SB3 VecFrameStack over the replayed raw frames (oracle/sb3_framestack.py): the
    stacked obs the policy sees at every step, the stacked terminal observations
    {(k, env): stack} and the final stack."""
    from oracle.sb3_framestack import StackedObservations

    K, O = obs_r.shape[0], obs_r.shape[2]
    term = {int(i): tobs[m] for m, i in enumerate(didx)}
    so = StackedObservations(n, n_stack, O)
    seen = [so.reset(obs0).copy()]
    stacked_term = {}
    for k in range(K):
        d = done_r[k] != 0
        infos = [{"terminal_observation": term[k * n + e]} if d[e] else {} for e in range(n)]
        st, infos = so.update(obs_r[k], d, infos)
        for e in np.nonzero(d)[0]:
            stacked_term[(k, int(e))] = infos[e]["terminal_observation"]
        seen.append(st.copy())
    return np.stack(seen[:-1]), stacked_term, seen[-1]


@pytest.mark.parametrize("system,n,K,kw", [
    ("hr", 777, 11, dict(add_noise=True, add_filter=True, max_episode_steps=4)),
    ("lorenz3", 300, 7, dict(max_episode_steps=3)),
    ("pmsm", 3, 5, dict(max_episode_steps=2)),          # a single partial 32-env tile
    ("hr", 33000, 3, dict(max_episode_steps=2)),        # grid-stride: 258 groups > 256 CUs
])
def test_attn_ln_framestack_rollout_bitexact(gl, pol, system, n, K, kw):
    """code/lorenz_filter/train.py's collection: VecFrameStack(4) + the LayerNorm
    extractor.  Env part bit-exact vs lz_rollout replaying the policy's own actions;
    the stacked observations the policy saw, and the final stack, bit-exact vs the SB3
    StackedObservations restatement (incl. zeroed stacks after a done)."""
    envp = gl.BatchedEnv(system, n, seed=11, **kw)
    envr = gl.BatchedEnv(system, n, seed=11, **kw)
    O, A = envp.obs_dim, envp.action_dim
    _, sd = _random_attn_ln(pol, 4 * O, A, seed=3)
    col = _col(pol, envp, sd, bootstrap=False, capture_terminal=K * n,
                                    frame_stack=4)
    assert col.attention_ln
    obs0 = _np(col.reset())
    assert np.array_equal(obs0, _np(envr.reset()))
    b = col.collect(K)
    lo, hi = pol.action_bounds(envp.system_name)
    acts = torch.clamp(b.actions, lo, hi).contiguous()
    obs_r, rew_r, done_r, (didx, tobs, nd) = envr.rollout(acts, capture_terminal=K * n)
    assert np.array_equal(_np(b.rewards), _np(rew_r))
    assert np.array_equal(_np(b.dones), _np(done_r))
    assert np.array_equal(_np(b.last_obs), _np(obs_r[-1]))
    m = int(nd.item())
    assert m > 0 and int(b.n_done.item()) == m
    seen, _, final = _sb3_stacks(obs0, _np(obs_r), _np(done_r), _np(didx[:m]), _np(tobs[:m]), n, 4)
    assert b.observations.shape == (K, n, 4 * O)
    assert np.array_equal(_np(b.observations), seen)
    assert np.array_equal(_np(b.last_stack), final)
    assert torch.isfinite(b.values).all()


def test_attn_ln_forward_and_bootstrap(gl, pol):
    """Deterministic actions / values vs the torch restatement on the stacked obs; the
    truncation bootstrap values the STACKED terminal observation (SB3 VecFrameStack
    rewrites infos['terminal_observation'])."""
    n, K, gamma = 1500, 9, 0.97
    ea = gl.BatchedEnv("hr", n, seed=21, max_episode_steps=4, add_filter=True)
    eb = gl.BatchedEnv("hr", n, seed=21, max_episode_steps=4, add_filter=True)
    _, sd = _random_attn_ln(pol, 24, 2, seed=4)
    ca = _col(pol, ea, sd, gamma=gamma, bootstrap=True, deterministic=True,
                                   capture_terminal=K * n, frame_stack=4)
    cb = _col(pol, eb, sd, gamma=gamma, bootstrap=False, deterministic=True,
                                   frame_stack=4)
    obs0 = _np(ca.reset())
    cb.reset()
    ba, bb = ca.collect(K), cb.collect(K)
    assert torch.equal(ba.actions, bb.actions)
    obs = ba.observations.reshape(-1, 24).cpu()
    mean_ref, val_ref = pol.reference_forward_attn_ln_bf16(sd, obs)
    ea_ = (ba.actions.reshape(-1, 2).cpu() - mean_ref).abs()
    ev_ = (ba.values.reshape(-1).cpu() - val_ref).abs()
    print("LN max |kernel - restatement|: mean %.3g value %.3g (median %.3g / %.3g)"
          % (ea_.max(), ev_.max(), ea_.median(), ev_.median()))
    np.testing.assert_allclose(_np(ba.actions).reshape(-1, 2), _np(mean_ref), atol=TOL_A, rtol=TOL_R)
    np.testing.assert_allclose(_np(ba.values).reshape(-1), _np(val_ref), atol=TOL_A, rtol=TOL_R)
    assert ev_.median().item() < 2e-3 and ea_.median().item() < 2e-3
    _, vl = pol.reference_forward_attn_ln_bf16(sd, ba.last_stack.cpu())
    np.testing.assert_allclose(_np(ba.last_values), _np(vl), atol=TOL_A, rtol=TOL_R)
    # bootstrap on the stacked terminal observations
    d = _np(ba.dones)
    trunc = (d & 2 != 0) & (d & 1 == 0)
    assert trunc.sum() > 0
    diff = _np(ba.rewards) - _np(bb.rewards)
    assert np.all(diff[~trunc] == 0)
    m = int(ba.n_done.item())
    obs_r = ba.observations.cpu().numpy()[:, :, -6:]  # raw frames the policy saw
    raw = np.concatenate([obs_r[1:], _np(ba.last_obs)[None]], 0)  # frame after step k
    _, sterm, _ = _sb3_stacks(obs0, raw, d, _np(ba.done_idx[:m]), _np(ba.terminal_obs[:m]), n, 4)
    keys = [(k, e) for (k, e) in sterm if trunc[k, e]]
    st = np.stack([sterm[key] for key in keys])
    _, vt = pol.reference_forward_attn_ln_bf16(sd, st)
    got = np.array([diff[k, e] for (k, e) in keys])
    np.testing.assert_allclose(got, np.float32(gamma) * _np(vt), atol=TOL_A, rtol=TOL_R)


def test_attn_ln_sb3_init_vs_fp32(gl, pol):
    n, K = 8192, 4
    env = gl.BatchedEnv("hr", n, seed=15, add_filter=True)
    net = pol.ActorCriticAttn(24, 2, seed=3, layer_norm=True)
    col = _col(pol, env, net.state_dict(), bootstrap=False, deterministic=True,
                                    frame_stack=4)
    col.reset()
    b = col.collect(K)
    obs = b.observations.reshape(-1, 24).cpu()
    with torch.no_grad():
        mean32, val32 = net(obs)
    dv = (b.values.reshape(-1).cpu() - val32).abs()
    dm = (b.actions.reshape(-1, 2).cpu() - mean32).abs()
    sv, sm = val32.abs().mean().item(), mean32.abs().mean().item()
    print("attn-LN bf16 vs fp32: value max %.3g mean %.3g (|V| ~ %.3g); action max %.3g mean "
          "%.3g (|mu| ~ %.3g)" % (dv.max(), dv.mean(), sv, dm.max(), dm.mean(), sm))
    assert dv.mean().item() < 0.02 * max(sv, 1e-3) + 1e-3
    assert dm.mean().item() < 0.02 * max(sm, 1e-3) + 1e-4
    assert dv.max().item() < 0.1 * max(sv, 1.0)
