"""GPU parity of the attention actor-critics at the reference's precision (float32:
lz_rollout_policy_attn_f32 / lz_rollout_policy_attn_stack_f32, the default of
FusedRolloutCollector for code/train.py:52-112's and code/lorenz_filter/train.py:54-132's
policies).

Bars, all bit for bit unless stated:
  * forward: every deterministic action (= the policy mean) and value the rollout
    recorded equals oracle.attn_f32 (lz_oracle.c orc_attn_f32, the CPU restatement of
    the kernel's operation order) of the input the kernel recorded for that step --
    raw HR obs (code/train.py), PMSM behind frozen VecNormalize statistics, the
    VecFrameStack(4) stack of the LayerNorm variant; last values likewise; at cfg5's
    per-GPU batch (HR 32,768 envs x K = 2,048) on sampled rows and on a ragged batch;
  * env part: vs lz_rollout fed the policy's own clipped actions (observations,
    rewards, dones, compact done list, final state); the LayerNorm variant's stacks vs
    the SB3 StackedObservations restatement (oracle/sb3_framestack.py);
  * truncation bootstrap: reward = env reward + float32(gamma * V(terminal input)),
    V from the oracle -- for the stacked variant V of SB3's stacked terminal
    observation;
  * sampling: z = (a - mean) / std ~ N(0, 1), log_prob the kernel's float32 formula;
  * against SB3's own arithmetic (torch float32 nn.MultiheadAttention / nn.LayerNorm,
    SB3-initialised policy): max |difference| <= 1e-5 of the output scale.
"""
import numpy as np
import pytest
import torch

from conftest import bits_equal

pytestmark = pytest.mark.gpu

AF_LOGSTD = 54400 + 2 * 102400  # lz_internal.h kAFLogStd


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
    kw.setdefault("precision", "fp32")
    return pol.FusedRolloutCollector(*args, **kw)


def _random_attn(pol, I, A, seed, ln=False, scale=0.3):
    net = pol.ActorCriticAttn(I, A, seed=seed, layer_norm=ln)
    g = torch.Generator().manual_seed(seed + 1)
    with torch.no_grad():
        for name, p in net.named_parameters():
            if "layer_norm" in name:
                p.copy_((1.0 if name.endswith("weight") else 0.0)
                        + 0.2 * torch.randn(p.shape, generator=g))
            else:
                p.copy_(torch.randn(p.shape, generator=g) * (scale if p.dim() > 1 else 0.3))
    return {k: v.detach().clone() for k, v in net.state_dict().items()}


def _check_forward(orc, sd, b, I, A, rows=None):
    obs = _np(b.observations).reshape(-1, I)
    act = _np(b.actions).reshape(-1, A)
    val = _np(b.values).reshape(-1)
    if rows is not None:
        obs, act, val = obs[rows], act[rows], val[rows]
    m, v = orc.attn_f32(sd, obs)
    assert bits_equal(act, m), np.nanmax(np.abs(act - m))
    assert bits_equal(val, v), np.nanmax(np.abs(val - v))


@pytest.mark.parametrize("system,n,K,kw", [
    ("hr", 1000, 12, dict(add_noise=True, add_filter=True, max_episode_steps=5)),
    ("pmsm", 777, 10, dict(add_noise=True, max_episode_steps=4)),
    ("lorenz3", 40000, 3, dict(max_episode_steps=2)),  # 2,500 tiles: grid-stride rounds
    ("hr", 5, 6, dict(max_episode_steps=2)),            # a single partial 16-env tile
])
def test_attn_f32_env_part_and_forward_bitexact(gl, pol, orc, system, n, K, kw):
    envp = gl.BatchedEnv(system, n, seed=11, **kw)
    envr = gl.BatchedEnv(system, n, seed=11, **kw)
    O, A = envp.obs_dim, envp.action_dim
    sd = _random_attn(pol, O, A, seed=3, scale=0.2)
    col = _col(pol, envp, sd, bootstrap=False, deterministic=True, capture_terminal=K * n)
    assert col.attention and col.f32
    obs0 = _np(col.reset())
    assert np.array_equal(obs0, _np(envr.reset()))
    b = col.collect(K)
    lo, hi = pol.action_bounds(envp.system_name)
    acts = torch.clamp(b.actions, lo, hi).contiguous()
    obs_r, rew_r, done_r, (didx, tobs, nd) = envr.rollout(acts, capture_terminal=K * n)
    assert torch.equal(b.observations[1:], obs_r[:-1])
    assert torch.equal(b.last_obs, obs_r[-1])
    assert torch.equal(b.rewards, rew_r)
    assert torch.equal(b.dones, done_r)
    m, mr = int(b.n_done.item()), int(nd.item())
    assert m == mr and m > 0
    o1, o2 = np.argsort(_np(b.done_idx[:m])), np.argsort(_np(didx[:mr]))
    assert np.array_equal(_np(b.done_idx[:m])[o1], _np(didx[:mr])[o2])
    assert np.array_equal(_np(b.terminal_obs[:m])[o1], _np(tobs[:mr])[o2])
    for p in range(3):
        assert torch.equal(envp.get_state(p), envr.get_state(p))
    rows = None if n * K <= 20000 else np.random.default_rng(0).choice(n * K, 3000, replace=False)
    _check_forward(orc, sd, b, O, A, rows)
    _, vl = orc.attn_f32(sd, _np(b.last_obs))
    assert bits_equal(_np(b.last_values), vl)


def test_attn_f32_vecnormalize_frozen_bitexact(gl, pol, orc):
    """PMSM behind frozen VecNormalize statistics (the pooled statistics path)."""
    from gym_lorenz.vec_normalize import DeviceRunningMeanStd

    n, K = 3001, 4
    env = gl.BatchedEnv("pmsm", n, seed=5, add_noise=True)
    sd = _random_attn(pol, 6, 2, seed=7, scale=0.2)
    rms = DeviceRunningMeanStd(6, env.device)
    rng = np.random.default_rng(1)
    rms.set_state(rng.normal(0, 2, 6), rng.uniform(0.5, 30, 6), 1e4)
    col = _col(pol, env, sd, bootstrap=False, deterministic=True, obs_rms=rms, training=False)
    col.reset()
    b = col.collect(K)
    _check_forward(orc, sd, b, 6, 2)
    x_last = np.clip((_np(b.last_obs).astype(np.float64) - rms.mean) / np.sqrt(rms.var + 1e-8),
                     -10.0, 10.0).astype(np.float32)
    _, vl = orc.attn_f32(sd, x_last)
    assert bits_equal(_np(b.last_values), vl)


def test_attn_f32_bootstrap_and_sampling(gl, pol, orc):
    n, K, gamma = 2000, 11, 0.97
    ea = gl.BatchedEnv("hr", n, seed=21, max_episode_steps=4)
    eb = gl.BatchedEnv("hr", n, seed=21, max_episode_steps=4)
    sd = _random_attn(pol, 6, 2, seed=4)
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
    ra, rb = _np(ba.rewards), _np(bb.rewards)
    assert np.array_equal(ra[~trunc], rb[~trunc])
    m = int(ba.n_done.item())
    idx = _np(ba.done_idx[:m])
    k, e = idx // n, idx % n
    sel = trunc[k, e]
    _, vt = orc.attn_f32(sd, _np(ba.terminal_obs[:m]))
    want = (rb[k, e] + (np.float32(gamma) * vt).astype(np.float32)).astype(np.float32)
    assert bits_equal(ra[k, e][sel], want[sel])
    # sampling: z ~ N(0, 1) around the oracle mean; log_prob the kernel's formula
    obs = _np(ba.observations).reshape(-1, 6)
    mean, val = orc.attn_f32(sd, obs)
    assert bits_equal(_np(ba.values).reshape(-1), val)
    act = _np(ba.actions).reshape(-1, 2)
    f = np.frombuffer(_np(ca.blob).tobytes(), np.float32)[AF_LOGSTD // 4: AF_LOGSTD // 4 + 16]
    scale, var2, lscale = f[4:8], f[8:12], f[12:16]
    z = (act - mean) / scale[:2]
    assert abs(z.mean()) < 0.03 and abs(z.std() - 1.0) < 0.03
    dd = (act - mean).astype(np.float32)
    lp = None
    for j in range(2):
        lpj = ((-(dd[:, j] * dd[:, j])) / var2[j] - lscale[j]) - np.float32(0.91893853320467274)
        lp = lpj if lp is None else (lp + lpj).astype(np.float32)
    assert np.array_equal(_np(ba.log_probs).reshape(-1), lp)


def test_attn_f32_cfg5_batch(gl, pol, orc):
    """cfg5's per-GPU batch: HR 32,768 envs x K = 2,048 (code/train.py's PPO n_steps),
    forward bit-exact on 4,000 sampled rows, env part bit-exact against lz_rollout."""
    n, K = 32768, 2048
    envp = gl.BatchedEnv("hr", n, seed=2)
    envr = gl.BatchedEnv("hr", n, seed=2)
    sd = _random_attn(pol, 6, 2, seed=9, scale=0.2)
    col = _col(pol, envp, sd, bootstrap=True, deterministic=True)
    col.reset()
    envr.reset()
    b = col.collect(K)
    lo, hi = pol.action_bounds("hr")
    obs_r, rew_r, done_r = envr.rollout(torch.clamp(b.actions, lo, hi).contiguous())
    assert torch.equal(b.observations[1:], obs_r[:-1])
    assert torch.equal(b.dones, done_r)
    assert torch.equal(b.last_obs, obs_r[-1])
    rows = np.random.default_rng(3).choice(n * K, 4000, replace=False)
    _check_forward(orc, sd, b, 6, 2, rows)


# --------------------------- code/lorenz_filter/train.py: LayerNorm extractor on VecFrameStack(4)
def _sb3_stacks(obs0, obs_r, done_r, didx, tobs, n, n_stack):
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
    ("pmsm", 3, 5, dict(max_episode_steps=2)),
    ("hr", 33000, 3, dict(max_episode_steps=2)),
])
def test_attn_ln_f32_framestack_bitexact(gl, pol, orc, system, n, K, kw):
    envp = gl.BatchedEnv(system, n, seed=11, **kw)
    envr = gl.BatchedEnv(system, n, seed=11, **kw)
    O, A = envp.obs_dim, envp.action_dim
    sd = _random_attn(pol, 4 * O, A, seed=3, ln=True, scale=0.2)
    col = _col(pol, envp, sd, bootstrap=False, deterministic=True, capture_terminal=K * n,
               frame_stack=4)
    assert col.attention_ln and col.f32
    obs0 = _np(col.reset())
    assert np.array_equal(obs0, _np(envr.reset()))
    b = col.collect(K)
    lo, hi = pol.action_bounds(envp.system_name)
    acts = torch.clamp(b.actions, lo, hi).contiguous()
    obs_r, rew_r, done_r, (didx, tobs, nd) = envr.rollout(acts, capture_terminal=K * n)
    assert torch.equal(b.rewards, rew_r)
    assert torch.equal(b.dones, done_r)
    assert torch.equal(b.last_obs, obs_r[-1])
    m = int(nd.item())
    assert m > 0 and int(b.n_done.item()) == m
    seen, _, final = _sb3_stacks(obs0, _np(obs_r), _np(done_r), _np(didx[:m]), _np(tobs[:m]), n, 4)
    assert b.observations.shape == (K, n, 4 * O)
    assert np.array_equal(_np(b.observations), seen)
    assert np.array_equal(_np(b.last_stack), final)
    rows = None if n * K <= 20000 else np.random.default_rng(0).choice(n * K, 3000, replace=False)
    _check_forward(orc, sd, b, 4 * O, A, rows)
    _, vl = orc.attn_f32(sd, final)
    assert bits_equal(_np(b.last_values), vl)


def test_attn_ln_f32_bootstrap_bitexact(gl, pol, orc):
    """The truncation bootstrap values SB3's stacked terminal observation."""
    n, K, gamma = 1500, 9, 0.97
    ea = gl.BatchedEnv("hr", n, seed=21, max_episode_steps=4, add_filter=True)
    eb = gl.BatchedEnv("hr", n, seed=21, max_episode_steps=4, add_filter=True)
    sd = _random_attn(pol, 24, 2, seed=4, ln=True)
    ca = _col(pol, ea, sd, gamma=gamma, bootstrap=True, deterministic=True,
              capture_terminal=K * n, frame_stack=4)
    cb = _col(pol, eb, sd, gamma=gamma, bootstrap=False, deterministic=True, frame_stack=4)
    obs0 = _np(ca.reset())
    cb.reset()
    ba, bb = ca.collect(K), cb.collect(K)
    assert torch.equal(ba.actions, bb.actions)
    d = _np(ba.dones)
    trunc = (d & 2 != 0) & (d & 1 == 0)
    assert trunc.sum() > 0
    ra, rb = _np(ba.rewards), _np(bb.rewards)
    assert np.array_equal(ra[~trunc], rb[~trunc])
    m = int(ba.n_done.item())
    raw = np.concatenate([_np(ba.observations)[1:, :, -6:], _np(ba.last_obs)[None]], 0)
    _, sterm, _ = _sb3_stacks(obs0, raw, d, _np(ba.done_idx[:m]), _np(ba.terminal_obs[:m]), n, 4)
    keys = [(k, e) for (k, e) in sterm if trunc[k, e]]
    _, vt = orc.attn_f32(sd, np.stack([sterm[key] for key in keys]))
    want = np.array([rb[k, e] for (k, e) in keys], np.float32) + (np.float32(gamma) * vt).astype(np.float32)
    got = np.array([ra[k, e] for (k, e) in keys], np.float32)
    assert bits_equal(got, want.astype(np.float32))


def test_attn_ln_f32_cfg5_batch(gl, pol, orc):
    """code/lorenz_filter/train.py's shape at cfg5's per-GPU batch: HR(add_filter) on
    VecFrameStack(4), 32,768 envs x K = 2,048, sampled rows bit-exact."""
    n, K = 32768, 2048
    envp = gl.BatchedEnv("hr", n, seed=4, add_filter=True)
    envr = gl.BatchedEnv("hr", n, seed=4, add_filter=True)
    sd = _random_attn(pol, 24, 2, seed=9, ln=True, scale=0.2)
    col = _col(pol, envp, sd, bootstrap=True, deterministic=True, frame_stack=4)
    col.reset()
    envr.reset()
    b = col.collect(K)
    lo, hi = pol.action_bounds("hr")
    obs_r, rew_r, done_r = envr.rollout(torch.clamp(b.actions, lo, hi).contiguous())
    assert torch.equal(b.observations[1:, :, -6:], obs_r[:-1])
    assert torch.equal(b.dones, done_r)
    rows = np.random.default_rng(3).choice(n * K, 4000, replace=False)
    _check_forward(orc, sd, b, 24, 2, rows)


@pytest.mark.parametrize("ln", [False, True])
def test_attn_f32_vs_sb3_torch_fp32(gl, pol, ln):
    """SB3-initialised policies on the obs the kernel saw, against the plain torch float32
    modules (what SB3 computes): max |difference| <= 1e-5 of the output scale."""
    n, K = 8192, 4
    env = gl.BatchedEnv("hr", n, seed=15, add_filter=ln)
    I = 24 if ln else 6
    net = pol.ActorCriticAttn(I, 2, seed=3, layer_norm=ln)
    col = _col(pol, env, net.state_dict(), bootstrap=False, deterministic=True,
               frame_stack=4 if ln else 1)
    col.reset()
    b = col.collect(K)
    obs = b.observations.reshape(-1, I).cpu()
    with torch.no_grad():
        mean32, val32 = net(obs)
    dv = (b.values.reshape(-1).cpu() - val32).abs().max().item()
    dm = (b.actions.reshape(-1, 2).cpu() - mean32).abs().max().item()
    sv, sm = val32.abs().max().item(), mean32.abs().max().item()
    print("attn%s f32 kernel vs torch fp32: value max %.3g (|V| <= %.3g), mean max %.3g "
          "(|mu| <= %.3g)" % ("-LN" if ln else "", dv, sv, dm, sm))
    assert dv <= 1e-5 * max(sv, 1.0)
    assert dm <= 1e-5 * max(sm, 1.0)


@pytest.mark.parametrize("tag", ["plain", "ln"])
def test_attn_f32_reference_class_weights_bitexact(gl, pol, orc, tag):
    """The weights of tests/golden/attn_ref.npz -- a policy built from the reference's own
    AttentionFeaturesExtractor classes (code/train.py:52-94, code/lorenz_filter/
    train.py:55-103; tests/golden/make_attn_ref.py), whose outputs the oracle reproduces
    within 2e-6 (tests/test_attn_f32_host.py) -- drive the float32 kernels on HR (plain:
    raw obs; ln: VecFrameStack(4)): every recorded action and value equals
    oracle.attn_f32 of the recorded input bit for bit (deterministic actions), and so do
    the last values."""
    from conftest import golden

    g = golden("attn_ref")
    pre = tag + "/"
    sd = {k[len(pre):]: torch.from_numpy(v) for k, v in g.items()
          if k.startswith(pre) and k[len(pre):] not in ("x", "features", "mean", "value")}
    n, K, stack = 2000, 24, 4 if tag == "ln" else 1
    env = gl.BatchedEnv("hr", n, seed=19, add_noise=True, max_episode_steps=9)
    col = _col(pol, env, sd, bootstrap=False, deterministic=True, frame_stack=stack)
    assert col.f32 and (col.attention_ln if tag == "ln" else col.attention)
    col.reset()
    b = col.collect(K)
    _check_forward(orc, sd, b, 6 * stack, 2)
    last = col.last_stack if tag == "ln" else b.last_obs
    _, vl = orc.attn_f32(sd, _np(last))
    assert bits_equal(_np(b.last_values), vl)
    env.close()
