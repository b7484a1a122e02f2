"""GPU parity of the opt-in "i8x4" attention actor-critics:
lz_rollout_policy_attn_f32 / _attn_stack_f32 with LZ_POLICY_I8X4 and an
lz_attn*_policy_pack_i8x4 blob -- the pi / vf nets' two wide layers as exact 4-digit int8
fixed-point products on v_mfma_i32_16x16x64_i8 (lz_policy.hip attn16_net_i8).

Bars:
  * forward bit for bit: every deterministic action (= the mean) and value the rollout
    recorded equals oracle.attn_f32(precision="i8x4") (lz_oracle.c orc_attn_i8x4) of the
    input the kernel recorded -- raw HR obs, frozen-VecNormalize PMSM, the LayerNorm
    variant's VecFrameStack(4) stacks, cfg5's 32,768 x 2,048 batch on sampled rows, the
    reference-class weights of tests/golden/attn_ref.npz; last values likewise;
  * env part: vs lz_rollout fed the policy's own clipped actions;
  * accuracy: within 1e-5 of torch float32 (SB3's own arithmetic), as the float32 path;
  * a NaN input poisons exactly its env (NaN action mean and value);
  * the flag is refused by the other policy kernels.
"""
import numpy as np
import pytest
import torch

from conftest import bits_equal

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
    m, v = orc.attn_f32(sd, obs, precision="i8x4")
    assert bits_equal(act, m), np.nanmax(np.abs(act - m))
    assert bits_equal(val, v), np.nanmax(np.abs(val - v))


@pytest.mark.parametrize("system,n,K,kw", [
    ("hr", 1000, 12, dict(add_noise=True, add_filter=True, max_episode_steps=5)),
    ("pmsm", 777, 10, dict(add_noise=True, max_episode_steps=4)),
    ("lorenz3", 40000, 3, dict(max_episode_steps=2)),  # grid-stride rounds
    ("hr", 5, 6, dict(max_episode_steps=2)),            # a single partial 16-env tile
])
def test_i8x4_env_part_and_forward_bitexact(gl, pol, orc, system, n, K, kw):
    envp = gl.BatchedEnv(system, n, seed=11, **kw)
    envr = gl.BatchedEnv(system, n, seed=11, **kw)
    O, A = envp.obs_dim, envp.action_dim
    sd = _random_attn(pol, O, A, seed=3, scale=0.2)
    col = pol.FusedRolloutCollector(envp, sd, bootstrap=False, deterministic=True,
                                    capture_terminal=K * n, precision="i8x4")
    assert col.attention and col.i8x4
    col.reset()
    envr.reset()
    b = col.collect(K)
    lo, hi = pol.action_bounds(envp.system_name)
    acts = torch.clamp(b.actions, lo, hi).contiguous()
    obs_r, rew_r, done_r = envr.rollout(acts)
    assert torch.equal(b.observations[1:], obs_r[:-1])
    assert torch.equal(b.last_obs, obs_r[-1])
    assert torch.equal(b.rewards, rew_r) and torch.equal(b.dones, done_r)
    rows = None if n * K <= 20000 else np.random.default_rng(0).choice(n * K, 3000, replace=False)
    _check_forward(orc, sd, b, O, A, rows)
    _, vl = orc.attn_f32(sd, _np(b.last_obs), precision="i8x4")
    assert bits_equal(_np(b.last_values), vl)
    # not the float32 path's bits (a different arithmetic) but its accuracy: both against
    # the same net in float64 (LORENZ3's raw +-30 obs through 0.2-scale random weights make
    # float32 itself ~1e-5 off there)
    x = _np(b.observations).reshape(-1, O)[:2000]
    net = pol.ActorCriticAttn(O, A)
    net.load_state_dict(sd)
    with torch.no_grad():
        m64 = net.double()(torch.from_numpy(x).double())[0].numpy()
    m32, _ = orc.attn_f32(sd, x)
    sc = max(1.0, np.abs(m64).max())
    e8 = np.abs(_np(b.actions).reshape(-1, A)[:2000] - m64).max() / sc
    e32 = np.abs(m32 - m64).max() / sc
    print("i8x4 vs float64 %.2e, float32 vs float64 %.2e" % (e8, e32))
    assert not np.array_equal(_np(b.actions).reshape(-1, A)[:2000], m32)
    assert e8 <= 1.5 * e32 + 1e-6


def test_i8x4_vecnormalize_frozen_bitexact(gl, pol, orc):
    from gym_lorenz.vec_normalize import DeviceRunningMeanStd

    n, K = 3001, 4
    env = gl.BatchedEnv("pmsm", n, seed=5, add_noise=True)
    sd = _random_attn(pol, 6, 2, seed=7, scale=0.2)
    rms = DeviceRunningMeanStd(6, env.device)
    rng = np.random.default_rng(1)
    rms.set_state(rng.normal(0, 2, 6), rng.uniform(0.5, 30, 6), 1e4)
    col = pol.FusedRolloutCollector(env, sd, bootstrap=False, deterministic=True, obs_rms=rms,
                                    training=False, precision="i8x4")
    col.reset()
    b = col.collect(K)
    _check_forward(orc, sd, b, 6, 2)


def test_i8x4_bootstrap_bitexact(gl, pol, orc):
    n, K, gamma = 2000, 11, 0.97
    ea = gl.BatchedEnv("hr", n, seed=21, max_episode_steps=4)
    eb = gl.BatchedEnv("hr", n, seed=21, max_episode_steps=4)
    sd = _random_attn(pol, 6, 2, seed=4)
    ca = pol.FusedRolloutCollector(ea, sd, gamma=gamma, bootstrap=True, capture_terminal=K * n,
                                   precision="i8x4")
    cb = pol.FusedRolloutCollector(eb, sd, gamma=gamma, bootstrap=False, precision="i8x4")
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
    _, vt = orc.attn_f32(sd, _np(ba.terminal_obs[:m]), precision="i8x4")
    want = (rb[k, e] + (np.float32(gamma) * vt).astype(np.float32)).astype(np.float32)
    assert bits_equal(ra[k, e][sel], want[sel])
    _, val = orc.attn_f32(sd, _np(ba.observations).reshape(-1, 6), precision="i8x4")
    assert bits_equal(_np(ba.values).reshape(-1), val)


@pytest.mark.parametrize("ln", [False, True])
def test_i8x4_cfg5_batch(gl, pol, orc, ln):
    """cfg5's per-GPU batch: HR 32,768 envs x K = 2,048 (code/train.py's n_steps; the
    LayerNorm variant on VecFrameStack(4)), forward bit-exact on sampled rows, env part
    bit-exact against lz_rollout."""
    n, K = 32768, 2048
    envp = gl.BatchedEnv("hr", n, seed=2, add_filter=ln)
    envr = gl.BatchedEnv("hr", n, seed=2, add_filter=ln)
    I = 24 if ln else 6
    sd = _random_attn(pol, I, 2, seed=9, ln=ln, scale=0.2)
    col = pol.FusedRolloutCollector(envp, sd, bootstrap=True, deterministic=True,
                                    frame_stack=4 if ln else 1, precision="i8x4")
    col.reset()
    envr.reset()
    b = col.collect(K)
    lo, hi = pol.action_bounds("hr")
    obs_r, rew_r, done_r = envr.rollout(torch.clamp(b.actions, lo, hi).contiguous())
    assert torch.equal(b.dones, done_r)
    if ln:
        assert torch.equal(b.observations[1:, :, -6:], obs_r[:-1])
    else:
        assert torch.equal(b.observations[1:], obs_r[:-1])
    rows = np.random.default_rng(3).choice(n * K, 4000, replace=False)
    _check_forward(orc, sd, b, I, 2, rows)


@pytest.mark.parametrize("ln", [False, True])
def test_i8x4_vs_sb3_torch_fp32(gl, pol, ln):
    """SB3-initialised policies on the obs the kernel saw, against the plain torch float32
    modules: max |difference| <= 1e-5 of the output scale (the float32 path's bar)."""
    n, K = 8192, 4
    env = gl.BatchedEnv("hr", n, seed=15, add_filter=ln)
    I = 24 if ln else 6
    net = pol.ActorCriticAttn(I, 2, seed=3, layer_norm=ln)
    col = pol.FusedRolloutCollector(env, net.state_dict(), bootstrap=False, deterministic=True,
                                    frame_stack=4 if ln else 1, precision="i8x4")
    col.reset()
    b = col.collect(K)
    obs = b.observations.reshape(-1, I).cpu()
    with torch.no_grad():
        mean32, val32 = net(obs)
    dv = (b.values.reshape(-1).cpu() - val32).abs().max().item()
    dm = (b.actions.reshape(-1, 2).cpu() - mean32).abs().max().item()
    sv, sm = val32.abs().max().item(), mean32.abs().max().item()
    print("attn%s i8x4 kernel vs torch fp32: value max %.3g (|V| <= %.3g), mean max %.3g "
          "(|mu| <= %.3g)" % ("-LN" if ln else "", dv, sv, dm, sm))
    assert dv <= 1e-5 * max(sv, 1.0)
    assert dm <= 1e-5 * max(sm, 1.0)


@pytest.mark.parametrize("tag", ["plain", "ln"])
def test_i8x4_reference_class_weights_bitexact(gl, pol, orc, tag):
    """The reference-class weights of tests/golden/attn_ref.npz (the oracle is within 2e-6
    of those classes' outputs: tests/test_i8x4_host.py) drive the i8x4 kernels on HR."""
    from conftest import golden

    g = golden("attn_ref")
    pre = tag + "/"
    sd = {k[len(pre):]: torch.from_numpy(v) for k, v in g.items()
          if k.startswith(pre) and k[len(pre):] not in ("x", "features", "mean", "value")}
    n, K, stack = 2000, 24, 4 if tag == "ln" else 1
    env = gl.BatchedEnv("hr", n, seed=19, add_noise=True, max_episode_steps=9)
    col = pol.FusedRolloutCollector(env, sd, bootstrap=False, deterministic=True,
                                    frame_stack=stack, precision="i8x4")
    col.reset()
    b = col.collect(K)
    _check_forward(orc, sd, b, 6 * stack, 2)
    last = col.last_stack if tag == "ln" else b.last_obs
    _, vl = orc.attn_f32(sd, _np(last), precision="i8x4")
    assert bits_equal(_np(b.last_values), vl)
    env.close()


def test_i8x4_nan_input_poisons_its_env_only(gl, pol, orc):
    """A NaN observation (a diverged env) gives that env NaN outputs and leaves every other
    env's bits as the oracle's."""
    n = 64
    env = gl.BatchedEnv("hr", n, seed=3)
    sd = _random_attn(pol, 6, 2, seed=5, scale=0.2)
    col = pol.FusedRolloutCollector(env, sd, bootstrap=False, deterministic=True, precision="i8x4")
    col.reset()
    col.last_obs[7, 2] = float("nan")
    b = col.collect(1)
    act, val = _np(b.actions)[0], _np(b.values)[0]
    assert np.isnan(act[7]).all() and np.isnan(val[7])
    m, v = orc.attn_f32(sd, _np(b.observations)[0], precision="i8x4")
    assert bits_equal(act, m) and bits_equal(val, v)


def test_i8x4_flag_refused_elsewhere(gl, pol):
    from gym_lorenz import _native as nat

    env = gl.BatchedEnv("hr", 100, seed=1)
    mlp = pol.ActorCriticMlp(6, 2).state_dict()
    col = pol.FusedRolloutCollector(env, mlp, precision="bf16")
    col.reset()
    col.i8x4 = True  # the flag on the bf16 MlpPolicy kernel: refused before any launch
    with pytest.raises(nat.LorenzEnvError):
        col.collect(2)
    env.close()
