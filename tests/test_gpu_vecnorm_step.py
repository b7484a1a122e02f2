"""SB3-exact VecNormalize in the fused float32 policy rollout (lz_rollout_policy_f32_vn,
SURVEY §8 f3; VERDICT r02 "next" 1).

The reference's PMSM learner (code/lorenz_pmsm/train.py:170-181: A2C MlpPolicy [128,128]
Tanh, n_steps=16, behind VecNormalize(norm_obs=True, norm_reward=False, clip_obs=10))
runs SB3 2.7.1 collect_rollouts, where VecNormalize.step_wait updates obs_rms with each
step's batch BEFORE normalising that step's observations and its terminal observations.
The check drives three consecutive K=16 collects from RunningMeanStd's count = 1e-4 at
65,637 PMSM envs (ragged: 2,051 tiles of 32 + 5 envs) and replays them step by step on
the CPU:

  * raw observations: a twin handle stepped by lz_rollout with the collect's clipped
    actions (the env part is bit-exact, tests/test_gpu_policy.py);
  * statistics: oracle.vn_tile_totals (lz_oracle.c orc_vn_tile_totals, the device's
    float64 moment order) + oracle.vn_rms_update (update_from_moments);
  * normalised observations of EVERY env and step, and obs_rms after every collect:
    bit for bit;
  * deterministic actions and values: oracle.mlp_f32 of the recorded observations,
    bit for bit (a sample of rows per step), last values likewise;
  * truncation bootstraps: reward = env reward + float32(gamma * V(terminal obs
    normalised with the statistics of ITS step)), bit for bit.

Against SB3's own statistics arithmetic (np.mean / np.var of the float32 rows,
oracle/sb3_vecnorm.py): the only difference is the moment summation (float64 sums in a
fixed tree here; float32 row-sequential sums in NumPy), so the normalised observations
differ by rounding of the statistics only -- the bound is printed and gated below.
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


def _random_policy(pol, O, A, seed, scale=0.4):
    net = pol.ActorCriticMlp(O, A, seed=seed)
    g = torch.Generator().manual_seed(seed + 1)
    with torch.no_grad():
        for p in net.parameters():
            p.copy_(torch.randn(p.shape, generator=g) * (scale if p.dim() > 1 else 0.3))
    return {k: v.detach().clone() for k, v in net.state_dict().items()}


def test_sb3_exact_vecnorm_three_collects(gl, pol, orc):
    from gym_lorenz.vec_normalize import DeviceRunningMeanStd
    from oracle.sb3_vecnorm import RunningMeanStd as SB3RMS

    n, K, R, gamma, eps, clip = 65637, 16, 3, 0.99, 1e-8, 10.0
    kw = dict(seed=3, add_noise=True, alpha=0.25, max_episode_steps=20)
    env = gl.BatchedEnv("pmsm", n, **kw)
    twin = gl.BatchedEnv("pmsm", n, **kw)
    sd = _random_policy(pol, 6, 2, seed=8)
    rms = DeviceRunningMeanStd(6, env.device)  # SB3 RunningMeanStd(epsilon=1e-4)
    col = pol.FusedRolloutCollector(env, sd, gamma=gamma, obs_rms=rms, clip_obs=clip,
                                    norm_eps=eps, training=True, bootstrap=True,
                                    deterministic=True, capture_terminal=K * n,
                                    precision="fp32")
    assert col.per_step_vecnorm
    raw = _np(col.reset())
    twin.reset()
    lo, hi = pol.action_bounds("pmsm")
    mean, var, count = np.zeros(6), np.ones(6), 1e-4
    s, q = orc.vn_tile_totals(raw)
    mean, var, count = orc.vn_rms_update(mean, var, count, n, s, q)
    sb3 = SB3RMS(shape=(6,))
    sb3.update(raw)
    rng = np.random.default_rng(0)
    worst_sb3, n_boot = 0.0, 0
    for r in range(R):
        b = col.collect(K)
        obs_t, rew_t, done_t = twin.rollout(torch.clamp(b.actions, lo, hi).contiguous())
        obs_t, rew_t, done_t = _np(obs_t), _np(rew_t), _np(done_t)
        assert np.array_equal(_np(b.dones), done_t)
        seen = _np(b.observations)
        stats = []
        for k in range(K):
            x = orc.vn_normalize(raw, mean, var, eps, clip)
            assert bits_equal(seen[k], x), (r, k, np.nanmax(np.abs(seen[k] - x)))
            x_sb3 = np.clip((raw - sb3.mean) / np.sqrt(sb3.var + eps), -clip, clip).astype(np.float32)
            fin = np.isfinite(x_sb3) & np.isfinite(x)
            worst_sb3 = max(worst_sb3, float(np.abs(x_sb3[fin] - x[fin]).max()))
            raw = obs_t[k]
            s, q = orc.vn_tile_totals(raw)
            mean, var, count = orc.vn_rms_update(mean, var, count, n, s, q)
            sb3.update(raw)
            stats.append((mean, var))
        # obs_rms after the collect: bit for bit
        st = _np(rms.state)
        assert bits_equal(st, np.concatenate([mean, var, [count]])), (st, mean, var, count)
        assert bits_equal(_np(b.last_obs), raw)
        # the policy forward on what it saw (deterministic: action = mean), sampled rows
        for k in range(K):
            rows = rng.choice(n, 384, replace=False)
            m, v = orc.mlp_f32(sd, seen[k][rows])
            assert bits_equal(_np(b.actions[k])[rows], m), (r, k)
            assert bits_equal(_np(b.values[k])[rows], v), (r, k)
        rows = np.concatenate([rng.choice(n, 512, replace=False), np.arange(n - 5, n)])
        _, vl = orc.mlp_f32(sd, orc.vn_normalize(raw[rows], mean, var, eps, clip))
        assert bits_equal(_np(b.last_values)[rows], vl)
        # rewards: the env's, plus the truncation bootstraps valued with their step's stats
        rew = _np(b.rewards)
        m_done = int(b.n_done.item())
        idx = _np(b.done_idx[:m_done])
        tobs = _np(b.terminal_obs[:m_done])
        kk, ee = idx // n, idx % n
        d = done_t[kk, ee]
        trunc = ((d & 2) != 0) & ((d & 1) == 0)
        boot = np.zeros((K, n), bool)
        boot[kk[trunc], ee[trunc]] = True
        assert np.array_equal(rew[~boot], rew_t[~boot])
        for k in range(K):
            sel = trunc & (kk == k)
            if not sel.any():
                continue
            mk, vk = stats[k]
            _, vt = orc.mlp_f32(sd, orc.vn_normalize(tobs[sel], mk, vk, eps, clip))
            want = (rew_t[k, ee[sel]] + (np.float32(gamma) * vt).astype(np.float32)).astype(np.float32)
            assert bits_equal(rew[k, ee[sel]], want), (r, k)
            n_boot += int(sel.sum())
    assert n_boot > 0, "no truncation inside the three collects"
    print("SB3-exact VecNormalize: 3 x %d steps x %d envs bit-exact vs the step-by-step oracle "
          "(%d truncation bootstraps); vs SB3's float32 np.mean / np.var statistics: max "
          "|d normalised obs| = %.3g" % (K, n, n_boot, worst_sb3))
    assert worst_sb3 <= 1e-3
    for e in (env, twin):
        e.close()


def test_sb3_exact_differs_from_pooled_and_matches_sb3_order(gl, pol, orc):
    """From count = 1e-4 the pooled mode (vecnorm_update="rollout") feeds the policy
    statistics of the reset batch only for all K steps; SB3's order moves them every
    step.  The two modes must agree on step 0 and differ after it."""
    from gym_lorenz.vec_normalize import DeviceRunningMeanStd

    n, K = 8192, 6
    outs = []
    for mode in ("step", "rollout"):
        env = gl.BatchedEnv("pmsm", n, seed=11, add_noise=True)
        rms = DeviceRunningMeanStd(6, env.device)
        col = pol.FusedRolloutCollector(env, _random_policy(pol, 6, 2, seed=4), obs_rms=rms,
                                        training=True, deterministic=True, bootstrap=False,
                                        precision="fp32", vecnorm_update=mode)
        col.reset()
        outs.append(_np(col.collect(K).observations))
        env.close()
    a, b = outs
    # step 0 normalised by the reset update in both (the reset moment orders differ:
    # tile sums vs lz_rms_moments, so allow rounding)
    np.testing.assert_allclose(a[0], b[0], rtol=0, atol=1e-5)
    assert np.abs(a[1:] - b[1:]).max() > 1e-3


def test_odd_k_collect_then_step_done_list(gl, pol):
    """a collect of the SB3-exact path flips the handle's call parity once per
    step (K flips) and runs on its own done cursor.  After an odd K (A2C's default
    n_steps = 5) the next lz_step must start its compact done list from 0, not from the
    count an earlier launch left in that parity slot: every step launch of the collect
    zeroes the slot the handle's next launch reads.  Here the earlier launch marked all n
    envs done (TimeLimit(1)); the step after the collect must report exactly its own n."""
    from gym_lorenz.vec_normalize import DeviceRunningMeanStd

    n = 4096
    env = gl.BatchedEnv("pmsm", n, seed=2, add_noise=True, max_episode_steps=1)
    rms = DeviceRunningMeanStd(6, env.device)
    col = pol.FusedRolloutCollector(env, _random_policy(pol, 6, 2, seed=1), obs_rms=rms,
                                    training=True, precision="fp32")
    assert col.per_step_vecnorm
    col.reset()
    a = torch.zeros((n, 2), device=env.device)
    env.step(a)  # every env truncates: this launch's cursor slot holds n
    assert int(env.n_done_dev.item()) == n
    col.collect(5)  # odd K
    didx = torch.full((2 * n + 1,), -1, dtype=torch.int32, device=env.device)
    tobs = torch.empty((2 * n, 6), device=env.device)
    nd = torch.zeros((1,), dtype=torch.int32, device=env.device)
    env.step(a, compact_out=(didx, tobs, nd))
    assert int(nd.item()) == n
    assert np.array_equal(np.sort(_np(didx[:n])), np.arange(n))
    assert (_np(didx[n:]) == -1).all()
    env.close()


def test_policy_step_order_guard(gl, pol):
    """lz_policy_step_f32 carries the terminal-obs carry, the collect's done
    cursor and the RNG parity from step to step, so it refuses (LZ_ERR_STATE) a step k > 0
    that is not the one expected next, or that follows another launch on the handle; a
    new collect (k = 0) always starts."""
    import ctypes

    from gym_lorenz import _native as nat
    from gym_lorenz.policy import pack_policy_f32
    from gym_lorenz.vec_normalize import DeviceRunningMeanStd

    n, K = 1000, 3
    env = gl.BatchedEnv("pmsm", n, seed=4)
    obs0 = env.reset().clone()
    dev = env.device
    rms = DeviceRunningMeanStd(6, dev)
    blob = torch.from_numpy(pack_policy_f32(_random_policy(pol, 6, 2, seed=3), 6, 2)).to(dev)
    bufs = dict(obs_buf=torch.empty((K, n, 6), device=dev), act_buf=torch.empty((K, n, 2), device=dev),
                logp_buf=torch.empty((K, n), device=dev), val_buf=torch.empty((K, n), device=dev),
                rew_buf=torch.empty((K, n), device=dev),
                done_buf=torch.empty((K, n), dtype=torch.uint8, device=dev),
                last_values=torch.empty((n,), device=dev))
    last = torch.empty((n, 6), device=dev)
    r = nat.LzPolicyRolloutArgs()
    r.K, r.flags = K, nat.POLICY_DETERMINISTIC
    r.blob, r.obs_in, r.obs_last = blob.data_ptr(), obs0.data_ptr(), last.data_ptr()
    for k_, v in bufs.items():
        setattr(r, k_, v.data_ptr())
    r.norm_eps, r.clip_obs, r.gamma, r.act_low, r.act_high = 1e-8, 10.0, 0.99, -1.0, 1.0
    state = ctypes.c_void_p(rms.state.data_ptr())
    step = lambda k: nat.lib.lz_policy_step_f32(env._h, ctypes.byref(r), k, state, None)  # noqa: E731
    assert step(1) == nat.LZ_ERR_STATE and b"out of order" in nat.lib.lz_last_error()
    assert step(0) == nat.LZ_OK and step(1) == nat.LZ_OK
    env.step(torch.zeros((n, 2), device=dev))  # another launch in the middle of the collect
    assert step(2) == nat.LZ_ERR_STATE
    for k in range(K + 1):  # a fresh collect runs through
        assert step(k) == nat.LZ_OK, (k, nat.lib.lz_last_error())
    assert step(1) == nat.LZ_ERR_STATE  # the collect has ended
    torch.cuda.synchronize()
    env.close()
