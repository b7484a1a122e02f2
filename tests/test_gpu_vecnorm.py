"""GPU: VecNormalize fused into the env step (lz_step_vecnorm + lz_vecnorm_apply,
SURVEY §8 f1).  Bars:
  * vs the NumPy restatement of SB3 2.7.1 VecNormalize (oracle/sb3_vecnorm.py) fed the
    raw outputs of an identical env: normalised obs / rewards / terminal observations
    rel/abs 2e-5, statistics rel 1e-5 (SB3 takes float32 np.mean / np.var, the device
    float64 sums) and rel 1e-10 against the same restatement fed float64 copies;
  * vs the unfused device path (separate moments / update / normalise launches):
    statistics rel 1e-12, outputs 1e-6 (same arithmetic, another summation order);
  * deterministic: two identical runs are bit-identical (fixed reduction order over
    workgroups and groups, whichever workgroup finishes last);
  * LZ_VN_DEFER (moments out, update in lz_vecnorm_apply -- the multi-GPU path with an
    all-reduce in between) is bit-identical to the in-kernel update.
"""
import ctypes

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def gl():
    import gym_lorenz

    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    return gym_lorenz


def _np(t):
    return t.detach().cpu().numpy() if isinstance(t, torch.Tensor) else np.asarray(t)


def _vn(gl, n, env_id="lorenz_pmsm-v0", seed=5, mes=37, dtype="float32", **kw):
    from gym_lorenz.vec_normalize import LorenzVecNormalize

    return LorenzVecNormalize(gl.make_vec(env_id, n, seed=seed, max_episode_steps=mes, dtype=dtype),
                              **kw)


@pytest.mark.parametrize("env_id,n,dtype,act_dim,obs_dim,norm_reward", [
    ("lorenz_pmsm-v0", 20000 + 37, "float32", 2, 6, True),    # 79 workgroups: 2 groups, ragged
    ("lorenz_pmsm-v0", 300, "float32", 2, 6, False),          # 2 workgroups, 1 group
    ("lorenz_transient-v0", 5000, "float32", 3, 8, True),     # obs_dim 8
    ("lorenz_dynamic-v0", 4096 + 5, "float64", 3, 6, True),   # fp64 env, float32 VecEnv view
    ("lorenz_pmsm-v0", 400000 + 13, "float32", 2, 6, True),   # 391 partials: split path
])
def test_fused_vecnormalize_matches_sb3_restatement(gl, env_id, n, dtype, act_dim, obs_dim,
                                                    norm_reward):
    from oracle.sb3_vecnorm import RunningMeanStd, VecNormalizeRef

    mes = 11
    raw = gl.make_vec(env_id, n, seed=5, max_episode_steps=mes, dtype=dtype)
    dev = _vn(gl, n, env_id, mes=mes, dtype=dtype, norm_obs=True, norm_reward=norm_reward,
              clip_obs=10.0)
    assert dev._fused
    ref = VecNormalizeRef(n, obs_dim, norm_obs=True, norm_reward=norm_reward, clip_obs=10.0)
    # the same statistics from float64 copies of the float32 obs: SB3's np.mean / np.var
    # run in float32 (rel error ~1e-6 at 20k rows), the device sums in float64
    ref64 = RunningMeanStd(shape=(obs_dim,))
    # above ~1e5 rows SB3's float32 np.mean / np.var over axis 0 (a row-by-row sum) is
    # itself off by ~1e-4: feed the restatement float64 copies there
    cast = (lambda x: x.astype(np.float64)) if n > 100000 else (lambda x: x)
    o_raw = raw.reset()
    ref64.update(o_raw.astype(np.float64))
    np.testing.assert_allclose(dev.reset(), ref.reset(cast(o_raw)), rtol=1e-5, atol=1e-5)
    rng = np.random.default_rng(0)
    lo = 1.0 if env_id != "lorenz_dynamic-v0" else 5.0
    saw_done = 0
    for k in range(25):
        a = rng.uniform(-lo, lo, (n, act_dim)).astype(np.float32)
        o_raw, r_raw, d_raw, i_raw = raw.step(a)
        term = {i: cast(i_raw[i]["terminal_observation"]) for i in np.nonzero(d_raw)[0]}
        o_ref, r_ref, d_ref, tn_ref = ref.step(cast(o_raw), r_raw, d_raw, term)
        ref64.update(o_raw.astype(np.float64))
        o_dev, r_dev, d_dev, i_dev = dev.step(a)
        assert np.array_equal(d_dev, d_raw)
        fin = np.isfinite(o_ref).all(axis=1)
        np.testing.assert_allclose(o_dev[fin], o_ref[fin], rtol=2e-5, atol=2e-5)
        np.testing.assert_allclose(r_dev, r_ref, rtol=2e-5, atol=2e-5)
        np.testing.assert_array_equal(_np(dev.get_original_obs()), o_raw)
        for i, t in tn_ref.items():
            saw_done += 1
            np.testing.assert_allclose(i_dev[int(i)]["terminal_observation"], t, rtol=2e-5, atol=2e-5)
            assert i_dev[int(i)]["TimeLimit.truncated"] == i_raw[int(i)]["TimeLimit.truncated"]
    assert saw_done >= n
    if np.isfinite(ref.obs_rms.mean).all():
        np.testing.assert_allclose(dev.obs_rms.mean, ref.obs_rms.mean, rtol=1e-5, atol=1e-5)
        np.testing.assert_allclose(dev.obs_rms.var, ref.obs_rms.var, rtol=1e-5)
        np.testing.assert_allclose(dev.obs_rms.mean, ref64.mean, rtol=1e-10, atol=1e-10)
        np.testing.assert_allclose(dev.obs_rms.var, ref64.var, rtol=1e-10)
    assert dev.obs_rms.count == pytest.approx(ref.obs_rms.count)
    np.testing.assert_allclose(dev.ret_rms.mean, ref.ret_rms.mean, rtol=1e-6, atol=1e-9)
    np.testing.assert_allclose(dev.ret_rms.var, ref.ret_rms.var, rtol=1e-6)
    np.testing.assert_allclose(_np(dev.returns), ref.returns, rtol=1e-6, atol=1e-9)


def test_fused_matches_unfused_and_is_deterministic(gl):
    n = 70000  # 274 workgroups -> 5 groups of 64
    runs = []
    for fused in (True, True, False):
        v = _vn(gl, n, mes=9, norm_reward=True)
        v._fused = fused
        v.reset()
        rng = np.random.default_rng(3)
        outs = []
        for k in range(12):
            o, r, d, info = v.step(rng.uniform(-1.2, 1.2, (n, 2)).astype(np.float32))
            outs.append((o, r, d))
        stats = np.concatenate([v.obs_rms.mean, v.obs_rms.var, [v.obs_rms.count],
                                v.ret_rms.mean.ravel(), v.ret_rms.var.ravel(), _np(v.returns)])
        runs.append((outs, stats))
        v.close()
    (a, sa), (b, sb), (c, sc) = runs
    assert np.array_equal(sa, sb)  # deterministic, bit for bit
    for x, y in zip(a, b):
        for p, q in zip(x, y):
            assert np.array_equal(p, q)
    np.testing.assert_allclose(sa, sc, rtol=1e-12, atol=1e-12)
    for x, y in zip(a, c):
        np.testing.assert_allclose(x[0], y[0], rtol=1e-6, atol=1e-6)
        np.testing.assert_allclose(x[1], y[1], rtol=1e-6, atol=1e-6)
        assert np.array_equal(x[2], y[2])


@pytest.mark.parametrize("n", [20000, 400000 + 13])  # fused / split reduction
def test_defer_matches_in_kernel_update(gl, n):
    """The multi-GPU split (moments out, all-reduce, update in lz_vecnorm_apply) with a
    one-rank 'all-reduce' (identity) is bit-identical to the in-kernel update, with the
    normalise pass reducing the partials itself (20k envs) or k_vn_colsum doing it once
    (400k envs: more than 384 partials per column)."""
    import gym_lorenz._native as nat

    va, vb = _vn(gl, n, norm_reward=True), _vn(gl, n, norm_reward=True)
    va.reset(), vb.reset()
    vb.group = object()  # DEFER flag; the all-reduce itself is skipped below
    be_b = vb.venv.backend
    rng = np.random.default_rng(1)
    for k in range(15):
        a = rng.uniform(-1, 1, (n, 2)).astype(np.float32)
        oa, ra, da, _ = va.step(a)
        # vb by hand: step (DEFER) -> [all-reduce] -> apply
        o, t = be_b.obs_dim, be_b.tdtype
        dev = be_b.device
        obs, rew = torch.empty((n, o), dtype=t, device=dev), torch.empty((n,), dtype=t, device=dev)
        done = torch.empty((n,), dtype=torch.uint8, device=dev)
        didx = torch.empty((n,), dtype=torch.int32, device=dev)
        tobs = torch.empty((n, o), dtype=t, device=dev)
        nd = torch.zeros((1,), dtype=torch.int32, device=dev)
        vn = vb._vn_args()
        assert vn.flags & nat.VN_DEFER
        be_b.step_vecnorm(torch.from_numpy(a).to(dev), vn, (obs, rew, done), (didx, tobs, nd))
        m = _np(vb._moments)
        assert m[0] == n and m[2 * o + 1] == n
        on, rn = torch.empty((n, o), device=dev), torch.empty((n,), device=dev)
        tn = torch.empty((n, o), device=dev)
        be_b.vecnorm_apply(vn, obs, rew, on, rn, tobs, nd, tn)
        assert np.array_equal(_np(on), oa) and np.array_equal(_np(rn), ra)
        assert np.array_equal(_np(done).astype(bool), da)
    for x, y in ((va.obs_rms, vb.obs_rms), (va.ret_rms, vb.ret_rms)):
        assert np.array_equal(x.mean, y.mean) and np.array_equal(x.var, y.var)
        assert x.count == y.count
    assert np.array_equal(_np(va.returns), _np(vb.returns))


def test_fused_not_training_and_tensor_path(gl):
    n = 3000
    v = _vn(gl, n, mes=4, norm_reward=True)
    vt = _vn(gl, n, mes=4, norm_reward=True)
    vt.venv.return_tensors = True
    v.reset(), vt.reset()
    rng = np.random.default_rng(2)
    for k in range(6):
        a = rng.uniform(-1, 1, (n, 2)).astype(np.float32)
        o, r, d, info = v.step(a)
        ot, rt, dt, it = vt.step(torch.from_numpy(a).cuda())
        assert np.array_equal(_np(ot), o) and np.array_equal(_np(rt), r)
        assert np.array_equal(_np(dt), d)
        for i in np.nonzero(d)[0]:
            assert np.array_equal(_np(it[int(i)]["terminal_observation"]),
                                  info[int(i)]["terminal_observation"])
    # evaluation mode: statistics frozen, returns only reset on done
    v.training = False
    mean, var, count = v.obs_rms.mean.copy(), v.obs_rms.var.copy(), v.obs_rms.count
    ret_before = _np(v.returns).copy()
    o, r, d, info = v.step(rng.uniform(-1, 1, (n, 2)).astype(np.float32))
    assert np.array_equal(v.obs_rms.mean, mean) and np.array_equal(v.obs_rms.var, var)
    assert v.obs_rms.count == count
    ret_after = _np(v.returns)
    assert np.array_equal(ret_after[~d], ret_before[~d]) and (ret_after[d] == 0).all()
    want = np.clip((_np(v.get_original_obs()).astype(np.float64) - mean) / np.sqrt(var + 1e-8),
                   -10, 10).astype(np.float32)
    assert np.array_equal(o, want)


def test_vecnorm_abi_errors(gl):
    import gym_lorenz._native as nat

    v = _vn(gl, 64)
    v.reset()
    be = v.venv.backend
    vn = v._vn_args()
    vn.ret_rms = v.obs_rms._h.value  # wrong dim (6 != 1)
    t = torch.empty((64 * 8,), device=be.device)
    args = [ctypes.c_void_p(t.data_ptr())] * 7
    assert nat.lib.lz_step_vecnorm(be._h, ctypes.byref(vn), *args) == nat.LZ_ERR_INVALID
    vn = v._vn_args()
    assert nat.lib.lz_step_vecnorm(be._h, ctypes.byref(vn), *args[:6], None) == nat.LZ_ERR_INVALID


def test_vecnorm_apply_refused_after_another_launch(gl):
    """lz_step_vecnorm leaves its done cursor and moment partials for the paired
    lz_vecnorm_apply; a launch in between (here a plain lz_step, which reuses the cursor)
    makes the apply refuse with LZ_ERR_STATE instead of publishing a wrong done count or
    stale statistics.  The next proper step_vecnorm + apply pair works again."""
    from gym_lorenz import _native as nat

    n = 4096
    dev = _vn(gl, n, norm_obs=True, norm_reward=False, clip_obs=10.0)
    dev.reset()
    be = dev.venv.backend
    vn = dev._vn_args()
    o = be.obs_dim
    buf = [torch.empty((n, o), device="cuda"), torch.empty((n,), device="cuda"),
           torch.empty((n,), dtype=torch.uint8, device="cuda"),
           torch.empty((n + 1,), dtype=torch.int32, device="cuda"),
           torch.empty((n, o), device="cuda"), torch.empty((n, o), device="cuda"),
           torch.empty((n,), device="cuda"), torch.empty((n,), dtype=torch.uint8, device="cuda"),
           torch.empty((n, o), device="cuda")]
    p = [t.data_ptr() for t in buf]
    acts = torch.zeros((n, 2), device="cuda")
    nat.check(nat.lib.lz_step_vecnorm(be._h, vn, acts.data_ptr(), p[0], p[1], p[2], p[3], p[4],
                                      p[3] + 4 * n))
    be.step(acts)  # another launch on the handle
    st = nat.lib.lz_vecnorm_apply(be._h, vn, p[0], p[1], p[2], p[5], p[6], p[7], p[4],
                                  p[3] + 4 * n, p[8])
    assert st == nat.LZ_ERR_STATE
    # a proper pair goes through
    nat.check(nat.lib.lz_step_vecnorm(be._h, vn, acts.data_ptr(), p[0], p[1], p[2], p[3], p[4],
                                      p[3] + 4 * n))
    nat.check(nat.lib.lz_vecnorm_apply(be._h, vn, p[0], p[1], p[2], p[5], p[6], p[7], p[4],
                                       p[3] + 4 * n, p[8]))
    torch.cuda.synchronize()
    obs, rew, done, infos = dev.step(np.zeros((n, 2), np.float32))  # the wrapper still works
    assert obs.shape == (n, o)
