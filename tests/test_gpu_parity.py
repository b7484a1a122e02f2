"""GPU parity: the HIP kernels (through the C-ABI) against the golden fixtures of the
reference and the CPU oracle.  Bars:
  * LORENZ3 / LORENZ4 fp64: bit-exact vs the reference (golden), every step.
  * all systems, both dtypes: bit-exact vs the oracle restatement of the device
    formulas (oracle mode DEV), NaN-aware.
  * PMSM vs reference: obs/state bit-exact; reward rel <= 1e-5 (glibc powf vs the
    device's pow: the reward's x**alpha and the Adam g**2 are the only libm calls).
  * HR fp64 vs reference: rel <= 1e-9 over 1000 RK4 steps (glibc pow(x,3)/(x,2) are
    not correctly rounded; the device's are).
  * LORENZ3 fp32 vs fp64 reference, teacher-forced per step: rel < 1e-5
    (BASELINE.md per-step gate; |d| / max(|s|, 1)).
"""
import numpy as np
import pytest
import torch

from conftest import bits_equal, golden

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def gl():
    import gym_lorenz

    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    return gym_lorenz


def _np(t):
    return t.detach().cpu().numpy()


def _planes(be, first, count):
    return np.stack([_np(be.get_state(first + j)) for j in range(count)], axis=1)


# ----------------------------------------------------------------- LORENZ3
@pytest.mark.parametrize("use_rollout", [False, True])
def test_l3_f64_golden_bitexact(gl, use_rollout):
    g = golden("l3")
    n, T = g["x0"].shape[0], g["obs"].shape[1]
    be = gl.BatchedEnv("lorenz3", n, dtype="float64", autoreset=False)
    obs0 = _np(be.reset(init=torch.from_numpy(g["x0"])))
    assert bits_equal(obs0, g["obs0"])
    acts = torch.from_numpy(np.ascontiguousarray(g["actions"].transpose(1, 0, 2))).cuda()
    if use_rollout:
        obs, rew, done = be.rollout(acts)
    else:
        obs = torch.empty((T, n, 6), dtype=torch.float64, device="cuda")
        rew = torch.empty((T, n), dtype=torch.float64, device="cuda")
        done = torch.empty((T, n), dtype=torch.uint8, device="cuda")
        for k in range(T):
            o, r, d = be.step(acts[k])
            obs[k].copy_(o)
            rew[k].copy_(r)
            done[k].copy_(d)
    assert bits_equal(_np(obs).transpose(1, 0, 2), g["obs"])
    assert bits_equal(_np(rew).T, g["reward"])
    assert not _np(done).any()


def test_l3_f32_bitexact_vs_oracle_ragged(gl, orc):
    """Device Philox resets + 200 steps, N not a multiple of 256 nor of 4."""
    n, T = 65536 + 37, 200
    be = gl.BatchedEnv("lorenz3", n, dtype="float32", seed=1234, autoreset=False)
    obs0 = _np(be.reset())
    init = orc.reset_draw("l3", np.float32, n, 0, 1234, 0)
    assert bits_equal(_planes(be, 0, 3), init)
    assert bits_equal(obs0, orc.l3_reset_obs(init))
    rng = np.random.default_rng(5)
    st = init.copy()
    for k in range(T):
        a = rng.uniform(-1, 1, (n, 3)).astype(np.float32)
        if k == 3:
            a[:100] *= 900.0  # clip path
        o, r, _ = be.step(torch.from_numpy(a))
        with np.errstate(all="ignore"):
            oo, rr = orc.l3_step(st, a.astype(np.float32))
        if k % 40 == 0 or k == T - 1:
            assert bits_equal(_np(o), oo), k
            assert bits_equal(_np(r), rr), k
    assert bits_equal(_planes(be, 0, 3), st)


def test_l3_f32_teacher_forced_vs_reference(gl):
    """Every (env, step) pair of the fp64 golden as its own env: start from the
    reference state rounded to f32, one f32 step, compare with the reference's
    next state.  Gate: relative error |d|/max(|s|,1) < 1e-5."""
    g = golden("l3")
    s_prev = np.concatenate([g["x0"][:, None, :], g["obs"][:, :-1, :3]], axis=1)  # [n,T,3]
    s_next = g["obs"][:, :, :3]
    acts = g["actions"]
    fin = np.isfinite(s_prev).all(-1) & np.isfinite(s_next).all(-1) & (np.abs(s_next) < 1e6).all(-1)
    sp, sn, a = s_prev[fin], s_next[fin], acts[fin]
    be = gl.BatchedEnv("lorenz3", sp.shape[0], dtype="float32", autoreset=False)
    be.reset(init=torch.from_numpy(sp.astype(np.float32)))
    o, r, _ = be.step(torch.from_numpy(a.astype(np.float32)))
    got = _np(o)[:, :3].astype(np.float64)
    rel = np.abs(got - sn) / np.maximum(np.abs(sn), 1.0)
    assert rel.max() < 1e-5, rel.max()


# ----------------------------------------------------------------- LORENZ4
def test_l4_f64_golden_bitexact(gl):
    g = golden("l4")
    n, T = g["init"].shape[0], g["obs"].shape[1]
    be = gl.BatchedEnv("lorenz4", n, dtype="float64", autoreset=False)
    assert bits_equal(_np(be.reset(init=torch.from_numpy(g["init"]))), g["obs0"])
    acts = torch.from_numpy(np.ascontiguousarray(g["actions"].transpose(1, 0, 2))).cuda()
    obs, rew, done = be.rollout(acts)
    assert bits_equal(_np(obs).transpose(1, 0, 2), g["obs"])
    assert bits_equal(_np(rew).T, g["reward"])
    assert np.array_equal(_np(done).T.astype(bool), g["done"])


def test_l4_f32_vs_oracle(gl, orc):
    n, T = 3000, 100
    be = gl.BatchedEnv("lorenz4", n, dtype="float32", seed=9, autoreset=False)
    be.reset()
    st = orc.reset_draw("l4", np.float32, n, 0, 9, 0)
    assert bits_equal(np.concatenate([_planes(be, 0, 4), _planes(be, 4, 4)], 1), st)
    st = st.copy()
    for k in range(T):
        o, r, d = be.step(torch.zeros((n, 3)))
        with np.errstate(all="ignore"):
            oo, rr, dd = orc.l4_step(st)
    assert bits_equal(_np(o), oo) and bits_equal(_np(r), rr)


@pytest.mark.parametrize("n,rollout", [(65536, False), (70001, False), (65536, True), (70001, True)])
def test_l4_f32_vs_oracle_cfg2(gl, orc, n, rollout):
    """cfg2's lorenz_env_transient at its size (65,536) and ragged (70,001): float32
    LORENZ4 vs the oracle bit for bit through lz_step (2048 steps) and through one K = 2048
    lz_rollout launch (the 256-lane kernel with the alternating obs tiles at both sizes:
    LORENZ4 f32 switches to it from 3/4 x 256 x CUs envs), with a TimeLimit(500) whose
    truncations are staggered by per-env step counters, auto-reset from device Philox:
    every step's obs / reward / done bytes, every compact done list (ids, terminal obs)
    and the final state planes."""
    from oracle_tl import OracleTL

    K, L = 2048, 500
    be = gl.BatchedEnv("lorenz4", n, dtype="float32", seed=13, max_episode_steps=L)
    be.reset()
    steps0 = np.random.default_rng(13).integers(0, L, n).astype(np.int32)
    be.set_state(gl._native.L4_STEP, torch.from_numpy(steps0))
    ref = OracleTL(orc, "l4", np.float32, n, 13, L, steps0)
    zero = torch.zeros((n, 3), device="cuda")
    if rollout:
        obs, rew, done, (didx, tobs, nd) = be.rollout(torch.zeros((K, n, 3), device="cuda"),
                                                      capture_terminal=8 * n)
        wi, wt = [], []
    for k in range(K):
        oo, rr, dd, idx, term = ref.step()
        if rollout:
            o, r, d = obs[k], rew[k], done[k]
            wi.append(k * n + idx)
            wt.append(term)
        else:
            o, r, d = be.step(zero)
            nd_k = int(be.n_done_dev.item())
            assert nd_k == idx.size, k
            if nd_k:
                gi, gt = be.done_list()
                assert np.array_equal(_np(gi), idx) and bits_equal(_np(gt), term), k
        assert bits_equal(_np(o), oo), k
        assert bits_equal(_np(r), rr), k
        assert np.array_equal(_np(d), dd), k
    if rollout:
        m = int(nd.item())
        wi = np.concatenate(wi)
        assert m == wi.size and m >= 4 * n
        order = torch.argsort(didx[:m])
        assert np.array_equal(_np(didx[:m][order]), wi)
        assert bits_equal(_np(tobs[:m][order]), np.concatenate(wt))
    st = np.stack([_np(be.get_state(p)) for p in range(8)], 1)
    assert bits_equal(st, ref.st)
    be.close()


# ----------------------------------------------------------------- PMSM
def _pmsm_case(gl, g, i):
    T = g["obs"].shape[1]
    be = gl.BatchedEnv("pmsm", 1, alpha=float(g["alpha"][i]), add_noise=bool(g["add_noise"][i]),
                       autoreset=False)
    be.reset(init=torch.from_numpy(g["init"][i, 0].reshape(1, 6)))
    noise = torch.from_numpy(g["noise"][i]).cuda()
    acts = torch.from_numpy(g["actions"][i]).cuda()
    obs = torch.empty((T, 6), device="cuda")
    rew = torch.empty((T,), device="cuda")
    flags = torch.empty((T,), dtype=torch.uint8, device="cuda")
    lam = torch.empty((T,), device="cuda")
    for k in range(T):
        if k == int(g["reset_at"]):
            be.reset(init=torch.from_numpy(g["init"][i, 1].reshape(1, 6)))
        o, r, d = be.step(acts[k:k + 1], noise[k:k + 1] if g["add_noise"][i] else None)
        obs[k].copy_(o[0])
        rew[k].copy_(r[0])
        flags[k].copy_(d[0])
        lam[k].copy_(be.get_state(6)[0])
    return _np(obs), _np(rew), _np(flags), _np(lam)


@pytest.mark.parametrize("i", range(9))
def test_pmsm_vs_reference_and_oracle(gl, orc, i):
    g = golden("pmsm")
    obs, rew, flags, lam = _pmsm_case(gl, g, i)
    # reference: state path bit-exact, reward within the powf tolerance
    assert bits_equal(obs, g["obs"][i])
    assert np.array_equal((flags & 1).astype(bool), g["terminated"][i])
    assert np.array_equal((flags & 2).astype(bool), g["truncated"][i])
    fin = np.isfinite(g["reward"][i])
    np.testing.assert_allclose(rew[fin], g["reward"][i][fin], rtol=1e-5, atol=0)
    # oracle DEV: everything bit-exact
    from test_oracle_golden import _run_pmsm

    ref = _run_pmsm(orc, g, i, orc.DEV)
    assert bits_equal(rew, ref["rew"])
    assert bits_equal(lam, ref["lam"])


# ----------------------------------------------------------------- HR
@pytest.mark.parametrize("i", range(8))
def test_hr_f64_vs_reference_and_oracle(gl, orc, i):
    g = golden("hr")
    T = g["obs"].shape[1]
    be = gl.BatchedEnv("hr", 1, dtype="float64", autoreset=False,
                       add_noise=bool(g["add_noise"][i]), add_filter=bool(g["add_filter"][i]),
                       eval_mode=bool(g["eval_mode"][i]))
    o0 = _np(be.reset(init=torch.from_numpy(g["init"][i].reshape(1, 7))))
    assert bits_equal(o0[0].astype(np.float32), g["obs0"][i])
    noise = torch.from_numpy(g["noise"][i]).cuda()
    acts = torch.from_numpy(g["actions"][i]).cuda()
    obs = torch.empty((T, 6), dtype=torch.float64, device="cuda")
    rew = torch.empty((T,), dtype=torch.float64, device="cuda")
    fl = torch.empty((T,), dtype=torch.uint8, device="cuda")
    for k in range(T):
        o, r, d = be.step(acts[k:k + 1], noise[k:k + 1] if g["add_noise"][i] else None)
        obs[k].copy_(o[0])
        rew[k].copy_(r[0])
        fl[k].copy_(d[0])
    obs, rew, fl = _np(obs), _np(rew), _np(fl)
    from test_oracle_golden import _run_hr

    oo, rr, tt = _run_hr(orc, g, i, orc.DEV)
    assert bits_equal(obs, oo) and bits_equal(rew, rr)
    assert np.array_equal((fl & 1).astype(bool), tt)
    np.testing.assert_allclose(obs.astype(np.float32), g["obs"][i], rtol=1e-6, atol=1e-7)
    np.testing.assert_allclose(rew, g["reward"][i], rtol=1e-9, atol=1e-12)
    assert np.array_equal((fl & 1).astype(bool), g["terminated"][i])


# ----------------------------------------------------------------- RNG / resets
@pytest.mark.parametrize("system,dtype,kw", [
    ("lorenz3", "float64", {}), ("lorenz4", "float64", {}), ("lorenz4", "float32", {}),
    ("pmsm", "float32", {}), ("hr", "float64", {"add_noise": True}),
    ("hr", "float32", {"add_noise": True, "eval_mode": True}), ("hr", "float32", {})])
def test_device_reset_draws_match_oracle(gl, orc, system, dtype, kw):
    n = 5000
    be = gl.BatchedEnv(system, n, dtype=dtype, seed=77, global_env_offset=123, autoreset=False, **kw)
    be.reset()
    want = orc.reset_draw({"lorenz3": "l3", "lorenz4": "l4", "pmsm": "pmsm", "hr": "hr"}[system],
                          np.dtype(dtype), n, 123, 77, 0, add_noise=kw.get("add_noise", False),
                          eval_mode=kw.get("eval_mode", False))
    cnt = want.shape[1]
    got = _planes(be, 0, cnt)
    if system == "hr" and not kw.get("add_noise"):
        want[:, 6] = 0
    assert bits_equal(got.astype(want.dtype), want)


def test_autoreset_compaction_truncation(gl, orc):
    """TimeLimit truncation at step 7: every env done, compact list complete,
    terminal obs = the oracle's pre-reset obs, returned obs = fresh reset obs."""
    n, L = 3000, 7
    be = gl.BatchedEnv("lorenz3", n, dtype="float32", seed=3, max_episode_steps=L)
    be.reset()
    st = orc.reset_draw("l3", np.float32, n, 0, 3, 0)
    a = np.random.default_rng(1).uniform(-1, 1, (n, 3)).astype(np.float32)
    for k in range(L):
        o, r, d = be.step(torch.from_numpy(a))
        oo, _ = orc.l3_step(st, a)
        if k < L - 1:
            assert not _np(d).any()
    assert (_np(d) == 2).all()
    idx, tobs = be.done_list()
    assert np.array_equal(_np(idx), np.arange(n))
    assert bits_equal(_np(tobs), oo)
    fresh = orc.reset_draw("l3", np.float32, n, 0, 3, L)  # auto-reset draws at tick L
    assert bits_equal(_np(o), orc.l3_reset_obs(fresh))
    assert bits_equal(_planes(be, 0, 3), fresh)
    assert (_np(be.get_state(3)) == 0).all()
    o, r, d = be.step(torch.from_numpy(a))
    assert not _np(d).any()


def test_done_cursor_zeroed_by_reset(gl, orc):
    """step (every env done) -> lz_reset -> step: the reset launch zeroes the compact
    list cursor the next step reads, so n_done / done_list() report only that step's
    done envs (the cursor used to start at the previous step's count)."""
    n, L = 2000, 3
    be = gl.BatchedEnv("lorenz3", n, dtype="float32", seed=9, max_episode_steps=L)
    be.reset()
    a = torch.zeros((n, 3))
    for _ in range(L):
        o, r, d = be.step(a)
    assert (_np(d) == 2).all() and int(be.n_done_dev.item()) == n
    be.reset()
    be.set_state(gl._native.L3_STEP, torch.from_numpy(np.where(np.arange(n) % 7 == 0, L - 1, 0)
                                                       .astype(np.int32)))
    o, r, d = be.step(a)
    want = np.nonzero(np.arange(n) % 7 == 0)[0]
    assert int(be.n_done_dev.item()) == want.size
    idx, _ = be.done_list()
    assert np.array_equal(_np(idx), want)
    assert np.array_equal(np.nonzero(_np(d))[0], want)


def test_seed_then_reset_reproducible(gl, orc):
    """VecEnv.seed(s) + reset() draws the same initial states whatever calls came
    before (lz_set_seed rewinds the device call counter)."""
    n = 1000
    be = gl.BatchedEnv("lorenz3", n, dtype="float32", seed=1)
    be.reset()
    for _ in range(5):
        be.step(torch.zeros((n, 3)))
    be.set_seed(42)
    o1 = _np(be.reset()).copy()
    be.step(torch.zeros((n, 3)))
    be.reset()
    be.set_seed(42)
    o2 = _np(be.reset()).copy()
    assert bits_equal(o1, o2)
    assert bits_equal(o1, orc.l3_reset_obs(orc.reset_draw("l3", np.float32, n, 0, 42, 0)))


def test_autoreset_termination_pmsm(gl, orc):
    """PMSM error_sum > 1000 termination with auto-reset; Adam state persists."""
    n = 512
    be = gl.BatchedEnv("pmsm", n, seed=5)
    init = orc.reset_draw("pmsm", np.float32, n, 0, 5, 0)
    init[::2, 3:] += np.array([600, -600, 600], np.float32)  # push every other slave away
    be.reset(init=torch.from_numpy(init))
    S = orc.PmsmState(n)
    S.st[:] = init
    with np.errstate(all="ignore"):
        oo, rr, te, tr = orc.pmsm_step(S, np.zeros((n, 2), np.float32), None, False, 0.5, orc.DEV)
    o, r, d = be.step(torch.zeros((n, 2)))
    dd = _np(d)
    assert te[::2].mean() > 0.9 and not te[1::2].any()
    assert np.array_equal((dd & 1).astype(bool), te) and not (dd & 2).any()
    assert bits_equal(_np(r), rr)
    idx, tobs = be.done_list()
    assert np.array_equal(_np(idx), np.nonzero(te)[0])
    assert bits_equal(_np(tobs), oo[te])
    fresh = orc.reset_draw("pmsm", np.float32, n, 0, 5, 1)
    assert bits_equal(_np(o)[te], orc.pmsm_reset_obs(fresh)[te])
    assert bits_equal(_np(o)[~te], oo[~te])
    assert (_np(be.get_state(9)) == 1).all()  # adam_step kept counting through the reset
    assert bits_equal(_np(be.get_state(6)), S.lam)


def test_shard_invariance(gl):
    """Two shards [0,n/2) and [n/2,n) reproduce one handle of n envs bit for bit."""
    n, T = 8192, 20
    full = gl.BatchedEnv("hr", n, dtype="float32", seed=11, add_noise=True, max_episode_steps=9)
    parts = [gl.BatchedEnv("hr", n // 2, dtype="float32", seed=11, add_noise=True,
                           global_env_offset=r * n // 2, max_episode_steps=9) for r in range(2)]
    of = _np(full.reset())
    op = np.concatenate([_np(p.reset()) for p in parts])
    assert bits_equal(of, op)
    a = np.random.default_rng(2).uniform(-1, 1, (T, n, 2)).astype(np.float32)
    for k in range(T):
        of, rf, df = [_np(x) for x in full.step(torch.from_numpy(a[k]))]
        outs = [[_np(x) for x in p.step(torch.from_numpy(a[k][r * n // 2:(r + 1) * n // 2]))]
                for r, p in enumerate(parts)]
        assert bits_equal(of, np.concatenate([x[0] for x in outs]))
        assert bits_equal(rf, np.concatenate([x[1] for x in outs]))
        assert np.array_equal(df, np.concatenate([x[2] for x in outs]))


def test_cfg3_shard_geometry(gl):
    """BASELINE configs[2]'s real split: 8 ranks x 131,072 LORENZ3 envs at
    global_env_offset = r * 131,072 (run one after another on this GPU) reproduce one
    1,048,576-env handle bit for bit over 30 steps with auto-reset (a 7-step TimeLimit,
    so resets fire and their draws are keyed by the global env id): observations,
    rewards, done bytes and the compact done lists (shard ids + offset)."""
    S, R, T = 131_072, 8, 30
    full = gl.BatchedEnv("lorenz3", S * R, dtype="float32", seed=21, max_episode_steps=7)
    parts = [gl.BatchedEnv("lorenz3", S, dtype="float32", seed=21, max_episode_steps=7,
                           global_env_offset=r * S) for r in range(R)]
    of = full.reset()
    for r, p in enumerate(parts):
        assert torch.equal(p.reset().view(torch.int32), of[r * S:(r + 1) * S].view(torch.int32))
    g = torch.Generator(device="cuda").manual_seed(8)
    resets = 0
    for k in range(T):
        a = torch.rand((S * R, 3), generator=g, device="cuda") * 2 - 1
        of, rf, df = full.step(a)
        fidx, fterm = full.done_list()
        resets += fidx.numel()
        for r, p in enumerate(parts):
            sl = slice(r * S, (r + 1) * S)
            o, rw, d = p.step(a[sl])
            assert torch.equal(o.view(torch.int32), of[sl].view(torch.int32)), (k, r)
            assert torch.equal(rw.view(torch.int32), rf[sl].view(torch.int32)), (k, r)
            assert torch.equal(d, df[sl]), (k, r)
            pidx, pterm = p.done_list()
            m = (fidx >= r * S) & (fidx < (r + 1) * S)
            assert torch.equal(pidx + r * S, fidx[m]), (k, r)
            assert torch.equal(pterm.view(torch.int32), fterm[m].view(torch.int32)), (k, r)
    assert resets == 4 * S * R  # truncations at steps 7, 14, 21, 28
    full.close()
    for p in parts:
        p.close()


@pytest.mark.parametrize("system,dtype,n", [("lorenz3", "float32", 1000), ("pmsm", "float32", 1000),
                                            ("hr", "float64", 1000), ("lorenz4", "float32", 1000),
                                            ("lorenz3", "float32", 40001),
                                            ("lorenz3", "float32", 140000),
                                            ("pmsm", "float32", 140000),
                                            ("hr", "float32", 140000),
                                            ("pmsm", "float32", 140001),
                                            ("hr", "float32", 140001),
                                            ("lorenz4", "float32", 49153),
                                            ("lorenz4", "float32", 65536),
                                            ("lorenz4", "float32", 70001),
                                            ("lorenz4", "float32", 140001),
                                            ("lorenz4", "float64", 140001),
                                            ("singlecontrol", "float32", 140001)])
def test_rollout_equals_steps(gl, system, dtype, n):
    """Fused rollout (one-wave workgroups below 131,072 envs, below 256 x CUs for LORENZ3
    f32, 3/4 of that for LORENZ4 f32 -- two lanes per env for LORENZ3 f32 from 32,768 -- 256-lane above) == K
    steps.  The action-free systems (LORENZ4, singlecontrol) at 256-lane sizes cover the
    alternating obs tiles of k_rollout (a single tile raced: a fast wave's next-step writes
    against a slower wave's reads, seen at LORENZ4 70,001)."""
    K = 33
    kw = {"add_noise": True} if system in ("pmsm", "hr") else {}
    a_be = gl.BatchedEnv(system, n, dtype=dtype, seed=4, max_episode_steps=10, **kw)
    b_be = gl.BatchedEnv(system, n, dtype=dtype, seed=4, max_episode_steps=10, **kw)
    a_be.reset()
    b_be.reset()
    A = torch.from_numpy(np.random.default_rng(3).uniform(-1.5, 1.5, (K, n, a_be.action_dim))
                         .astype(np.float32)).cuda()
    obs, rew, done, (didx, tobs, nd) = a_be.rollout(A, capture_terminal=K * n)
    for k in range(K):
        o, r, d = b_be.step(A[k])
        assert bits_equal(_np(obs[k]), _np(o)), k
        assert bits_equal(_np(rew[k]), _np(r)), k
        assert np.array_equal(_np(done[k]), _np(d)), k
    nd = int(nd.item())
    assert nd == int((_np(done) != 0).sum())


@pytest.mark.parametrize("system,dtype,n,K", [("pmsm", "float32", 32768, 300), ("hr", "float32", 65536, 200),
                                              ("hr", "float64", 4160, 100), ("pmsm", "float32", 4097, 100),
                                              ("pmsm", "float32", 140001, 40)])
def test_rollout_noise_producer_equals_steps(gl, system, dtype, n, K):
    """Rollout of a system with process noise: the default (each step draws its normals),
    the opt-in noise-producer wave (variant bit 1<<25, one-wave groups only: a second wave
    per group draws the normals ahead into an LDS ring, k_rollout_np, lz_kernels.hip --
    reported as 2 waves per group) and the software-pipelined draws (variant bit 1<<26,
    kZN: the next step's normals drawn in registers during this step) each equal K lz_step
    calls (which draw their own) bit for bit: obs, reward, done, the compact done list and
    the final state; ragged sizes run the last group without a producer; 140,001 envs run
    the 256-lane kernel."""
    from gym_lorenz import _native as nat

    one_wave = n < 131072
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    for variant in ((0, 1 << 25, 1 << 26) if one_wave else (0, 1 << 26)):
        a_be = gl.BatchedEnv(system, n, dtype=dtype, seed=9, max_episode_steps=37, add_noise=True, variant=variant)
        b_be = gl.BatchedEnv(system, n, dtype=dtype, seed=9, max_episode_steps=37, add_noise=True)
        sh = nat.launch_shape(a_be._h, nat.CALL_ROLLOUT)
        # (PMSM at 2 < 32-env waves per CU <= 4 defaults to the lane-pair kernel,
        # test_gpu_rollout_pair.py)
        pair = system == "pmsm" and variant == 0 and 2 * cus < (n + 31) // 32 <= 4 * cus
        assert sh["kernel"] == ("rollout_pair" if pair else "rollout_wave" if one_wave else "rollout"), sh
        assert sh["waves"] == (2 if variant == 1 << 25 else 1 if one_wave or pair else 4), sh
        a_be.reset()
        b_be.reset()
        A = torch.from_numpy(np.random.default_rng(5).uniform(-1.2, 1.2, (K, n, a_be.action_dim))
                             .astype(np.float32)).cuda()
        obs, rew, done, (didx, tobs, nd) = a_be.rollout(A, capture_terminal=K * n)
        want_idx = []
        for k in range(K):
            o, r, d = b_be.step(A[k])
            assert bits_equal(_np(obs[k]), _np(o)), (variant, k)
            assert bits_equal(_np(rew[k]), _np(r)), (variant, k)
            assert np.array_equal(_np(done[k]), _np(d)), (variant, k)
            want_idx.append(k * n + np.nonzero(_np(d))[0])
        m = int(nd.item())
        wi = np.concatenate(want_idx)
        assert m == wi.size and m > 0
        assert np.array_equal(np.sort(_np(didx[:m])), wi)
        for p in range(a_be.info.n_planes):
            assert bits_equal(_np(a_be.get_state(p)), _np(b_be.get_state(p))), (variant, p)
        a_be.close()
        b_be.close()


@pytest.mark.parametrize("system,dtype", [("lorenz3", "float32"), ("pmsm", "float32"),
                                          ("lorenz4", "float64"), ("hr", "float32")])
@pytest.mark.parametrize("n", [2016, 1000])
def test_rollout_split_lanes_bitexact(gl, system, dtype, n):
    """Small-N rollout with two lanes per env (variant bit 512, the default up to 65,536
    envs) == one lane per env (bit 256): outputs, final state and compact done list
    (full one-wave groups at n=2016, a ragged last group at n=1000)."""
    K = 40
    kw = {"add_noise": True} if system in ("pmsm", "hr") else {}
    res = []
    A = None
    for var in (256, 512):
        be = gl.BatchedEnv(system, n, dtype=dtype, seed=6, max_episode_steps=7, variant=var, **kw)
        if A is None:
            A = torch.from_numpy(np.random.default_rng(9).uniform(
                -1.5, 1.5, (K, n, be.action_dim)).astype(np.float32)).cuda()
        be.reset()
        be.rollout(A[:3])  # warm state (both kernels from the same start)
        out = be.rollout(A, capture_terminal=K * n)
        obs, rew, done, (didx, tobs, nd) = out
        m = int(nd.item())
        order = torch.argsort(didx[:m])
        st = [_np(be.get_state(p)) for p in range(be.info.n_planes)]
        res.append((_np(obs), _np(rew), _np(done), _np(didx[:m][order]), _np(tobs[:m][order]), st))
    (o1, r1, d1, i1, t1, s1), (o2, r2, d2, i2, t2, s2) = res
    assert bits_equal(o1, o2) and bits_equal(r1, r2) and np.array_equal(d1, d2)
    assert len(i1) > 0 and np.array_equal(i1, i2) and bits_equal(t1, t2)
    for a, b in zip(s1, s2):
        assert bits_equal(a, b)


def test_l3_1m_envs_vs_oracle(gl, orc):
    """BASELINE size: 1,048,576 envs, 30 fp32 steps, bit-exact on the whole batch."""
    n, T = 1 << 20, 30
    be = gl.BatchedEnv("lorenz3", n, dtype="float32", seed=0, autoreset=False)
    be.reset()
    st = orc.reset_draw("l3", np.float32, n, 0, 0, 0)
    A = np.random.default_rng(0).uniform(-1, 1, (T, n, 3)).astype(np.float32)
    At = torch.from_numpy(A).cuda()
    with np.errstate(all="ignore"):
        for k in range(T):
            o, r, _ = be.step(At[k])
            oo, rr = orc.l3_step(st, A[k])
    assert bits_equal(_np(o), oo) and bits_equal(_np(r), rr)


# ----------------------------------------------------------------- drop-in classes
def test_dropin_dynamic_reproduces_reference(gl):
    """gym_lorenz.envs.LorenzDynamicEnv with the reference's np.random seeding gives
    the reference's exact obs0 and trajectory (fp64)."""
    g = golden("l3")
    for i in (0, 5, 11):
        np.random.seed(int(g["seeds"][i]))
        env = gl.LorenzDynamicEnv()
        o = env.reset()
        assert o.dtype == np.float64 and bits_equal(o, g["obs0"][i])
        for k in range(200):
            o, r, d, info = env.step(g["actions"][i, k])
            assert bits_equal(o, g["obs"][i, k]) and bits_equal(r, g["reward"][i, k])
            assert d is False and info == {}
        env.close()


def test_dropin_pmsm_reproduces_reference(gl):
    g = golden("pmsm")
    for i in (0, 2):
        env = gl.make("lorenz_pmsm-v0", alpha=float(g["alpha"][i]), add_noise=bool(g["add_noise"][i]))
        o, info = env.reset(seed=int(g["seeds"][i]))
        assert o.dtype == np.float32 and bits_equal(o, g["obs0"][i, 0])
        for k in range(300):
            o, r, te, tr, _ = env.step(g["actions"][i, k])
            assert bits_equal(o, g["obs"][i, k]), k
            assert abs(r - g["reward"][i, k]) <= 1e-5 * abs(g["reward"][i, k])
        env.close()


def test_dropin_hr_close_to_reference(gl):
    g = golden("hr")
    for i in (0, 4):
        np.random.seed(10 + i)
        env = gl.HRSyncEnv(add_noise=bool(g["add_noise"][i]), eval_mode=bool(g["eval_mode"][i]),
                           add_filter=bool(g["add_filter"][i]))
        o, _ = env.reset(seed=10 + i)
        assert bits_equal(o, g["obs0"][i])
        for k in range(300):
            o, r, te, tr, _ = env.step(g["actions"][i, k])
        np.testing.assert_allclose(o, g["obs"][i, 299], rtol=1e-6, atol=1e-7)
        env.close()


def test_dropin_l4_reproduces_reference(gl):
    g = golden("l4")
    np.random.seed(100)
    env = gl.make("lorenz_transient-v0")
    o = env.reset()
    assert bits_equal(o, g["obs0"][0])
    for k in range(100):
        o, r, d, info = env.step(g["actions"][0, k])
    assert bits_equal(o, g["obs"][0, 99])
    m, s = env.unwrapped.get_current()
    assert np.isfinite(m) and np.isfinite(s)
    env.close()


# ----------------------------------------------------------------- VecEnv
def test_vecenv_sb3_contract(gl):
    n = 4096
    venv = gl.make_vec("lorenz_pmsm-v0", n, seed=1)
    obs = venv.reset()
    assert obs.shape == (n, 6) and obs.dtype == np.float32
    a = np.zeros((n, 2), np.float32)
    for k in range(2000):
        obs, rew, dones, infos = venv.step(a)
    assert obs.shape == (n, 6) and rew.dtype == np.float32 and dones.dtype == bool
    assert dones.all()  # PMSM truncates at 2000 steps
    i0 = infos[0]
    assert i0["TimeLimit.truncated"] is True and i0["terminal_observation"].shape == (6,)
    assert len(venv.get_attr("lambda_coef")) == n
    venv.close()


@pytest.mark.parametrize("add_filter", [False, True])
def test_hr_f32_vs_oracle(gl, orc, add_filter):
    """HR in fp32 (the VecEnv default): device RK4 == the oracle's fp32 DEV restatement,
    injected noise, filter on/off, 300 steps, 2048 envs."""
    n, T = 2048, 300
    be = gl.BatchedEnv("hr", n, dtype="float32", seed=21, add_noise=True, add_filter=add_filter,
                       autoreset=False)
    be.reset()
    init = orc.reset_draw("hr", np.float32, n, 0, 21, 0, add_noise=True)
    assert bits_equal(_planes(be, 0, 7), init)
    st = np.ascontiguousarray(init[:, :6])
    fa = np.zeros((n, 2), np.float32)
    rng = np.random.default_rng(8)
    with np.errstate(all="ignore"):
        for k in range(T):
            a = rng.uniform(-1.2, 1.2, (n, 2)).astype(np.float32)
            nz = rng.normal(0, 1, (n, 3)) * init[:, 6:7]
            o, r, d = be.step(torch.from_numpy(a), torch.from_numpy(nz))
            oo, rr, tt = orc.hr_step(st, fa, a, nz.astype(np.float32), True, add_filter, orc.DEV)
    assert bits_equal(_np(o), oo) and bits_equal(_np(r), rr)
    assert np.array_equal((_np(d) & 1).astype(bool), tt)


def test_device_noise_statistics(gl, orc):
    """On-device Philox/Box-Muller process noise: PMSM N(0,3) enters the slave's Euler
    update (lorenz_env_try_pmsm.py:80-93), so (state2_device - state2_noiseless)/dt
    recovers the noise up to f32 rounding (~0.03 abs); its moments must be N(0, 3),
    independent across components."""
    n = 1 << 18
    be = gl.BatchedEnv("pmsm", n, seed=3, add_noise=True, autoreset=False)
    be.reset()
    S = orc.PmsmState(n)
    S.st[:] = orc.reset_draw("pmsm", np.float32, n, 0, 3, 0)
    a = np.zeros((n, 2), np.float32)
    be.step(torch.from_numpy(a))
    orc.pmsm_step(S, a, None, False, 0.5, orc.DEV)
    s2 = _planes(be, 3, 3).astype(np.float64)
    nz = (s2 - S.st[:, 3:].astype(np.float64)) / 1e-3
    assert abs(nz.mean()) < 0.03 and abs(nz.std() - 3.0) < 0.03
    c = np.corrcoef(nz.T)
    assert np.abs(c - np.eye(3)).max() < 0.01
    # the master is noiseless (lorenz_env_try_pmsm.py:88)
    assert bits_equal(_planes(be, 0, 3), S.st[:, :3])


# ----------------------------------------------------------------- VecNormalize (f1)
@pytest.mark.parametrize("norm_reward", [False, True])
def test_device_vecnormalize_matches_sb3_restatement(gl, norm_reward):
    """LorenzVecNormalize (device statistics) vs the NumPy restatement of SB3 2.7.1
    VecNormalize (oracle/sb3_vecnorm.py) fed the raw outputs of an identical env, as
    code/lorenz_pmsm/train.py:170 configures it (norm_obs, clip_obs=10)."""
    from gym_lorenz.vec_normalize import LorenzVecNormalize
    from oracle.sb3_vecnorm import VecNormalizeRef

    n, T = 4096, 120
    raw = gl.make_vec("lorenz_pmsm-v0", n, seed=5, max_episode_steps=37)
    dev = LorenzVecNormalize(gl.make_vec("lorenz_pmsm-v0", n, seed=5, max_episode_steps=37),
                             norm_obs=True, norm_reward=norm_reward, clip_obs=10.0)
    ref = VecNormalizeRef(n, 6, norm_obs=True, norm_reward=norm_reward, clip_obs=10.0)
    o_raw = raw.reset()
    o_ref = ref.reset(o_raw)
    o_dev = dev.reset()
    np.testing.assert_allclose(o_dev, o_ref, rtol=1e-5, atol=1e-5)
    rng = np.random.default_rng(0)
    saw_done = False
    for k in range(T):
        a = rng.uniform(-1, 1, (n, 2)).astype(np.float32)
        o_raw, r_raw, d_raw, i_raw = raw.step(a)
        term = {i: i_raw[i]["terminal_observation"] for i in range(n) if d_raw[i]}
        o_ref, r_ref, d_ref, tn_ref = ref.step(o_raw, r_raw, d_raw, term)
        o_dev, r_dev, d_dev, i_dev = dev.step(a)
        assert np.array_equal(d_dev, d_raw)
        np.testing.assert_allclose(o_dev, o_ref, rtol=2e-5, atol=2e-5)
        np.testing.assert_allclose(r_dev, r_ref, rtol=2e-5, atol=2e-5)
        for i, t in tn_ref.items():
            saw_done = True
            np.testing.assert_allclose(i_dev[i]["terminal_observation"], t, rtol=2e-5, atol=2e-5)
            assert i_dev[i]["TimeLimit.truncated"] == i_raw[i]["TimeLimit.truncated"]
    assert saw_done
    np.testing.assert_allclose(dev.obs_rms.mean, ref.obs_rms.mean, rtol=1e-6, atol=1e-6)
    np.testing.assert_allclose(dev.obs_rms.var, ref.obs_rms.var, rtol=1e-6)
    assert dev.obs_rms.count == pytest.approx(ref.obs_rms.count)
    np.testing.assert_allclose(dev.ret_rms.var, ref.ret_rms.var, rtol=1e-6)
    dev.save("/tmp/_vn.npz")
    dev2 = LorenzVecNormalize(gl.make_vec("lorenz_pmsm-v0", 16, seed=1))
    dev2.load("/tmp/_vn.npz")
    np.testing.assert_array_equal(dev2.obs_rms.mean, dev.obs_rms.mean)


def test_vecenv_return_tensors_matches_numpy(gl):
    """The sync-free device-tensor VecEnv path (DeviceLazyInfos) returns what the NumPy
    path returns: obs / rewards / dones and, for done envs, terminal_observation and
    TimeLimit.truncated."""
    n = 3000
    va = gl.make_vec("lorenz_pmsm-v0", n, return_tensors=True, max_episode_steps=4, seed=5)
    vb = gl.make_vec("lorenz_pmsm-v0", n, max_episode_steps=4, seed=5)
    assert np.array_equal(_np(va.reset()), vb.reset())
    rng = np.random.default_rng(0)
    seen = 0
    for k in range(9):
        a = rng.uniform(-1, 1, (n, 2)).astype(np.float32)
        oa, ra, da, ia = va.step(torch.from_numpy(a).cuda())
        ob, rb, db, ib = vb.step(a)
        assert np.array_equal(_np(oa), ob) and np.array_equal(_np(ra), rb)
        assert np.array_equal(_np(da), db)
        for i in np.nonzero(db)[0]:
            assert np.array_equal(_np(ia[int(i)]["terminal_observation"]),
                                  ib[int(i)]["terminal_observation"])
            assert ia[int(i)]["TimeLimit.truncated"] == ib[int(i)]["TimeLimit.truncated"]
            seen += 1
        assert len(ia) == n and ia[0] is not None
    assert seen > 0


def test_import_order_gym_lorenz_first():
    """A fresh interpreter that imports gym_lorenz before anything touches torch /
    HIP (the order of a script that starts with `import gym_lorenz`) can create and
    step envs: _native.py loads torch's HIP runtime first."""
    import subprocess
    import sys

    from conftest import ROOT

    code = ("import sys; sys.path.insert(0, %r)\n"
            "import gym_lorenz as gl\n"
            "e = gl.make('lorenz_dynamic-v0'); o = e.reset(); o2 = e.step([0.0, 0.0, 0.0])[0]\n"
            "assert o.shape == (6,) and o2.shape == (6,)\n"
            "print('ok')\n" % (ROOT + "/gym-lorenz_amd"))
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and "ok" in r.stdout, r.stderr[-2000:]
