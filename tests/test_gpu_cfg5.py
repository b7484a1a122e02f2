"""BASELINE cfg5 at its own size: the 2,048-step fused rollout (lz_rollout) against
K = 2048 oracle steps, bit for bit.

  * LORENZ3 f32, 32,768 envs (cfg5's per-GPU batch): the two-lanes-per-env
    k_rollout_split path (DMA prologue, vmcnt ladder, steady-state loop);
  * LORENZ3 f32, 262,144 envs (cfg5's whole batch on one GPU): the 256-lane k_rollout
    path;
  * PMSM f32 (noise off), 32,768 envs: the one-wave k_rollout path with the Adam dual
    and PMSM's own 2000-step truncation.

Every env starts at a random position of its episode (the step plane is set per env),
so TimeLimit truncations -- and the auto-resets, compact done list (capture_terminal)
and terminal observations they produce -- are spread over the whole 2048 steps.
Reference: dynamic.py:61-90 (LORENZ3 step), lorenz_env_try_pmsm.py:76-184 (PMSM step),
SB3 DummyVecEnv auto-reset; BASELINE.json configs[4].
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

K = 2048


@pytest.fixture(scope="module")
def gl():
    import gym_lorenz

    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    return gym_lorenz


def _nan_eq(a, b):
    """Bitwise equality where any NaN matches any NaN (host NaN payloads differ)."""
    an, bn = np.isnan(a), np.isnan(b)
    if not np.array_equal(an, bn):
        return False
    ia, ib = a.view(np.uint32), b.view(np.uint32)
    return bool(((ia == ib) | an).all())


def _run(gl, orc, system, n, L, seed, lo, hi):
    nat = gl._native
    plane = nat.L3_STEP if system == "lorenz3" else nat.PMSM_STEP
    be = gl.BatchedEnv(system, n, dtype="float32", seed=seed, max_episode_steps=L)
    be.reset()
    o_name = "l3" if system == "lorenz3" else "pmsm"
    rng = np.random.default_rng(seed)
    steps = rng.integers(0, L, n).astype(np.int32)
    be.set_state(plane, torch.from_numpy(steps))
    if system == "lorenz3":
        st = orc.reset_draw("l3", np.float32, n, 0, seed, 0).copy()
    else:
        S = orc.PmsmState(n)
        S.st[:] = orc.reset_draw("pmsm", np.float32, n, 0, seed, 0)
        S.cur_step[:] = steps
    gen = torch.Generator(device=be.device)
    gen.manual_seed(seed)
    A = (torch.rand((K, n, be.action_dim), generator=gen, device=be.device) * (hi - lo) + lo)
    cap = n * (K // L + 2)
    obs, rew, done, (didx, tobs, nd) = be.rollout(A, capture_terminal=cap)
    torch.cuda.synchronize()
    exp_idx, exp_term = [], []
    gids = np.arange(n, dtype=np.int64)
    bad = []
    with np.errstate(all="ignore"):
        for k in range(K):
            a = A[k].cpu().numpy()
            if system == "lorenz3":
                oo, rr = orc.l3_step(st, a)
                steps += 1
                te = np.zeros(n, bool)
                tr = steps >= L
            else:
                oo, rr, te, tr = orc.pmsm_step(S, a, None, False, 0.5, orc.DEV)
                steps = S.cur_step
            code = te.astype(np.uint8) | (tr.astype(np.uint8) << 1)
            fin = code != 0
            go = obs[k].cpu().numpy()
            if not np.array_equal(done[k].cpu().numpy(), code):
                bad.append((k, "done"))
            if not _nan_eq(rew[k].cpu().numpy(), rr):
                bad.append((k, "reward"))
            if fin.any():
                ids = gids[fin]
                exp_idx.append(k * n + ids)
                exp_term.append(oo[fin])
                fresh = orc.reset_draw_idx(o_name, np.float32, ids, seed, 1 + k)
                if system == "lorenz3":
                    st[fin] = fresh
                    steps[fin] = 0
                    oo[fin] = orc.l3_reset_obs(fresh)
                else:
                    S.st[fin] = fresh
                    S.cur_step[fin] = 0
                    oo[fin] = orc.pmsm_reset_obs(fresh)
            if not _nan_eq(go, oo):
                bad.append((k, "obs"))
            assert len(bad) < 5, bad
    assert not bad, bad
    # compact done list: exactly the (k, env) pairs that finished, with pre-reset obs
    m = int(nd.item())
    exp_idx = np.concatenate(exp_idx)
    exp_term = np.concatenate(exp_term)
    assert m == exp_idx.size and m > n // 2, (m, exp_idx.size)
    order = torch.argsort(didx[:m])
    got_idx = didx[:m][order].cpu().numpy()
    assert np.array_equal(got_idx, exp_idx)  # exp_idx is ascending (k-major, env-minor)
    assert _nan_eq(tobs[:m][order].cpu().numpy(), exp_term)
    # state after the rollout (the kernel wrote the VGPR-resident state back)
    assert np.array_equal(be.get_state(plane).cpu().numpy(), steps)
    if system == "lorenz3":
        got = np.stack([be.get_state(j).cpu().numpy() for j in range(3)], axis=1)
        assert _nan_eq(got, st)
    else:
        got = np.stack([be.get_state(j).cpu().numpy() for j in range(6)], axis=1)
        assert _nan_eq(got, S.st)
        assert _nan_eq(be.get_state(nat.PMSM_LAMBDA).cpu().numpy(), S.lam)
        assert np.array_equal(be.get_state(nat.PMSM_ADAM_STEP).cpu().numpy(), S.adam_step)
    be.close()


@pytest.mark.parametrize("n", [32768, 262144])
def test_cfg5_l3_rollout_k2048_bitexact(gl, orc, n):
    """LORENZ3 f32, K = 2048, TimeLimit 300 with ragged episode starts (every env
    truncates ~7 times at its own steps)."""
    _run(gl, orc, "lorenz3", n, L=300, seed=31, lo=-1.5, hi=1.5)


def test_cfg5_pmsm_rollout_k2048_bitexact(gl, orc):
    """PMSM f32 (noise off), K = 2048 at 32,768 envs: PMSM's own 2000-step truncation
    from ragged starts, actions U(-1.2, 1.2) (exercising the [-1, 1] clip), Adam dual
    carried across the auto-resets."""
    _run(gl, orc, "pmsm", 32768, L=2000, seed=32, lo=-1.2, hi=1.2)


@pytest.mark.parametrize("n", [32768, 40001, 65536, 100003, 262144])
def test_cfg5_l3_rollout_no_timelimit_bitexact(gl, orc, n):
    """The bench's cfg5 workload as dynamic.py runs it: no TimeLimit, and the
    reference's own done (t == 10) never fires -- the launch takes the kernel without
    done bookkeeping (kNoDone).  K = 2048 oracle steps bit for bit, every done byte 0,
    the final state; and the same bits as the general kernel (variant bit 2048).
    n = 40,001 adds a ragged last workgroup (the non-DMA path of the same kernel);
    65,536 (= 256 x CUs: the first size on the 256-lane kernel since round 3), 100,003
    (its ragged last workgroup) and 262,144 run the 256-lane k_rollout path."""
    seed = 41
    gen = torch.Generator(device="cuda")
    gen.manual_seed(seed)
    A = torch.rand((K, n, 3), generator=gen, device="cuda") * 3 - 1.5
    res = []
    for var in (0, 2048):
        be = gl.BatchedEnv("lorenz3", n, dtype="float32", seed=seed, variant=var)
        be.reset()
        obs, rew, done = be.rollout(A)
        torch.cuda.synchronize()
        res.append((obs, rew, done, np.stack([be.get_state(j).cpu().numpy() for j in range(3)], 1)))
        be.close()
    (o0, r0, d0, s0), (o1, r1, d1, s1) = res
    assert torch.equal(d0, d1) and int(d0.count_nonzero()) == 0
    assert _nan_eq(s0, s1)
    st = orc.reset_draw("l3", np.float32, n, 0, seed, 0).copy()
    bad = []
    with np.errstate(all="ignore"):
        for k in range(K):
            oo, rr = orc.l3_step(st, A[k].cpu().numpy())
            for tag, got, other, want in (("obs", o0[k], o1[k], oo), ("reward", r0[k], r1[k], rr)):
                g = got.cpu().numpy()
                if not (_nan_eq(g, want) and _nan_eq(other.cpu().numpy(), g)):
                    bad.append((k, tag))
            assert len(bad) < 5, bad
    assert not bad, bad
    assert _nan_eq(s0, st)