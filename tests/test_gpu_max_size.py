"""Maximum sizes: LORENZ3 float32 at 720,000,001 envs, so that every index the kernels
form crosses the 32-bit lines -- an obs element index i * 6 passes 2^31 (env 357,913,942)
and 2^32 (env 715,827,883), a state plane's byte offset passes 2^31 (env 536,870,912), the
obs buffer is 17.3 GB -- and N is odd (the ragged, non-vector staging path).

A sample of envs (both ends, each crossing, random ids) runs through the oracle on its own
global ids (the Philox draws are keyed by (seed, global env id, tick), so a subset
reproduces exactly) and must match bit for bit: obs, reward, done bytes and, for the
sampled envs that finish, their terminal obs in the compact done list.  Over ALL envs the
done bytes and the done list's ids must equal the TimeLimit schedule computed on the
device from the step counters.  The same for one K = 2 fused rollout, and PMSM (eleven
state planes, Adam dual variable) at 536,870,913 envs, where each float32 plane passes 2 GiB.

Reference: dynamic.py:61-90 (step), gymnasium TimeLimit + SB3 DummyVecEnv auto-reset
(SURVEY §8)."""
import numpy as np
import pytest
import torch

from conftest import bits_equal
from oracle_tl import OracleTL

pytestmark = [pytest.mark.gpu, pytest.mark.filterwarnings("ignore::RuntimeWarning")]

N = 720_000_001
L = 3
CROSS = (357_913_941, 536_870_911, 715_827_882)


@pytest.fixture(scope="module")
def gl():
    import gym_lorenz

    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    free, _ = torch.cuda.mem_get_info()
    if free < 160 * 2**30:  # an MI355X has 288 GB; a smaller or shared card cannot hold these
        pytest.skip(f"the max-size cases need ~160 GiB of HBM free ({free / 2**30:.0f} GiB)")
    return gym_lorenz


def _sample():
    rng = np.random.default_rng(5)
    parts = [np.arange(0, 1024), np.arange(N - 1024, N), rng.integers(0, N, 2048)]
    parts += [np.arange(c - 256, c + 256) for c in CROSS]
    return np.unique(np.concatenate(parts)).astype(np.int64)


def _free():
    torch.cuda.synchronize()
    torch.cuda.empty_cache()


def test_step_max_size_vs_oracle(gl):
    import oracle as orc
    from gym_lorenz import _native as nat

    gids = _sample()
    gd = torch.from_numpy(gids).cuda()
    be = gl.BatchedEnv("lorenz3", N, dtype="float32", seed=17, max_episode_steps=L)
    be.reset()
    g = torch.Generator(device="cuda").manual_seed(17)
    steps = torch.randint(0, L, (N,), dtype=torch.int32, device="cuda", generator=g)
    be.set_state(nat.L3_STEP, steps)
    ref = OracleTL(orc, "l3", np.float32, gids.size, 17, L, steps[gd].cpu().numpy(), gids=gids)
    for k in range(4):
        a = torch.rand((N, 3), dtype=torch.float32, device="cuda", generator=g).mul_(2.0).sub_(1.0)
        a[gd[::7]] *= 900.0  # some sampled envs at the +-500 action clip
        o, r, d = be.step(a)
        oo, rr, dd, idx, term = ref.step(a[gd].cpu().numpy())
        assert bits_equal(o[gd].cpu().numpy(), oo), k
        assert bits_equal(r[gd].cpu().numpy(), rr), k
        assert np.array_equal(d[gd].cpu().numpy(), dd), k
        # every env: the TimeLimit schedule (LORENZ3 never terminates on its own)
        steps += 1
        due = steps >= L
        steps[due] = 0
        assert torch.equal(d, due.to(torch.uint8) << 1), k
        del a
        di, dt = be.done_list()
        assert torch.equal(di, torch.nonzero(due).squeeze(1)), k
        if idx.size:  # the sampled finishers' terminal obs, found in the sorted list
            pos = torch.searchsorted(di, torch.from_numpy(gids[idx]).cuda())
            assert bits_equal(dt[pos].cpu().numpy(), term), k
        del di, dt, due
    for p in range(3):
        assert bits_equal(be.get_state(p, gd).cpu().numpy(), ref.st[:, p])
    assert torch.equal(be.get_state(nat.L3_STEP), steps)
    be.close()
    del be, steps
    _free()


def test_rollout_max_size_vs_oracle(gl):
    import oracle as orc
    from gym_lorenz import _native as nat

    K = 2
    gids = _sample()
    gd = torch.from_numpy(gids).cuda()
    be = gl.BatchedEnv("lorenz3", N, dtype="float32", seed=23, max_episode_steps=L)
    be.reset()
    g = torch.Generator(device="cuda").manual_seed(23)
    steps = torch.randint(0, L, (N,), dtype=torch.int32, device="cuda", generator=g)
    be.set_state(nat.L3_STEP, steps)
    ref = OracleTL(orc, "l3", np.float32, gids.size, 23, L, steps[gd].cpu().numpy(), gids=gids)
    a = torch.rand((K, N, 3), dtype=torch.float32, device="cuda", generator=g).mul_(2.0).sub_(1.0)
    obs, rew, done = be.rollout(a)
    for k in range(K):
        oo, rr, dd, _, _ = ref.step(a[k][gd].cpu().numpy())
        assert bits_equal(obs[k][gd].cpu().numpy(), oo), k
        assert bits_equal(rew[k][gd].cpu().numpy(), rr), k
        assert np.array_equal(done[k][gd].cpu().numpy(), dd), k
        steps += 1
        due = steps >= L
        steps[due] = 0
        assert torch.equal(done[k], due.to(torch.uint8) << 1), k
        del due
    for p in range(3):
        assert bits_equal(be.get_state(p, gd).cpu().numpy(), ref.st[:, p])
    assert torch.equal(be.get_state(nat.L3_STEP), steps)
    be.close()
    del be, steps, a, obs, rew, done
    _free()


def test_pmsm_step_max_size_vs_oracle(gl):
    """PMSM float32 at 536,870,913 envs (every plane's byte offsets pass 2^31), noise off,
    3 steps: the sampled envs' obs, reward, done bits and every state plane vs the
    oracle's DEV restatement, bit for bit."""
    import oracle as orc

    n, T, seed = 536_870_913, 3, 29
    rng = np.random.default_rng(7)
    gids = np.unique(np.concatenate([np.arange(0, 1024), np.arange(n - 1024, n), rng.integers(0, n, 2048),
                                     np.arange((1 << 29) - 512, (1 << 29) + 1)])).astype(np.int64)
    gd = torch.from_numpy(gids).cuda()
    be = gl.BatchedEnv("pmsm", n, seed=seed, autoreset=False)
    be.reset()
    S = orc.PmsmState(gids.size)
    S.st[:] = orc.reset_draw_idx("pmsm", np.float32, gids, seed, 0)
    g = torch.Generator(device="cuda").manual_seed(seed)
    with np.errstate(all="ignore"):
        for k in range(T):
            a = torch.rand((n, 2), dtype=torch.float32, device="cuda", generator=g).mul_(2.4).sub_(1.2)
            o, r, d = be.step(a)
            oo, rr, te, tr = orc.pmsm_step(S, a[gd].cpu().numpy(), None, False, 0.5, orc.DEV)
            assert bits_equal(o[gd].cpu().numpy(), oo), k
            assert bits_equal(r[gd].cpu().numpy(), rr), k
            dd = d[gd].cpu().numpy()
            assert np.array_equal((dd & 1).astype(bool), te) and np.array_equal((dd & 2).astype(bool), tr), k
            del a
    planes = {p: be.get_state(p, gd).cpu().numpy() for p in range(11)}
    assert bits_equal(np.stack([planes[p] for p in range(6)], 1), S.st)
    assert bits_equal(planes[6], S.lam) and bits_equal(planes[7], S.m) and bits_equal(planes[8], S.v)
    assert np.array_equal(planes[9], S.adam_step) and np.array_equal(planes[10], S.cur_step)
    be.close()
    del be
    _free()


def _sample_n(n, seed):
    rng = np.random.default_rng(seed)
    parts = [np.arange(0, 1024), np.arange(n - 1024, n), rng.integers(0, n, 2048)]
    parts += [np.arange(max(0, c - 256), min(n, c + 256)) for c in (1 << 28, 1 << 29, (1 << 31) // 8)]
    return np.unique(np.concatenate(parts)).astype(np.int64)


def test_l4_step_max_size_vs_oracle(gl):
    """LORENZ4 (eight float32 planes, obs 8: element indices pass 2^32 at env 536,870,912)
    at 536,870,913 envs, TimeLimit(3) with staggered counters, 4 steps: the sample vs the
    oracle bit for bit, and the done bytes of every env vs the schedule (its own
    termination, reward < -1e6, cannot fire in 4 steps from the reference's initial
    states: asserted through the oracle's sample)."""
    import oracle as orc
    from gym_lorenz import _native as nat

    n, seed = 536_870_913, 37
    gids = _sample_n(n, 3)
    gd = torch.from_numpy(gids).cuda()
    be = gl.BatchedEnv("lorenz4", n, dtype="float32", seed=seed, max_episode_steps=L)
    be.reset()
    g = torch.Generator(device="cuda").manual_seed(seed)
    steps = torch.randint(0, L, (n,), dtype=torch.int32, device="cuda", generator=g)
    be.set_state(nat.L4_STEP, steps)
    ref = OracleTL(orc, "l4", np.float32, gids.size, seed, L, steps[gd].cpu().numpy(), gids=gids)
    for k in range(4):
        a = torch.rand((n, 3), dtype=torch.float32, device="cuda", generator=g).mul_(2.0).sub_(1.0)
        o, r, d = be.step(a)
        oo, rr, dd, idx, term = ref.step(a[gd].cpu().numpy())
        assert bits_equal(o[gd].cpu().numpy(), oo), k
        assert bits_equal(r[gd].cpu().numpy(), rr), k
        assert np.array_equal(d[gd].cpu().numpy(), dd), k
        assert not (dd & 1).any(), k
        steps += 1
        due = steps >= L
        steps[due] = 0
        assert torch.equal(d, due.to(torch.uint8) << 1), k
        del a, due
    for p in range(8):
        assert bits_equal(be.get_state(p, gd).cpu().numpy(), ref.st[:, p]), p
    be.close()
    del be, steps
    _free()


def test_hr_step_max_size_vs_oracle(gl):
    """Hindmarsh-Rose (RK4 in registers, obs 6) at 400,000,003 envs (odd N; obs element
    indices past 2^31), noise off, 3 steps: the sample's obs, reward, termination bits and
    master / slave planes vs the oracle's DEV restatement, bit for bit."""
    import oracle as orc
    from gym_lorenz import _native as nat

    n, seed = 400_000_003, 41
    gids = _sample_n(n, 4)
    gd = torch.from_numpy(gids).cuda()
    be = gl.BatchedEnv("hr", n, dtype="float32", seed=seed, autoreset=False, add_noise=False)
    be.reset()
    init = orc.reset_draw_idx("hr", np.float32, gids, seed, 0)
    st = np.ascontiguousarray(init[:, :6])
    fa = np.zeros((gids.size, 2), np.float32)
    g = torch.Generator(device="cuda").manual_seed(seed)
    with np.errstate(all="ignore"):
        for k in range(3):
            a = torch.rand((n, 2), dtype=torch.float32, device="cuda", generator=g).mul_(2.4).sub_(1.2)
            o, r, d = be.step(a)
            oo, rr, tt = orc.hr_step(st, fa, a[gd].cpu().numpy(), None, False, False, orc.DEV)
            assert bits_equal(o[gd].cpu().numpy(), oo) and bits_equal(r[gd].cpu().numpy(), rr), k
            assert np.array_equal((d[gd].cpu().numpy() & 1).astype(bool), tt), k
            del a
    got = np.stack([be.get_state(nat.HR_M + j, gd).cpu().numpy() for j in range(6)], 1)
    assert bits_equal(got, st)
    be.close()
    del be
    _free()
