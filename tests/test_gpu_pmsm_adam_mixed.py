"""GPU: PMSM's Adam bias correction when the envs of one wavefront are at DIFFERENT Adam
steps (lorenz_env_try_pmsm.py:121-131: k counts every step and is never reset, so a
batch whose envs were set or created apart carries mixed k).  The kernel loads the
(1 - beta1**k, 1 - beta2**k) pair for the wave's first lane's k with one scalar load and
falls back to a per-step waterfall only when the wave's k differ (SysPMSM::bias_pair);
this drives that fallback -- k mixed within every wave, around the table's end and far
past it (1.0 there) -- through the per-step kernel and both fused rollout kernels, bit
for bit against the oracle (obs, reward, lambda / m / v, k)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

K = 32


def _nan_eq(a, b):
    an, bn = np.isnan(a), np.isnan(b)
    if not np.array_equal(an, bn):
        return False
    return bool(((a.view(np.uint32) == b.view(np.uint32)) | an).all())


def _adam_start(n, rng):
    k = rng.integers(0, 400, n)
    # runs of equal k (uniform waves) next to mixed ones; some around the table's end
    # (1 - 0.999**k reaches 1.0f near k = 17,000) and far past it
    k[: n // 4] = 7
    sel = rng.random(n) < 0.2
    k[sel] = rng.integers(16500, 17600, int(sel.sum()))
    sel = rng.random(n) < 0.05
    k[sel] = rng.integers(40000, 1 << 30, int(sel.sum()))
    return k.astype(np.int32)


@pytest.mark.parametrize("n,mode", [(4099, "step"), (4099, "rollout"), (32768, "rollout"),
                                    (70001, "rollout")])
def test_pmsm_mixed_adam_steps_bitexact(orc, n, mode):
    import gym_lorenz as gl

    nat = gl._native
    seed = 57
    rng = np.random.default_rng(n)
    be = gl.BatchedEnv("pmsm", n, dtype="float32", seed=seed)
    be.reset()
    k0 = _adam_start(n, rng)
    be.set_state(nat.PMSM_ADAM_STEP, torch.from_numpy(k0))
    S = orc.PmsmState(n)
    S.st[:] = orc.reset_draw("pmsm", np.float32, n, 0, seed, 0)
    S.adam_step[:] = k0
    A = torch.from_numpy(rng.uniform(-1.2, 1.2, (K, n, 2)).astype(np.float32)).to(be.device)
    if mode == "rollout":
        obs, rew, done = be.rollout(A)
        torch.cuda.synchronize()
        got = [(obs[k].cpu().numpy(), rew[k].cpu().numpy(), done[k].cpu().numpy()) for k in range(K)]
    else:
        got = []
        for k in range(K):
            o, r, d = be.step(A[k])
            got.append((o.cpu().numpy().copy(), r.cpu().numpy().copy(), d.cpu().numpy().copy()))
    bad = []
    with np.errstate(all="ignore"):
        for k in range(K):
            oo, rr, te, tr = orc.pmsm_step(S, A[k].cpu().numpy(), None, False, 0.5, orc.DEV)
            assert not te.any() and not tr.any()  # no resets in this window: a pure Adam check
            go, gr, gd = got[k]
            if not _nan_eq(go, oo):
                bad.append((k, "obs"))
            if not _nan_eq(gr, rr):
                bad.append((k, "reward"))
            if gd.any():
                bad.append((k, "done"))
            assert len(bad) < 5, bad
    assert not bad, bad
    assert _nan_eq(be.get_state(nat.PMSM_LAMBDA).cpu().numpy(), S.lam)
    assert _nan_eq(be.get_state(nat.PMSM_M).cpu().numpy(), S.m)
    assert _nan_eq(be.get_state(nat.PMSM_V).cpu().numpy(), S.v)
    assert np.array_equal(be.get_state(nat.PMSM_ADAM_STEP).cpu().numpy(), S.adam_step)
    assert np.array_equal(S.adam_step, k0 + K)
    be.close()
