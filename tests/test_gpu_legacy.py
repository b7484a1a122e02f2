"""GPU parity of the legacy, unregistered variants:
lorenz_env_transient1.py (T1), lorenz_env_transient2.py (T2),
lorenz_env_transient_pmsm.py (TP), lorenz_singlecontrol.py (SC).

  * fp64: observations and states bit-exact vs the reference's own trajectories
    (tests/golden/legacy.npz) every step; rewards bit-exact for T1 / SC; T2 / TP
    rewards (-S - S**(1/3), -S - S**(1/10)) within 1e-14 relative -- the GPU's pow is
    OCML's, not glibc's (both faithful, neither always correctly rounded); dones equal.
  * fp32: bit-exact vs the oracle's f32 restatement (same rule for the pow rewards).
  * on-device reset draws == the oracle's Philox restatement; fused rollout == steps.
"""
import numpy as np
import pytest
import torch

from conftest import bits_equal, golden

pytestmark = pytest.mark.gpu

NAMES = {"t1": "transient1", "t2": "transient2", "tp": "transient_pmsm", "sc": "singlecontrol"}
POW_REWARD = ("t2", "tp")


@pytest.fixture(scope="module")
def gl():
    import gym_lorenz

    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    return gym_lorenz


def _np(t):
    return t.detach().cpu().numpy()


def _rew_ok(key, got, want):
    if key in POW_REWARD:
        fin = np.isfinite(want)
        if not np.array_equal(fin, np.isfinite(got)):
            return False
        return np.allclose(got[fin], want[fin], rtol=1e-14, atol=0)
    return bits_equal(got, want)


@pytest.mark.parametrize("key", ["t1", "t2", "tp", "sc"])
def test_legacy_f64_golden(gl, key):
    g = golden("legacy")
    init = g[key + "_init"]
    n, T = init.shape[0], g[key + "_obs"].shape[1]
    be = gl.BatchedEnv(NAMES[key], n, dtype="float64", autoreset=False)
    assert bits_equal(_np(be.reset(init=torch.from_numpy(np.ascontiguousarray(init)))),
                      g[key + "_obs0"])
    A = be.action_dim
    acts = torch.from_numpy(np.ascontiguousarray(g[key + "_actions"][:, :, :A].transpose(1, 0, 2)))
    noise = torch.from_numpy(np.ascontiguousarray(g[key + "_noise"].transpose(1, 0, 2))).cuda()
    acts = acts.cuda() if key != "sc" else torch.zeros((T, n, A), device="cuda")
    for k in range(T):
        nz = noise[k] if key in ("tp", "sc") else None
        o, r, d = be.step(acts[k].contiguous(), nz)
        assert bits_equal(_np(o), g[key + "_obs"][:, k]), k
        assert _rew_ok(key, _np(r), g[key + "_reward"][:, k]), k
        assert np.array_equal(_np(d) & 1 != 0, g[key + "_done"][:, k]), k


@pytest.mark.parametrize("key", ["t1", "t2", "tp", "sc"])
def test_legacy_f32_vs_oracle_and_reset_draws(gl, orc, key):
    n, T = 1000, 50
    be = gl.BatchedEnv(NAMES[key], n, dtype="float32", seed=7, autoreset=False)
    obs0 = _np(be.reset())
    st = orc.reset_draw(key, np.float32, n, 0, 7, 0)
    # the device's initial states are the oracle's Philox draws
    planes = np.stack([_np(be.get_state(j)) for j in range(st.shape[1])], 1)
    assert bits_equal(planes, st)
    assert bits_equal(obs0, orc.legacy_reset_obs(key, st))
    rng = np.random.default_rng(3)
    A = be.action_dim
    for k in range(T):
        a = rng.uniform(-1.5, 1.5, (n, A)).astype(np.float32)
        nz = rng.normal(0, 3, (n, 3)) if key in ("tp", "sc") else None
        o, r, d = be.step(torch.from_numpy(a).cuda(),
                          None if nz is None else torch.from_numpy(nz).cuda())
        with np.errstate(all="ignore"):
            oo, rr, dd = orc.legacy_step(key, st, None if key == "sc" else a, nz)
        assert bits_equal(_np(o), oo), k
        if key in POW_REWARD:
            np.testing.assert_allclose(_np(r), rr, rtol=1e-6)
        else:
            assert bits_equal(_np(r), rr), k
        assert np.array_equal(_np(d) & 1 != 0, dd), k


@pytest.mark.parametrize("n", [777, 140001])  # one-wave kernel; 256-lane, ragged
@pytest.mark.parametrize("key", ["t1", "t2", "tp", "sc"])
def test_legacy_rollout_equals_steps(gl, key, n):
    K = 20
    a = gl.BatchedEnv(NAMES[key], n, seed=5, max_episode_steps=6)
    b = gl.BatchedEnv(NAMES[key], n, seed=5, max_episode_steps=6)
    a.reset()
    b.reset()
    acts = (torch.rand((K, n, a.action_dim), device="cuda") * 2 - 1).contiguous()
    obs, rew, done = a.rollout(acts)
    for k in range(K):
        o, r, d = b.step(acts[k].contiguous())
        assert bits_equal(_np(o), _np(obs[k])), k
        assert bits_equal(_np(r), _np(rew[k])), k
        assert np.array_equal(_np(d), _np(done[k])), k
    assert (_np(done) & 2).any()  # TimeLimit truncation + auto-reset exercised
