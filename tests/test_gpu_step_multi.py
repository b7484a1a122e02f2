"""GPU parity of the multi-tile step kernel (k_step_multi, lz_kernels.hip): E = 2 or 4
256-env tiles per workgroup with every tile's loads issued at entry must give exactly
the bits of k_step (one tile per workgroup, itself bit-exact vs the oracle in
test_gpu_parity.py) -- obs, reward, done, compact done list + terminal obs, every state
plane -- for PMSM (device noise, Adam dual) and HR float32 (noise, action filter),
with truncation + auto-reset inside the window, ragged last tiles and the trailing
empty tiles of the last workgroup.  Variant bits 14-15 select the tile count
(16384: 1 = k_step, 32768: 2, 49152: 4)."""
import numpy as np
import pytest
import torch

from conftest import bits_equal

pytestmark = pytest.mark.gpu

E1, E2, E4 = 16384, 32768, 49152


@pytest.fixture(scope="module")
def gl():
    import gym_lorenz

    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    return gym_lorenz


def _np(t):
    return t.detach().cpu().numpy()


def _run(gl, system, n, variant, A, kw, noise=None):
    be = gl.BatchedEnv(system, n, dtype="float32", seed=11, max_episode_steps=9, variant=variant, **kw)
    be.reset()
    outs = []
    for k in range(A.shape[0]):
        o, r, d = be.step(A[k], noise=None if noise is None else noise[k])
        idx, tobs = be.done_list()
        outs.append((_np(o), _np(r), _np(d), _np(idx), _np(tobs)))
    st = [_np(be.get_state(p)) for p in range(be.info.n_planes)]
    be.close()
    return outs, st


CASES = [("pmsm", {"add_noise": True}), ("pmsm", {"add_noise": False, "alpha": 0.3}),
         ("hr", {"add_noise": True}), ("hr", {"add_noise": True, "add_filter": True}),
         ("lorenz3", {})]  # LORENZ3 f32: multi-tile only when forced (A/B), 3 actions


@pytest.mark.parametrize("system,kw", CASES, ids=[c[0] + str(i) for i, c in enumerate(CASES)])
@pytest.mark.parametrize("n", [1613, 2048, 70000])
def test_step_multi_equals_step(gl, system, kw, n):
    """n = 1613: 6.3 tiles (E = 4: the second workgroup's trailing tiles are empty, the
    last live one ragged); 2048: whole groups; 70,000: 274 groups, ragged."""
    K = 20
    na = 3 if system == "lorenz3" else 2
    A = torch.from_numpy(np.random.default_rng(5).uniform(-1.3, 1.3, (K, n, na))
                         .astype(np.float32)).cuda()
    ref_out, ref_st = _run(gl, system, n, E1, A, kw)
    assert sum(len(x[3]) for x in ref_out) > 0  # truncations happened inside the window
    for var in (E2, E4):
        out, st = _run(gl, system, n, var, A, kw)
        for k in range(K):
            for a, b in zip(ref_out[k], out[k]):
                assert a.shape == b.shape and bits_equal(a, b), (var, k)
        for a, b in zip(ref_st, st):
            assert bits_equal(a, b), var


def test_step_multi_misaligned_actions(gl):
    """Actions whose base is not 16-B aligned (vec_ok = 0): the scalar action loads."""
    n, K = 3000, 6
    base = torch.from_numpy(np.random.default_rng(8).uniform(-1, 1, (K, n * 2 + 1))
                            .astype(np.float32)).cuda()
    A = base[:, 1:].reshape(K, n, 2)  # offset by 4 B
    res = [_run(gl, "pmsm", n, var, A, {"add_noise": True}) for var in (E1, E4)]
    for k in range(K):
        for a, b in zip(res[0][0][k], res[1][0][k]):
            assert bits_equal(a, b), k


def test_step_multi_injected_noise(gl):
    """Injected (caller-supplied float64) process noise through the multi-tile kernel."""
    n, K = 1500, 5
    A = torch.from_numpy(np.random.default_rng(2).uniform(-1, 1, (K, n, 2)).astype(np.float32)).cuda()
    nz = torch.from_numpy(np.random.default_rng(3).normal(0, 3, (K, n, 3))).cuda()
    res = [_run(gl, "pmsm", n, var, A, {"add_noise": True}, noise=nz) for var in (E1, E2)]
    for k in range(K):
        for a, b in zip(res[0][0][k], res[1][0][k]):
            assert bits_equal(a, b), k


@pytest.fixture(scope="module")
def orc():
    import oracle

    return oracle


def _planes(be, p0, k):
    return np.stack([_np(be.get_state(p0 + j)) for j in range(k)], 1)


def test_hr_1m_injected_noise_vs_oracle(gl, orc):
    """HR at 1,048,576 envs with INJECTED noise: step_tiles sends every injected-noise
    launch to k_step (k_step_multi draws its noise on the device; that default launch is
    covered in test_gpu_default_launch.py) -- asserted through LZ_CALL_STEP_NOISE.  6
    float32 steps, the whole batch bit for bit against the oracle's DEV restatement."""
    from gym_lorenz import _native as nat

    n, T = 1 << 20, 6
    be = gl.BatchedEnv("hr", n, dtype="float32", seed=5, add_noise=True, autoreset=False)
    assert nat.launch_shape(be._h, nat.CALL_STEP_NOISE)["kernel"] == "step"
    be.reset()
    init = orc.reset_draw("hr", np.float32, n, 0, 5, 0, add_noise=True)
    st = np.ascontiguousarray(init[:, :6])
    fa = np.zeros((n, 2), np.float32)
    rng = np.random.default_rng(12)
    with np.errstate(all="ignore"):
        for k in range(T):
            a = rng.uniform(-1.2, 1.2, (n, 2)).astype(np.float32)
            nz = rng.normal(0, 1, (n, 3)) * init[:, 6:7]
            o, r, d = be.step(torch.from_numpy(a).cuda(), torch.from_numpy(nz).cuda())
            oo, rr, tt = orc.hr_step(st, fa, a, nz.astype(np.float32), True, False, orc.DEV)
            assert bits_equal(_np(o), oo) and bits_equal(_np(r), rr), k
            assert np.array_equal((_np(d) & 1).astype(bool), tt), k
    assert bits_equal(_planes(be, 0, 6), st)
    be.close()


def test_pmsm_1m_injected_noise_vs_oracle(gl, orc):
    """PMSM at 1,048,576 envs with INJECTED noise (k_step, asserted; the device-noise
    default k_step_multi is test_gpu_default_launch.py's): 6 steps, obs / state / lambda
    path bit for bit vs the oracle's DEV mode."""
    from gym_lorenz import _native as nat

    n, T = 1 << 20, 6
    be = gl.BatchedEnv("pmsm", n, seed=6, add_noise=True, autoreset=False)
    assert nat.launch_shape(be._h, nat.CALL_STEP_NOISE)["kernel"] == "step"
    be.reset()
    S = orc.PmsmState(n)
    S.st[:] = orc.reset_draw("pmsm", np.float32, n, 0, 6, 0)
    rng = np.random.default_rng(13)
    with np.errstate(all="ignore"):
        for k in range(T):
            a = rng.uniform(-1.2, 1.2, (n, 2)).astype(np.float32)
            nz = rng.normal(0, 3, (n, 3))
            o, r, d = be.step(torch.from_numpy(a).cuda(), torch.from_numpy(nz).cuda())
            oo, rr, tt = orc.pmsm_step(S, a, nz, True, 0.5, orc.DEV)[:3]
            assert bits_equal(_np(o), oo) and bits_equal(_np(r), rr), k
    assert bits_equal(_planes(be, 0, 6), S.st)
    be.close()
