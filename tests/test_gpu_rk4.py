"""GPU: the RK4 integrator mode of LORENZ3 / LORENZ4 (lz_config.integrator =
LZ_INT_RK4; SysL3RK4 / SysL4RK4 in lz_systems.h) against the oracle's restatement
(orc_l3_step_rk4 / orc_l4_step_rk4), bit for bit, NaN-aware, through every path the
mode runs on: lz_step (k_step), lz_rollout (one-wave k_rollout below 131,072 envs, the
256-lane kernel above), the resident drop-in server and lz_step_vecnorm's step.

Parity vs the reference: UNPINNED -- the reference has no RK4 Lorenz (dynamic.py:70-75
is forward Euler).  The oracle is pinned instead to an independent NumPy float64 RK4
of dynamic.py's RHS and to fourth-order convergence (tests/test_rk4_host.py)."""
import numpy as np
import pytest
import torch

from conftest import bits_equal
from oracle_tl import OracleTL

pytestmark = [pytest.mark.gpu, pytest.mark.filterwarnings("ignore::RuntimeWarning")]


@pytest.fixture(scope="module")
def gl():
    import gym_lorenz

    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    return gym_lorenz


def _np(t):
    return t.detach().cpu().numpy()


def _setup(gl, orc, name, system, dtype, n, seed, L):
    npd = np.float64 if dtype == "float64" else np.float32
    be = gl.BatchedEnv(name, n, dtype=dtype, seed=seed, max_episode_steps=L, integrator="rk4")
    assert be.integrator == "rk4" and be.config.integrator == gl._native.INT_RK4
    be.reset()
    steps0 = np.random.default_rng(seed).integers(0, L, n).astype(np.int32)
    plane = gl._native.L3_STEP if system == "l3" else gl._native.L4_STEP
    be.set_state(plane, torch.from_numpy(steps0))
    return be, OracleTL(orc, system, npd, n, seed, L, steps0, rk4=True)


def _actions(n, count=5):
    rng = np.random.default_rng(11)
    A = [rng.uniform(-1, 1, (n, 3)).astype(np.float32) for _ in range(count)]
    A[1][: n // 50] *= 900.0  # the +-500 clip
    return A, [torch.from_numpy(a).cuda() for a in A]


@pytest.mark.parametrize("n,dtype,T,every", [(65536, "float32", 1000, 1), (65536, "float64", 300, 1),
                                             (65573, "float32", 200, 1), (1 << 20, "float32", 1000, 50)])
def test_l3_rk4_step_vs_oracle(gl, orc, n, dtype, T, every):
    """lz_step, 1000 steps with staggered TimeLimit(300) truncations + auto-reset: obs,
    reward, done bytes, the compact done list (ids and terminal obs) and the final state
    planes equal the oracle.  At 1,048,576 envs (BASELINE's size) the obs / reward are
    compared every 50th step, the done lists at every step."""
    be, ref = _setup(gl, orc, "lorenz3", "l3", dtype, n, 17, 300)
    A, At = _actions(n)
    resets = 0
    for k in range(T):
        o, r, d = be.step(At[k % len(A)])
        oo, rr, dd, idx, term = ref.step(A[k % len(A)])
        nd = int(be.n_done_dev.item())
        assert nd == idx.size, k
        resets += nd
        if nd:
            gi, gt = be.done_list()
            assert np.array_equal(_np(gi), idx), k
            assert bits_equal(_np(gt), term), k
        if k % every == 0 or k == T - 1:
            assert bits_equal(_np(o), oo), k
            assert bits_equal(_np(r), rr), k
            assert np.array_equal(_np(d), dd), k
    st = np.stack([_np(be.get_state(p)) for p in range(3)], 1)
    assert bits_equal(st, ref.st)
    assert resets >= n * (T // 300)
    be.close()


@pytest.mark.parametrize("n,K,launches", [(65536, 250, 4), (70001, 100, 3), (1 << 20, 100, 10)])
def test_l3_rk4_rollout_vs_oracle(gl, orc, n, K, launches):
    """lz_rollout of the RK4 system (one-wave kernel at 65,536 / 70,001 -- ragged -- and
    the 256-lane kernel at 1M) over K * launches steps with auto-reset == the oracle:
    every step's obs / reward / done at 65,536 and 70,001, the last step of each launch
    at 1M; the compact done list (k * N + env, terminal obs) of every launch."""
    be, ref = _setup(gl, orc, "lorenz3", "l3", "float32", n, 23, 300)
    A, At = _actions(n)
    full = n < (1 << 20)
    for L in range(launches):
        acts = torch.stack([At[(L * K + k) % len(A)] for k in range(K)])
        obs, rew, done, (didx, tobs, nd) = be.rollout(acts, capture_terminal=2 * n)
        want_idx, want_term = [], []
        for k in range(K):
            oo, rr, dd, idx, term = ref.step(A[(L * K + k) % len(A)])
            want_idx.append(k * n + idx)
            want_term.append(term)
            if full or k == K - 1:
                assert bits_equal(_np(obs[k]), oo), (L, k)
                assert bits_equal(_np(rew[k]), rr), (L, k)
                assert np.array_equal(_np(done[k]), dd), (L, k)
        m = int(nd.item())
        wi = np.concatenate(want_idx)
        assert m == wi.size, L
        order = torch.argsort(didx[:m])
        assert np.array_equal(_np(didx[:m][order]), wi), L
        assert bits_equal(_np(tobs[:m][order]), np.concatenate(want_term)), L
    st = np.stack([_np(be.get_state(p)) for p in range(3)], 1)
    assert bits_equal(st, ref.st)
    be.close()


@pytest.mark.parametrize("n,dtype,rollout", [(65536, "float32", False), (70001, "float32", True),
                                             (65536, "float64", True), (140001, "float32", True)])
def test_l4_rk4_vs_oracle(gl, orc, n, dtype, rollout):
    """LORENZ4 (lorenz_env_transient.py) in RK4 mode, 300 steps with TimeLimit(120)
    auto-reset, through lz_step or lz_rollout (K = 100: the one-wave kernel below its
    3/4 x 256 x CUs bound only for the Euler system -- RK4 takes the generic 131,072 bound
    -- and the 256-lane kernel with alternating obs tiles at 140,001)."""
    be, ref = _setup(gl, orc, "lorenz4", "l4", dtype, n, 31, 120)
    zero = torch.zeros((100, n, 3), device="cuda")
    for L in range(3):
        if rollout:
            obs, rew, done = be.rollout(zero)
        for k in range(100):
            oo, rr, dd, idx, term = ref.step(None)
            if not rollout:
                o, r, d = be.step(zero[0])
                if idx.size:
                    gi, gt = be.done_list()
                    assert np.array_equal(_np(gi), idx) and bits_equal(_np(gt), term), k
            else:
                o, r, d = obs[k], rew[k], done[k]
            if rollout or k % 10 == 0:
                assert bits_equal(_np(o), oo), (L, k)
                assert bits_equal(_np(r), rr), (L, k)
                assert np.array_equal(_np(d), dd), (L, k)
    st = np.concatenate([np.stack([_np(be.get_state(p)) for p in range(8)], 1)])
    assert bits_equal(st, ref.st)
    be.close()


@pytest.mark.parametrize("system,n,dtype", [("lorenz3", 1, "float64"), ("lorenz3", 64, "float32"),
                                            ("lorenz4", 3, "float32")])
def test_rk4_resident_server_vs_oracle(gl, orc, system, n, dtype):
    """The per-env drop-in path: lz_resident_step on an RK4 handle equals lz_step_host on
    another and the oracle, 300 steps (the resident wave runs SysL3RK4 / SysL4RK4's
    step_body, no launch per step)."""
    from gym_lorenz import _native as nat
    from gym_lorenz.core import BatchedEnv

    npd = np.float64 if dtype == "float64" else np.float32
    envs = []
    for _ in range(2):
        be = BatchedEnv(system, n, dtype=dtype, seed=3, autoreset=False, compact=False, integrator="rk4")
        be.reset()
        envs.append(be)
    key = "l3" if system == "lorenz3" else "l4"
    st = np.ascontiguousarray(orc.reset_draw(key, npd, n, 0, 3, 0).copy())
    O = envs[0].obs_dim
    bufs = [(np.zeros((n, O), npd), np.zeros(n, npd), np.zeros(n, np.uint8)) for _ in range(2)]
    rng = np.random.default_rng(4)
    for k in range(300):
        act = rng.uniform(-1, 1, (n, 3)).astype(np.float32)
        for fn, be, (o, r, d) in ((nat.lib.lz_step_host, envs[0], bufs[0]),
                                  (nat.lib.lz_resident_step, envs[1], bufs[1])):
            nat.check(fn(be._h, act.ctypes.data, None, o.ctypes.data, r.ctypes.data, d.ctypes.data))
        oo, rr = orc.l3_step_rk4(st, act) if key == "l3" else orc.l4_step_rk4(st)[:2]
        for o, r, d in bufs:
            assert bits_equal(o, oo), k
            assert bits_equal(r, rr), k
    for be in envs:
        be.close()


def test_rk4_vecnorm_step_and_policy_rejection(gl, orc):
    """lz_step_vecnorm's step runs the RK4 system too (raw outputs == lz_step's), and the
    policy rollouts -- Euler only -- refuse an RK4 handle with LZ_ERR_UNSUPPORTED."""
    from gym_lorenz import _native as nat
    from gym_lorenz.policy import ActorCriticMlp, FusedRolloutCollector
    from gym_lorenz.vec_env import LorenzVecEnv
    from gym_lorenz.vec_normalize import LorenzVecNormalize

    n = 4096
    venv = LorenzVecNormalize(LorenzVecEnv("lorenz_dynamic-v0", n, seed=5, return_tensors=True,
                                           integrator="rk4"), norm_obs=True, norm_reward=False)
    be = gl.BatchedEnv("lorenz3", n, seed=5, integrator="rk4")
    venv.reset()
    be.reset()
    a = torch.from_numpy(np.random.default_rng(0).uniform(-1, 1, (n, 3)).astype(np.float32)).cuda()
    for _ in range(5):
        venv.step(a)
        o, r, d = be.step(a)
    assert bits_equal(_np(venv.get_original_obs()), _np(o))
    sd = ActorCriticMlp(6, 3, seed=0).state_dict()
    with pytest.raises(nat.LorenzEnvError, match="Euler"):
        col = FusedRolloutCollector(be, sd, precision="fp32", vecnorm_update="rollout")
        col.reset()
        col.collect(2)
