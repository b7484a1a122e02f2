"""A rollout's ragged LAST group on the full DMA path (r06; lz_kernels.hip rollout_loop /
split_loop kRag): N a multiple of 4 (the launch's vec_ok) but not of the group's env count.
The group's DMA sources are clamped to its own rows and the lanes past its envs store
nothing (the noise-free systems, LZ_RAG = 2; PMSM / HR keep the staged path with a
one-step register prefetch).  Bar: K fused steps == K lz_step calls bit for bit (obs,
reward, done, the compact done list, every final state plane) for each kernel family
whose last group is partial: one-wave (LORENZ3, PMSM, HR), split lanes (LORENZ3), lane
pairs (PMSM), with TimeLimit truncations inside the launch.  (N not a multiple of 4 keeps the staged path:
test_gpu_parity.py's 4,097 / 70,001 cases.)"""
import numpy as np
import pytest
import torch

from conftest import bits_equal

pytestmark = [pytest.mark.gpu, pytest.mark.filterwarnings("ignore::RuntimeWarning")]


@pytest.fixture(scope="module")
def gl():
    import gym_lorenz

    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    return gym_lorenz


def _np(t):
    return t.detach().cpu().numpy()


@pytest.mark.parametrize("system,n,kernel", [
    ("lorenz3", 16400, "rollout_wave"),   # 256 whole 64-env groups + 16 envs
    ("lorenz3", 32784, "rollout_split"),  # 1,024 whole 32-env groups + 16
    ("pmsm", 24592, "rollout_pair"),      # 768 whole pair groups + 16
    ("pmsm", 4100, "rollout_wave"),       # + 4 envs
    ("hr", 32784, "rollout_wave"),
    ("hr", 1028, "rollout_wave"),
])
def test_ragged_group_full_path_equals_steps(gl, system, n, kernel):
    from gym_lorenz import _native as nat

    K = 41
    kw = {"add_noise": True} if system in ("pmsm", "hr") else {}
    a_be = gl.BatchedEnv(system, n, seed=21, max_episode_steps=13, **kw)
    b_be = gl.BatchedEnv(system, n, seed=21, max_episode_steps=13, **kw)
    assert nat.launch_shape(a_be._h, nat.CALL_ROLLOUT)["kernel"] == kernel
    a_be.reset()
    b_be.reset()
    A = torch.from_numpy(np.random.default_rng(7).uniform(-1.2, 1.2, (K, n, a_be.action_dim))
                         .astype(np.float32)).cuda()
    obs, rew, done, (didx, tobs, nd) = a_be.rollout(A, capture_terminal=K * n)
    want = []
    for k in range(K):
        o, r, d = b_be.step(A[k])
        assert bits_equal(_np(obs[k]), _np(o)), k
        assert bits_equal(_np(rew[k]), _np(r)), k
        assert np.array_equal(_np(done[k]), _np(d)), k
        want.append(k * n + np.nonzero(_np(d))[0])
    m = int(nd.item())
    wi = np.concatenate(want)
    assert m == wi.size and m > 0
    assert np.array_equal(np.sort(_np(didx[:m])), wi)
    for p in range(a_be.info.n_planes):
        assert bits_equal(_np(a_be.get_state(p)), _np(b_be.get_state(p))), p
    a_be.close()
    b_be.close()
