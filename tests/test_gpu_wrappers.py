"""GPU: the on-device VecFrameStack (lz_frame_stack, LorenzVecFrameStack) against the
NumPy restatement of SB3 2.7.1's StackedObservations (oracle/sb3_framestack.py),
bit-exact, including the stacked terminal observations of done envs."""
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


@pytest.mark.parametrize("n,S,O,misalign", [
    (3001, 4, 6, False),   # LDS tiles, 16-B vectors, a ragged last tile, obs tail scalar
    (512, 4, 8, False),    # whole tiles, all-vector
    (3001, 4, 6, True),    # obs not 16-B aligned: scalar tile path
    (300, 3, 5, False),    # S*O = 15: scalar tile path
    (1, 2, 3, False),
    (100, 20, 6, False),   # S*O + O > 64: the per-row kernel
])
def test_frame_stack_kernel_vs_sb3(gl, n, S, O, misalign):
    from gym_lorenz import _native as nat
    from oracle.sb3_framestack import StackedObservations

    rng = np.random.default_rng(0)
    ref = StackedObservations(n, S, O)
    st = torch.zeros((n, S * O), dtype=torch.float32, device="cuda")
    sp = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    P = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731

    def dev(a):  # optionally 4 B past a 16-B boundary
        t = torch.zeros(a.size + 1, dtype=torch.float32, device="cuda")
        v = t[1:] if misalign else t[:-1]
        v.copy_(torch.from_numpy(a.reshape(-1)))
        return v

    obs = rng.normal(size=(n, O)).astype(np.float32)
    ref.reset(obs)
    nat.check(nat.lib.lz_frame_stack(P(st), P(dev(obs)), None, n, S, O, 1, 0, sp))
    assert np.array_equal(st.cpu().numpy(), ref.stacked_obs)
    for _ in range(12):
        obs = rng.normal(size=(n, O)).astype(np.float32)
        done = rng.random(n) < 0.1
        ref.update(obs, done, [{} for _ in range(n)])
        d = torch.from_numpy(done.astype(np.uint8)).cuda()
        nat.check(nat.lib.lz_frame_stack(P(st), P(dev(obs)), P(d), n, S, O, 0, 0, sp))
        assert np.array_equal(st.cpu().numpy(), ref.stacked_obs)


@pytest.mark.parametrize("tensors", [False, True])
def test_vec_frame_stack_hr_vs_sb3(gl, tensors):
    from gym_lorenz.vec_frame_stack import LorenzVecFrameStack
    from oracle.sb3_framestack import StackedObservations

    n, S = 257, 4
    kw = dict(max_episode_steps=6, add_noise=True, seed=3)
    va = LorenzVecFrameStack(gl.make_vec("lorenz_try-v0", n, return_tensors=tensors, **kw), S)
    vb = gl.make_vec("lorenz_try-v0", n, **kw)
    assert va.observation_space.shape == (S * 6,)
    ref = StackedObservations(n, S, 6)
    oa = va.reset()
    ob = ref.reset(vb.reset())
    assert np.array_equal(oa.cpu().numpy() if tensors else oa, ob)
    rng = np.random.default_rng(1)
    seen = 0
    for _ in range(15):
        act = rng.uniform(-1, 1, (n, 2)).astype(np.float32)
        oa, ra, da, ia = va.step(torch.from_numpy(act).cuda() if tensors else act)
        o2, r2, d2, i2 = vb.step(act)
        ob, i2 = ref.update(o2, d2, i2)
        oa_h = oa.cpu().numpy() if tensors else oa
        assert np.array_equal(oa_h, ob)
        da_h = da.cpu().numpy() if tensors else da
        assert np.array_equal(da_h, d2)
        for i in np.nonzero(d2)[0]:
            ta = ia[int(i)]["terminal_observation"]
            ta = ta.cpu().numpy() if isinstance(ta, torch.Tensor) else ta
            assert np.array_equal(ta, i2[int(i)]["terminal_observation"])
            seen += 1
    assert seen > 0
