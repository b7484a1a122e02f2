"""GPU: indexed state access (lz_get_state / lz_set_state with an env-id list) -- the
boundary SURVEY.md §8b names for the per-env attribute reads / writes of a DummyVecEnv
caller.  The CS-5 injection of code/lorenz_pmsm/test_evaluate.py:100-102
(`base_env.state1 = fixed_init_state1; base_env.state2 = fixed_init_state2`) into ONE
env of cfg4's 262,144-env PMSM handle, then 100 closed-loop steps: that env follows the
single-env oracle (orc_pmsm_step) bit for bit and every other env is bit-identical to a
twin handle that was not touched."""
import ctypes

import numpy as np
import pytest
import torch

from conftest import bits_equal

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def gl():
    import gym_lorenz

    return gym_lorenz


def _np(t):
    return t.cpu().numpy()


def test_inject_one_env_pmsm_262k(gl, orc):
    import gym_lorenz._native as nat

    n, j, K = 1 << 18, 123_456, 100
    A = gl.BatchedEnv("pmsm", n, seed=3, add_noise=True, autoreset=False, compact=False)
    B = gl.BatchedEnv("pmsm", n, seed=3, add_noise=True, autoreset=False, compact=False)
    A.reset(), B.reset()
    s1 = np.array([10.0, -10.0, 15.0], np.float32)  # test_evaluate.py fixed_init_state1
    for c in range(3):
        A.set_state(nat.PMSM_S1 + c, s1[c:c + 1], indices=[j])
        A.set_state(nat.PMSM_S2 + c, np.zeros(1, np.float32), indices=[j])
    # the single-env oracle starts from what the handle now holds for env j (a gather)
    S = orc.PmsmState(1)
    for p in range(6):
        S.st[0, p] = _np(A.get_state(p, indices=[j]))[0]
    S.lam[0] = _np(A.get_state(nat.PMSM_LAMBDA, indices=[j]))[0]
    S.m[0] = _np(A.get_state(nat.PMSM_M, indices=[j]))[0]
    S.v[0] = _np(A.get_state(nat.PMSM_V, indices=[j]))[0]
    S.adam_step[0] = _np(A.get_state(nat.PMSM_ADAM_STEP, indices=[j]))[0]
    S.cur_step[0] = _np(A.get_state(nat.PMSM_STEP, indices=[j]))[0]
    assert bits_equal(S.st[0], np.concatenate([s1, np.zeros(3, np.float32)]))
    g = torch.Generator(device="cuda").manual_seed(5)
    keep = torch.ones(n, dtype=torch.bool, device="cuda")
    keep[j] = False
    for k in range(K):
        act = torch.rand((n, 2), generator=g, device="cuda") * 2 - 1
        noise = torch.randn((n, 3), generator=g, device="cuda", dtype=torch.float64) * 3.0
        oa, ra, da = A.step(act, noise=noise)
        ob, rb, db = B.step(act, noise=noise)
        oo, rr, te, tr = orc.pmsm_step(S, _np(act[j:j + 1]), _np(noise[j:j + 1]), True, 0.5, orc.DEV)
        assert bits_equal(_np(oa[j:j + 1]), oo), k
        assert bits_equal(_np(ra[j:j + 1]), rr), k
        assert int(da[j]) == int(te[0]) | (2 * int(tr[0])), k
        assert torch.equal(oa[keep].view(torch.int32), ob[keep].view(torch.int32)), k
        assert torch.equal(ra[keep].view(torch.int32), rb[keep].view(torch.int32)), k
        assert torch.equal(da[keep], db[keep]), k
    for p in range(11):
        pa, pb = A.get_state(p), B.get_state(p)
        assert torch.equal(pa[keep].view(torch.int32), pb[keep].view(torch.int32)), p
    assert bits_equal(_np(A.get_state(nat.PMSM_LAMBDA, indices=[j])), S.lam)
    assert int(_np(A.get_state(nat.PMSM_STEP, indices=[j]))[0]) == int(S.cur_step[0])
    A.close(), B.close()


@pytest.mark.parametrize("system,dtype", [("hr", "float64"), ("lorenz3", "float32"),
                                          ("pmsm", "float32")])
def test_indexed_roundtrip(gl, system, dtype):
    """Gather in the order asked; scatter touches only the listed envs; a repeated id
    keeps its last value (the wrapper dedupes); int planes; empty lists; host-side
    range checks."""
    n = 10_007  # ragged
    be = gl.BatchedEnv(system, n, dtype=dtype, seed=1, autoreset=False, compact=False)
    be.reset()
    rng = np.random.default_rng(4)
    info_planes = {"hr": 10, "lorenz3": 4, "pmsm": 11}[system]
    for p in range(info_planes):
        full = _np(be.get_state(p)).copy()
        ids = rng.choice(n, 300, replace=False)
        assert bits_equal(_np(be.get_state(p, indices=ids)), full[ids])
        vals = (rng.standard_normal(300) * 7).astype(full.dtype)
        ids2 = np.concatenate([ids, ids[:5]])  # repeats: the last occurrence wins
        vals2 = np.concatenate([vals, vals[:5] + 1])
        be.set_state(p, vals2, indices=ids2)
        want = full.copy()
        want[ids2] = vals2  # numpy assignment: the last occurrence wins
        assert bits_equal(_np(be.get_state(p)), want), p
        be.set_state(p, vals[:0], indices=np.zeros(0, np.int64))  # empty: no-op
        assert _np(be.get_state(p, indices=[])).size == 0
    with pytest.raises(IndexError):
        be.get_state(0, indices=[n])
    with pytest.raises(IndexError):
        be.set_state(0, [1.0], indices=[-1])
    be.close()


def test_indexed_out_of_range_at_the_abi(gl):
    """Straight through the C-ABI (no host check): ids outside [0, N) read as zero and
    are skipped by the scatter -- no fault, nothing else written."""
    import gym_lorenz._native as nat

    n = 1000
    be = gl.BatchedEnv("lorenz3", n, dtype="float64", seed=2, autoreset=False, compact=False)
    be.reset()
    full = _np(be.get_state(0)).copy()
    idx = torch.tensor([3, -1, n, 1 << 40, 7], dtype=torch.int64, device="cuda")
    dst = torch.full((5,), 99.0, dtype=torch.float64, device="cuda")
    nat.check(nat.lib.lz_get_state(be._h, 0, ctypes.c_void_p(dst.data_ptr()),
                                   ctypes.c_void_p(idx.data_ptr()), 5))
    be.sync()
    assert bits_equal(_np(dst), np.array([full[3], 0, 0, 0, full[7]]))
    src = torch.arange(5, dtype=torch.float64, device="cuda") + 100
    nat.check(nat.lib.lz_set_state(be._h, 0, ctypes.c_void_p(src.data_ptr()),
                                   ctypes.c_void_p(idx.data_ptr()), 5))
    want = full.copy()
    want[3], want[7] = 100.0, 104.0
    assert bits_equal(_np(be.get_state(0)), want)
    st = nat.lib.lz_get_state(be._h, 0, ctypes.c_void_p(dst.data_ptr()), None, 5)
    assert st == nat.LZ_ERR_INVALID  # whole plane with a count that is not N
    be.close()


def test_vecenv_set_attr_one_env(gl):
    """LorenzVecEnv.set_attr / get_attr(indices=[i]) over the device gather / scatter."""
    n, j = 4096, 1234
    v = gl.LorenzVecEnv("lorenz_pmsm-v0", n, seed=0)
    v.reset()
    before = np.stack(v.get_attr("state1"))
    v.set_attr("state1", np.array([10.0, -10.0, 15.0]), indices=[j])
    v.set_attr("state2", np.zeros(3), indices=[j])
    after = np.stack(v.get_attr("state1"))
    assert np.array_equal(after[j], [10, -10, 15])
    keep = np.arange(n) != j
    assert bits_equal(after[keep], before[keep])
    assert np.array_equal(v.get_attr("state2", indices=j)[0], [0, 0, 0])
    v.close()
