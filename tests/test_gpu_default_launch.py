"""The DEFAULT lz_step launch at the sizes that select it.

step_tiles (lz_kernels.hip) picks k_step_multi (4 tiles of 256 envs per workgroup) on its
own only on a balanced grid: 4 workgroups of 1,024 envs per CU (PMSM / HR / LORENZ3 f32 at
1,048,576 on 256 CUs) or, for PMSM / LORENZ3, 3 per CU (786,432) -- and only when the noise
is drawn on the device.  test_gpu_step_multi.py compares the two kernels under FORCED
variants at <= 70,000 envs; here the default choice runs at its own size, asserted through
lz_get_launch_shape, against a forced-k_step twin (variant 16384, itself bit-exact vs the
oracle) bit for bit: obs, reward, done bytes, compact done list + terminal obs, every
state plane, with device noise and TimeLimit(9) auto-reset inside the 20-step window.
The headline kernel (LORENZ3 f32, 1M) also runs against the oracle with TimeLimit(7)
auto-reset and compaction for 30 steps.

Reference: lorenz_env_try_pmsm.py:76-184, lorenz_env_try.py:80-179, dynamic.py:61-90."""
import numpy as np
import pytest
import torch

from conftest import bits_equal
from oracle_tl import OracleTL

pytestmark = [pytest.mark.gpu, pytest.mark.filterwarnings("ignore::RuntimeWarning")]

FORCE_K_STEP = 16384  # variant bits 14-15 = 1: one tile per workgroup


@pytest.fixture(scope="module")
def gl():
    import gym_lorenz

    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    return gym_lorenz


@pytest.fixture(scope="module")
def cus():
    return torch.cuda.get_device_properties(0).multi_processor_count


def _np(t):
    return t.detach().cpu().numpy()


def _balanced(n, cus, three):
    """lz_kernels.hip step_tiles_balanced (mirrored in test_kernel_hash.py): multi-tile?"""
    groups = (n + 1023) // 1024
    return groups == 4 * cus or (three and groups == 3 * cus)


def _bits(t):
    return t.view(torch.int32) if t.dtype == torch.float32 else t.view(torch.int64) \
        if t.dtype == torch.float64 else t


def _same(a, b):
    return a.shape == b.shape and torch.equal(_bits(a), _bits(b))


CASES = [("pmsm", 1 << 20, {"add_noise": True}), ("hr", 1 << 20, {"add_noise": True}),
         ("pmsm", 786432, {"add_noise": True}), ("lorenz3", 786432, {}),
         ("lorenz3", 1 << 20, {}), ("hr", 786432, {"add_noise": True}),
         ("lorenz3", 262144, {}),  # r06: one tile by default (the two-tile mode is bimodal) ...
         ("lorenz3", 262144, {"variant": 32768})]  # ... and two tiles, forced


@pytest.mark.parametrize("system,n,kw", CASES,
                         ids=["%s-%d%s" % (c[0], c[1], "-v%d" % c[2]["variant"] if "variant" in c[2] else "")
                              for c in CASES])
def test_default_step_launch_vs_forced_k_step(gl, cus, system, n, kw):
    from gym_lorenz import _native as nat

    kw = dict(kw)
    forced = kw.pop("variant", 0)
    be = gl.BatchedEnv(system, n, dtype="float32", seed=31, max_episode_steps=9, variant=forced, **kw)
    tw = gl.BatchedEnv(system, n, dtype="float32", seed=31, max_episode_steps=9,
                       variant=FORCE_K_STEP, **kw)
    want = "step_multi" if forced or _balanced(n, cus, system != "hr") else "step"
    if cus == 256:  # MI355X: the sizes above are exactly the ones that select each branch
        assert want == ("step" if (system, n, forced) in (("hr", 786432, 0), ("lorenz3", 262144, 0))
                        else "step_multi")
    assert nat.launch_shape(be._h, nat.CALL_STEP)["kernel"] == want
    assert nat.launch_shape(be._h, nat.CALL_STEP_NOISE)["kernel"] == "step"
    assert nat.launch_shape(tw._h, nat.CALL_STEP)["kernel"] == "step"
    be.reset()
    tw.reset()
    # staggered step counters: truncations (and auto-resets) at every step of the window
    steps0 = torch.from_numpy(np.random.default_rng(4).integers(0, 9, n).astype(np.int32)).cuda()
    plane = {"pmsm": nat.PMSM_STEP, "hr": nat.HR_STEP, "lorenz3": nat.L3_STEP}[system]
    be.set_state(plane, steps0)
    tw.set_state(plane, steps0)
    g = torch.Generator(device="cuda").manual_seed(7)
    dones = 0
    for k in range(20):
        a = torch.rand((n, be.action_dim), generator=g, device="cuda") * 2.6 - 1.3
        o1, r1, d1 = be.step(a)
        o2, r2, d2 = tw.step(a)
        assert _same(o1, o2) and _same(r1, r2) and torch.equal(d1, d2), k
        i1, t1 = be.done_list()
        i2, t2 = tw.done_list()
        assert torch.equal(i1, i2) and _same(t1, t2), k
        dones += int(i1.numel())
    assert dones >= n * 2  # every env truncated at least twice in 20 steps
    for p in range(be.info.n_planes):
        assert _same(be.get_state(p), tw.get_state(p)), p
    be.close()
    tw.close()


def test_headline_l3_1m_autoreset_vs_oracle(gl, cus):
    """The bench headline's kernel (LORENZ3 f32, 1,048,576 envs: k_step_multi on 256 CUs)
    with TimeLimit(7) auto-reset and compaction, 30 steps vs the oracle: obs, reward, done
    bytes, the compact done list (ids + terminal obs) every step, the state planes at the
    end."""
    import oracle as orc
    from gym_lorenz import _native as nat

    n, L, T = 1 << 20, 7, 30
    be = gl.BatchedEnv("lorenz3", n, dtype="float32", seed=41, max_episode_steps=L)
    assert nat.launch_shape(be._h, nat.CALL_STEP)["kernel"] == (
        "step_multi" if _balanced(n, cus, True) else "step")
    be.reset()
    steps0 = np.random.default_rng(41).integers(0, L, n).astype(np.int32)
    be.set_state(nat.L3_STEP, torch.from_numpy(steps0).cuda())
    ref = OracleTL(orc, "l3", np.float32, n, 41, L, steps0)
    rng = np.random.default_rng(3)
    resets = 0
    for k in range(T):
        a = rng.uniform(-1, 1, (n, 3)).astype(np.float32)
        a[: n // 64] *= 900.0  # the +-500 action clip
        o, r, d = be.step(torch.from_numpy(a).cuda())
        oo, rr, dd, idx, term = ref.step(a)
        nd = int(be.n_done_dev.item())
        assert nd == idx.size, k
        resets += nd
        if nd:
            gi, gt = be.done_list()
            assert np.array_equal(_np(gi), idx), k
            assert bits_equal(_np(gt), term), k
        assert bits_equal(_np(o), oo), k
        assert bits_equal(_np(r), rr), k
        assert np.array_equal(_np(d), dd), k
    st = np.stack([_np(be.get_state(p)) for p in range(3)], 1)
    assert bits_equal(st, ref.st)
    assert resets >= n * (T // L)
    be.close()
