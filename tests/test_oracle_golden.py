"""Pin the CPU oracle to the reference: mode REF must reproduce the golden fixtures
(outputs of the reference env classes, tests/golden/make_golden.py) BIT-EXACTLY.

Also checks mode DEV (the device kernel's formulas) against mode REF within the
tolerance that glibc's not-correctly-rounded pow/powf allows (1 ulp level)."""
import numpy as np
import pytest

from conftest import bits_equal, golden


def test_l3_golden_bitexact(orc):
    """dynamic.py:35-90 in fp64: obs, reward, done, 1000 steps, incl. +-500 clip and
    two trajectories that overflow to inf/NaN."""
    g = golden("l3")
    st = g["x0"].copy()
    assert bits_equal(orc.l3_reset_obs(st), g["obs0"])
    with np.errstate(all="ignore"):
        for k in range(g["obs"].shape[1]):
            o, r = orc.l3_step(st, g["actions"][:, k].astype(np.float64))
            assert bits_equal(o, g["obs"][:, k]), k
            assert bits_equal(r, g["reward"][:, k]), k
    assert not g["done"].any()  # dynamic.py:86 never fires (t == 10 on a float sum)
    assert not np.isfinite(g["obs"][-2:, -1]).all()  # the divergent seeds did diverge


def test_l3_done_accumulator(orc):
    """The reference's 't += 0.01; done = t == 10' never fires; the host
    replay used by lz_create must agree with the reference's own accumulator."""
    g = golden("l3")
    t = g["t_hist"]
    assert not (t == 10.0).any()
    assert orc.t_done_step(0.01, 10.0) == -1
    assert orc.t_done_step(0.001, 5.0) == -1  # lorenz_env_transient.py:364,369
    assert orc.t_done_step(0.25, 1.0) == 4  # an accumulator that does hit T exactly


def test_l4_golden_bitexact(orc):
    g = golden("l4")
    st = g["init"].copy()
    assert bits_equal(orc.l4_reset_obs(st), g["obs0"])
    with np.errstate(all="ignore"):
        for k in range(g["obs"].shape[1]):
            o, r, d = orc.l4_step(st)
            assert bits_equal(o, g["obs"][:, k]), k
            assert bits_equal(r, g["reward"][:, k]), k
            assert np.array_equal(d, g["done"][:, k]), k


def _run_pmsm(orc, g, i, mode):
    n_steps = g["obs"].shape[1]
    S = orc.PmsmState(1)
    S.st[0] = g["init"][i, 0].reshape(6)
    out = {"obs": [], "rew": [], "te": [], "tr": [], "lam": [], "m": [], "v": []}
    with np.errstate(all="ignore"):
        for k in range(n_steps):
            if k == int(g["reset_at"]):
                S.st[0] = g["init"][i, 1].reshape(6)
                S.cur_step[0] = 0
            o, r, te, tr = orc.pmsm_step(S, g["actions"][i, k][None], g["noise"][i, k][None],
                                         bool(g["add_noise"][i]), float(np.float32(g["alpha"][i])),
                                         mode)
            for key, val in (("obs", o[0]), ("rew", r[0]), ("te", te[0]), ("tr", tr[0]),
                             ("lam", S.lam[0]), ("m", S.m[0]), ("v", S.v[0])):
                out[key].append(np.copy(val))
    return {k: np.array(v) for k, v in out.items()}


@pytest.mark.parametrize("i", range(9))
def test_pmsm_golden_bitexact(orc, i):
    """lorenz_env_try_pmsm.py:59-184, fp32: obs, reward, Adam m/v, lambda, flags,
    across a reset (Adam/lambda persist), with and without f64 process noise."""
    g = golden("pmsm")
    if not g["injected"][i]:
        assert bits_equal(orc.pmsm_reset_obs(g["init"][i, 0].reshape(1, 6))[0], g["obs0"][i, 0])
    assert bits_equal(orc.pmsm_reset_obs(g["init"][i, 1].reshape(1, 6))[0], g["obs0"][i, 1])
    out = _run_pmsm(orc, g, i, orc.REF)
    assert bits_equal(out["obs"], g["obs"][i])
    assert bits_equal(out["m"], g["m_t"][i])
    assert bits_equal(out["v"], g["v_t"][i])
    assert bits_equal(out["lam"], g["lambda_coef"][i])
    assert bits_equal(out["rew"].astype(np.float64), g["reward"][i])
    assert np.array_equal(out["te"], g["terminated"][i])
    assert np.array_equal(out["tr"], g["truncated"][i])


@pytest.mark.parametrize("i", range(8))
def test_pmsm_dev_mode_close(orc, i):
    """Device formulas (x*x, (float)pow(double)) vs glibc powf: states/obs identical
    (no power on the state path), reward within rel 1e-5."""
    g = golden("pmsm")
    a = _run_pmsm(orc, g, i, orc.REF)
    b = _run_pmsm(orc, g, i, orc.DEV)
    assert bits_equal(a["obs"], b["obs"])
    assert np.array_equal(a["te"], b["te"])
    fin = np.isfinite(a["rew"])
    np.testing.assert_allclose(b["rew"][fin], a["rew"][fin], rtol=1e-5, atol=0)


def _run_hr(orc, g, i, mode, dtype=np.float64):
    st = g["init"][i, :6].astype(dtype).reshape(1, 6).copy()
    fa = np.zeros((1, 2), np.float32)
    obs, rew, te = [], [], []
    with np.errstate(all="ignore"):
        for k in range(g["obs"].shape[1]):
            o, r, t = orc.hr_step(st, fa, g["actions"][i, k][None], g["noise"][i, k][None].astype(dtype),
                                  bool(g["add_noise"][i]), bool(g["add_filter"][i]), mode)
            obs.append(o[0].copy())
            rew.append(r[0])
            te.append(t[0])
    return np.array(obs), np.array(rew), np.array(te)


@pytest.mark.parametrize("i", range(8))
def test_hr_golden_bitexact(orc, i):
    """lorenz_env_try.py:49-179: RK4 fp64 with glibc pow, filter, injected noise."""
    g = golden("hr")
    assert bits_equal(orc.hr_reset_obs(g["init"][i, :6].reshape(1, 6))[0].astype(np.float32),
                      g["obs0"][i])
    o, r, t = _run_hr(orc, g, i, orc.REF)
    assert bits_equal(o.astype(np.float32), g["obs"][i])
    assert bits_equal(r, g["reward"][i])
    assert np.array_equal(t, g["terminated"][i])


@pytest.mark.parametrize("i", range(8))
def test_hr_dev_mode_close(orc, i):
    """Correctly rounded x^2 / x^3 (device) vs glibc pow (reference): the fp64
    trajectories stay within 1e-9 relative over 1000 RK4 steps."""
    g = golden("hr")
    oa, ra, ta = _run_hr(orc, g, i, orc.REF)
    ob, rb, tb = _run_hr(orc, g, i, orc.DEV)
    np.testing.assert_allclose(ob, oa, rtol=1e-9, atol=1e-12)
    np.testing.assert_allclose(rb, ra, rtol=1e-9, atol=1e-12)
    assert np.array_equal(ta, tb)


def test_philox_known_answer(orc):
    """Philox4x32-10 known-answer vectors (Salmon et al., SC'11, Random123 kat_vectors)."""
    assert orc.philox([0, 0, 0, 0], [0, 0]) == [0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8]
    assert orc.philox([0xFFFFFFFF] * 4, [0xFFFFFFFF] * 2) == [0x408F276D, 0x41C83B0E, 0xA20BC7C6,
                                                             0x6D5451FD]
    assert orc.philox([0x243F6A88, 0x85A308D3, 0x13198A2E, 0x03707344],
                      [0xA4093822, 0x299F31D0]) == [0xD16CFE09, 0x94FDCCEB, 0x5001E420,
                                                     0x24126EA1]


def test_reset_draw_ranges(orc):
    for sysname, lo, hi in (("l3", -30, 30), ("l4", 0, 5), ("pmsm", -30, 30)):
        for dt in (np.float32, np.float64):
            v = orc.reset_draw(sysname, dt, 4096, 0, 7, 3)
            assert v.min() >= lo and v.max() < hi
            assert abs(v.mean() - (lo + hi) / 2) < 0.05 * (hi - lo)
    v = orc.reset_draw("hr", np.float64, 4096, 0, 7, 3, add_noise=True)
    assert v[:, :6].min() >= -10 and v[:, :6].max() < 20 and 0 <= v[:, 6].min() and v[:, 6].max() < 2
    assert (orc.reset_draw("hr", np.float64, 8, 0, 7, 3, add_noise=True, eval_mode=True)[:, 6] == 2).all()
    assert (orc.reset_draw("hr", np.float32, 8, 0, 7, 3)[:, 6] == 0).all()
    # keyed by global id: a shard reproduces the slice of the full draw
    full = orc.reset_draw("l3", np.float32, 100, 0, 11, 5)
    assert np.array_equal(orc.reset_draw("l3", np.float32, 50, 50, 11, 5), full[50:])


# ----------------------------------------------------------------- legacy variants
def _legacy_init(g, key):
    return np.ascontiguousarray(g[key + "_init"], np.float64)


@pytest.mark.parametrize("key", ["t1", "t2", "tp", "sc"])
def test_legacy_golden_bitexact(orc, key):
    """The unregistered variants (lorenz_env_transient1/2.py, lorenz_env_transient_pmsm.py,
    lorenz_singlecontrol.py), fp64: reset observation and every step bit-exact against
    the reference's own outputs (tests/golden/legacy.npz), noise injected for TP / SC."""
    g = golden("legacy")
    st = _legacy_init(g, key)
    assert bits_equal(orc.legacy_reset_obs(key, st), g[key + "_obs0"])
    acts = g[key + "_actions"]
    with np.errstate(all="ignore"):
        for k in range(g[key + "_obs"].shape[1]):
            a = None if key == "sc" else acts[:, k]
            nz = g[key + "_noise"][:, k] if key in ("tp", "sc") else None
            o, r, d = orc.legacy_step(key, st, a, nz)
            assert bits_equal(o, g[key + "_obs"][:, k]), k
            assert bits_equal(r, g[key + "_reward"][:, k]), k
            assert np.array_equal(d, g[key + "_done"][:, k]), k


def test_legacy_done_accumulators_never_fire(orc):
    """'t == T' on the reference's float accumulators (t1 :99-100, t2 :230-235,
    tp :124-129, sc :166-169) never holds exactly: t_done_step = -1."""
    for key in ("t1", "t2", "tp", "sc"):
        p = orc.PARAMS[key]
        assert orc.t_done_step(p[3], p[5]) == -1, key


def test_ref_loop_restatement_matches_reference_fixture():
    """oracle/ref_loop.py (bench.py's reference-semantics CPU baseline) reproduces the
    reference's dynamic.py trajectories bit for bit (fixture from the reference)."""
    import numpy as np

    from conftest import golden
    from oracle.ref_loop import LorenzRefEnv

    g = golden("l3")
    for e in range(g["x0"].shape[0]):
        env = LorenzRefEnv(g["x0"][e])
        with np.errstate(all="ignore"):
            for k in range(200):
                obs, rew, done, _ = env.step(g["actions"][e, k])
                assert np.array_equal(obs, g["obs"][e, k], equal_nan=True)
                assert (rew == g["reward"][e, k]) or (np.isnan(rew) and np.isnan(g["reward"][e, k]))
                assert done == g["done"][e, k]
