"""The per-env drop-in classes' host logic on CPU: with the kernel replaced by the
oracle in REF mode (FakeSingleCore), seeding exactly as the reference's own scripts
do reproduces the reference's golden trajectories bit for bit -- i.e. the classes
consume np.random / self.np_random in the reference's order and wire the spaces,
attributes and return types the same way."""
import numpy as np
import pytest

import gym_lorenz
from conftest import bits_equal, golden
from fake_backend import FakeSingleCore
from gym_lorenz.envs import dynamic, lorenz_env_transient, lorenz_env_try, lorenz_env_try_pmsm


@pytest.fixture(autouse=True)
def fake_core(monkeypatch):
    for mod in (dynamic, lorenz_env_transient, lorenz_env_try, lorenz_env_try_pmsm):
        monkeypatch.setattr(mod, "SingleEnvCore", FakeSingleCore)


def test_dynamic_class_reproduces_reference():
    g = golden("l3")
    for i in (0, 7, 12):  # incl. a divergent seed
        np.random.seed(int(g["seeds"][i]))
        env = gym_lorenz.LorenzDynamicEnv()
        o = env.reset()
        assert o.dtype == np.float64 and o.shape == (6,) and bits_equal(o, g["obs0"][i])
        assert env.observation_space.shape == (6,) and env.action_space.shape == (3,)
        assert env.action_space.dtype == np.float32 and float(env.action_space.high[0]) == 500.0
        for k in range(300):
            o, r, d, info = env.step(g["actions"][i, k])
            assert bits_equal(o, g["obs"][i, k]) and bits_equal(r, g["reward"][i, k])
            assert d is False and info == {}
        assert env.t == pytest.approx(3.0) and env.u1 == np.clip(g["actions"][i, 299, 0], -500, 500)


def test_l4_class_reproduces_reference_via_make():
    g = golden("l4")
    np.random.seed(100 + 3)
    env = gym_lorenz.make("lorenz_transient-v0")  # TimeLimit(4000), classic 4-tuple API
    o = env.reset()
    assert bits_equal(o, g["obs0"][3])
    for k in range(400):
        o, r, d, info = env.step(g["actions"][3, k])
        assert bits_equal(o, g["obs"][3, k]) and bits_equal(r, g["reward"][3, k])
    m, s = env.unwrapped.get_current2()
    assert np.isfinite(m) and np.isfinite(s)


@pytest.mark.parametrize("i", [0, 2, 5, 8])
def test_pmsm_class_reproduces_reference(i):
    g = golden("pmsm")
    env = gym_lorenz.make("lorenz_pmsm-v0", alpha=float(g["alpha"][i]),
                          add_noise=bool(g["add_noise"][i]))
    o, info = env.reset(seed=int(g["seeds"][i]))
    if g["injected"][i]:  # CS-5 style injection through the attribute setter
        env.unwrapped.state2 = g["init"][i, 0, 3:]
    else:
        assert bits_equal(o, g["obs0"][i, 0]) and info == {}
    T = int(g["reset_at"])
    for k in range(T + 50):
        if k == T:
            o, _ = env.reset()
            assert bits_equal(o, g["obs0"][i, 1])
        o, r, te, tr, info = env.step(g["actions"][i, k])
        assert bits_equal(o, g["obs"][i, k]), k
        assert bits_equal(np.float64(r), g["reward"][i, k]), k
        assert te == g["terminated"][i, k] and tr == g["truncated"][i, k]
    assert env.unwrapped.current_step == 50
    assert bits_equal(np.float32(env.unwrapped.lambda_coef), g["lambda_coef"][i, T + 49])


@pytest.mark.parametrize("i", [0, 3, 5, 7])
def test_hr_class_reproduces_reference(i):
    g = golden("hr")
    np.random.seed(10 + i)
    env = gym_lorenz.HRSyncEnv(add_noise=bool(g["add_noise"][i]), eval_mode=bool(g["eval_mode"][i]),
                               add_filter=bool(g["add_filter"][i]))
    o, _ = env.reset(seed=10 + i)
    assert o.dtype == np.float32 and bits_equal(o, g["obs0"][i])
    assert env.sigma == g["init"][i, 6]
    for k in range(400):
        o, r, te, tr, _ = env.step(g["actions"][i, k])
        assert bits_equal(o, g["obs"][i, k]) and bits_equal(np.float64(r), g["reward"][i, k])
        assert te == g["terminated"][i, k] and tr is False


def test_hr_derivatives_helper_is_the_reference_formula():
    from gym_lorenz.envs import hr_derivatives

    d = hr_derivatives(np.array([0.5, -1.0, 2.0]), 3.0, -2.0, 1.0, 3.0, 1.0, 5.0, 0.006, 4.0, 3.2, -1.6)
    x1, x2, x3 = 0.5, -1.0, 2.0
    assert np.array_equal(d, [x2 - x1 ** 3 + 3 * x1 ** 2 - x3 + 3.2, 1 - 5 * x1 ** 2 - x2 + 3.0,
                              0.006 * (4 * (x1 + 1.6) - x3) - 2.0])


def test_pmsm_get_derivatives_helper_promotes_like_reference():
    env = gym_lorenz.PMSM_Sync_Env()
    st = np.array([1.5, -2.25, 3.0], np.float32)
    d = env._get_derivatives(st, [0.5, -0.5], [0.1, 0.2, 0.3])
    assert d.dtype == np.float32
    assert d[0] == np.float32(-st[0] + st[1] * st[2] + np.float32(0.5) + 0.1)


@pytest.mark.parametrize("key,cls", [("t1", "LorenzTransient1Env"), ("t2", "LorenzTransient2Env"),
                                     ("tp", "LorenzTransientPmsmEnv"),
                                     ("sc", "LorenzSingleControlEnv")])
def test_legacy_classes_reproduce_reference(monkeypatch, key, cls):
    """The unregistered variants: np.random.seed(s) + reset() + step() reproduce the
    reference's golden trajectories (the host consumes the global RNG as the reference
    does -- incl. the unused per-step normal draws of t1 / t2 -- and injects tp / sc's
    process noise)."""
    from gym_lorenz.envs import legacy

    monkeypatch.setattr(legacy, "SingleEnvCore", FakeSingleCore)
    g = golden("legacy")
    seed0 = {"t1": 300, "t2": 310, "tp": 320, "sc": 330}[key]
    for i in (0, 1):
        np.random.seed(seed0 + i)
        env = getattr(legacy, cls)()
        o = env.reset()
        assert bits_equal(o, g[key + "_obs0"][i])
        for k in range(200):
            if key == "sc":
                o, r, d, info = env.step()
            else:
                o, r, d, info = env.step(g[key + "_actions"][i, k])
            assert bits_equal(o, g[key + "_obs"][i, k]), k
            assert bits_equal(r, g[key + "_reward"][i, k]), k
            assert d == bool(g[key + "_done"][i, k]) and info == {}
        assert env.observation_space.shape == (8 if key == "t2" else 6,)
        m, s = env._get_current()
        assert np.isfinite(m)
