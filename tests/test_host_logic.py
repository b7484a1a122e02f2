"""Host logic above the kernel, on CPU: the SB3 VecEnv contract (infos, terminal
observations, TimeLimit.truncated, lazy infos, get/set_attr, env_method, seed), the
TimeLimit wrapper, the env-id registry and the shard arithmetic.  The kernel is
replaced by the oracle-driven FakeBackend (tests/fake_backend.py)."""
import numpy as np
import pytest

import gym_lorenz
from fake_backend import FakeBackend
from gym_lorenz import parallel
from gym_lorenz.compat import Box, TimeLimit
from gym_lorenz.vec_env import LazyInfos, LorenzVecEnv


def test_registry_matches_reference_registration():
    """gym_lorenz/__init__.py:4-23 of the reference + the restored historical id."""
    s = gym_lorenz.SPECS
    assert s["lorenz_try-v0"].max_episode_steps == 5000
    assert s["lorenz_try-v0"].entry_point == "gym_lorenz.envs:HRSyncEnv"
    assert s["lorenz_pmsm-v0"].max_episode_steps == 2000
    assert s["lorenz_pmsm-v0"].entry_point == "gym_lorenz.envs:PMSM_Sync_Env"
    assert s["lorenz_transient-v0"].max_episode_steps == 4000
    for spec in s.values():
        assert spec.reward_threshold == 1e50
        assert spec.entry_class() is not None
    obs, act = s["lorenz_try-v0"].spaces()
    assert obs.shape == (6,) and act.shape == (2,) and act.dtype == np.float32
    assert float(obs.low.min()) == -1.0  # HR obs space is Box(-1, 1) (lorenz_env_try.py:31)
    _, act = s["lorenz_dynamic-v0"].spaces()
    assert act.shape == (3,) and float(act.high.max()) == 500.0
    with pytest.raises(KeyError):
        gym_lorenz.spec_for("nope-v0")


def test_vecenv_step_wait_contract():
    n, L = 64, 5
    be = FakeBackend("lorenz3", n, seed=2, max_episode_steps=L)
    v = LorenzVecEnv("lorenz_dynamic-v0", n, backend=be, lazy_infos=False)
    obs = v.reset()
    assert obs.shape == (n, 6) and obs.dtype == np.float32
    a = np.random.default_rng(0).uniform(-1, 1, (n, 3)).astype(np.float32)
    for k in range(L):
        obs, rew, dones, infos = v.step(a)
        assert rew.shape == (n,) and rew.dtype == np.float32 and dones.dtype == bool
        assert isinstance(infos, list) and len(infos) == n
        if k < L - 1:
            assert not dones.any() and all(i == {} for i in infos)
    assert dones.all()
    for i in range(n):
        assert infos[i]["TimeLimit.truncated"] is True
        assert infos[i]["terminal_observation"].shape == (6,)
    # returned obs are the post-reset observations, terminal obs the pre-reset ones
    assert not np.array_equal(obs[0], infos[0]["terminal_observation"])


def test_vecenv_termination_is_not_truncation():
    n = 16
    be = FakeBackend("pmsm", n, seed=4)
    v = LorenzVecEnv("lorenz_pmsm-v0", n, backend=be)
    v.reset()
    init = be._draw(0)
    init[::2, 3:] += np.array([400, -400, 300], np.float32)
    be.reset(init=init)
    obs, rew, dones, infos = v.step(np.zeros((n, 2), np.float32))
    assert dones[::2].all() and not dones[1::2].any()
    assert infos[0]["TimeLimit.truncated"] is False
    assert "terminal_observation" in infos[0] and infos[1] == {}
    assert (rew[::2] == -1000.0).all()


def test_lazy_infos_sequence():
    li = LazyInfos(5, {3: {"terminal_observation": 1}})
    assert len(li) == 5 and li[0] == {} and li[3]["terminal_observation"] == 1
    li[1]["episode"] = {"r": 1.0}  # VecMonitor-style mutation persists
    assert li[1]["episode"]["r"] == 1.0
    assert li[-2]["terminal_observation"] == 1
    assert [d for d in li][4] == {}
    assert li.done_indices() == [3]
    with pytest.raises(IndexError):
        li[5]


def test_vecenv_attrs_methods_seed():
    n = 8
    be = FakeBackend("pmsm", n, seed=1)
    v = LorenzVecEnv("lorenz_pmsm-v0", n, backend=be)
    v.reset()
    s1 = v.get_attr("state1")
    assert len(s1) == n and s1[0].shape == (3,)
    v.set_attr("state1", [1.0, 2.0, 3.0], indices=[2])
    assert np.array_equal(v.get_attr("state1", indices=2)[0], [1, 2, 3])
    after = v.get_attr("state1")
    for i in range(n):  # only env 2 was written
        if i != 2:
            assert np.array_equal(after[i], s1[i])
    got = v.get_attr("state1", indices=[5, 2])  # in the order asked
    assert np.array_equal(got[0], s1[5]) and np.array_equal(got[1], [1, 2, 3])
    with pytest.raises(ValueError):
        v.set_attr("state1", [1.0, 2.0], indices=[2])  # wrong component count
    assert v.get_attr("lambda_coef")[0] == 0.0
    assert v.env_is_wrapped(object) == [False] * n
    assert v.seed(123)[:2] == [123, 124] and be.seed == 123
    with pytest.raises(AttributeError):
        v.get_attr("no_such_attr")
    assert v.get_attr("observation_space")[0].shape == (6,)


def test_time_limit_wrapper_both_apis():
    class Old:
        observation_space = action_space = None

        def reset(self):
            return 0

        def step(self, a):
            return 0, 1.0, False, {}

        @property
        def unwrapped(self):
            return self

    class New(Old):
        def reset(self, **kw):
            return 0, {}

        def step(self, a):
            return 0, 1.0, False, False, {}

    w = TimeLimit(Old(), 3)
    w.reset()
    outs = [w.step(0) for _ in range(3)]
    assert [o[2] for o in outs] == [False, False, True]
    assert outs[-1][3]["TimeLimit.truncated"] is True
    w = TimeLimit(New(), 2)
    w.reset()
    assert w.step(0)[3] is False and w.step(0)[3] is True


def test_box_fallback():
    b = Box(-2, 2, shape=(3,), dtype=np.float32)
    x = b.sample()
    assert x.shape == (3,) and x.dtype == np.float32 and b.contains(x)
    assert not b.contains(np.array([3, 0, 0], np.float32))


@pytest.mark.parametrize("n,w", [(1048576, 8), (10, 3), (7, 8), (1, 1), (65536, 2)])
def test_shard_bounds_partition(n, w):
    spans = [parallel.shard_bounds(n, r, w) for r in range(w)]
    assert sum(c for _, c in spans) == n
    off = 0
    for s, c in spans:
        assert s == off
        off += c
    assert max(c for _, c in spans) - min(c for _, c in spans) <= 1


def test_fake_backend_shards_reproduce_full_run():
    """The RNG is keyed by global env id: per-env trajectories do not depend on how
    the env axis is split (the property the GPU shard test checks on device)."""
    n, T = 100, 12
    full = FakeBackend("lorenz3", n, seed=7, max_episode_steps=5)
    parts = [FakeBackend("lorenz3", c, seed=7, global_env_offset=s, max_episode_steps=5)
             for s, c in (parallel.shard_bounds(n, r, 3) for r in range(3))]
    a = np.random.default_rng(1).uniform(-1, 1, (T, n, 3)).astype(np.float32)
    of = full.reset().numpy().copy()
    op = np.concatenate([p.reset().numpy() for p in parts])
    assert np.array_equal(of, op)
    off = [parallel.shard_bounds(n, r, 3) for r in range(3)]
    for k in range(T):
        of = full.step(a[k])[0].numpy().copy()
        op = np.concatenate([p.step(a[k][s:s + c])[0].numpy() for p, (s, c) in zip(parts, off)])
        assert np.array_equal(of, op)
