"""Generate the golden fixtures under tests/golden/ by running the REFERENCE envs.

Test infrastructure only: this script imports the reference env modules from
/root/reference (read-only) in the build container, with gym / gymnasium /
stable_baselines3 stubbed in sys.modules (none of them is installed and the
reference's hot path uses none of their arithmetic -- SURVEY.md §8c). The
reference never travels to the GPU box; only the .npz files written here do.

Run:  python tests/golden/make_golden.py        (needs /root/reference)

Fixtures (all arrays are what the reference itself returned / held):
  l3.npz    dynamic.py:5 lorenzEnv_transient      (Euler dt=0.01, fp64)
  l4.npz    lorenz_env_transient.py:247 lorenzEnv_transient (4-state, fp64)
  pmsm.npz  lorenz_env_try_pmsm.py:7 PMSM_Sync_Env (fp32, Adam dual)
  hr.npz    lorenz_env_try.py:13 HRSyncEnv        (RK4 dt=0.001, fp64)
  legacy.npz  the unregistered variants (fp64): lorenz_env_transient1.py:18 (t1_*),
            lorenz_env_transient2.py:115 (t2_*), lorenz_env_transient_pmsm.py:17
            (tp_*), lorenz_singlecontrol.py:97 (sc_*)
"""
import importlib.util
import os
import sys
import types

import numpy as np

sys.dont_write_bytecode = True  # never write .pyc into /root/reference
REF_ENVS = "/root/reference/code/gym-lorenz/gym_lorenz/envs"
OUT = os.path.dirname(os.path.abspath(__file__))


# --------------------------------------------------------------------------- stubs
class _Box:
    def __init__(self, low, high, shape=None, dtype=np.float32):
        self.low, self.high, self.shape, self.dtype = low, high, shape, np.dtype(dtype)


class _OldEnv:  # classic gym.Env: no seeding on reset
    metadata = {}


class _GymnasiumEnv:  # gymnasium.Env.reset(seed) seeding semantics
    _np_random = None

    @property
    def np_random(self):
        if self._np_random is None:
            self._np_random = np.random.default_rng()
        return self._np_random

    def reset(self, seed=None, options=None):
        if seed is not None:
            # gymnasium.utils.seeding.np_random(seed) ==
            # Generator(PCG64(SeedSequence(seed))) == default_rng(seed)
            self._np_random = np.random.default_rng(seed)


def _install_stubs():
    # the legacy env modules import plotting / ODE helpers they never call
    for name in ("matplotlib", "matplotlib.pyplot", "mpl_toolkits", "mpl_toolkits.mplot3d"):
        m = types.ModuleType(name)
        m.Axes3D = object
        sys.modules.setdefault(name, m)
    spaces = types.ModuleType("spaces")
    spaces.Box = _Box
    for name, env in (("gym", _OldEnv), ("gymnasium", _GymnasiumEnv)):
        m = types.ModuleType(name)
        m.Env = env
        m.spaces = spaces
        m.error = types.ModuleType(name + ".error")
        m.utils = types.ModuleType(name + ".utils")
        m.utils.seeding = types.ModuleType(name + ".utils.seeding")
        sys.modules[name] = m
        sys.modules[name + ".spaces"] = spaces
        sys.modules[name + ".error"] = m.error
        sys.modules[name + ".utils"] = m.utils
        sys.modules[name + ".utils.seeding"] = m.utils.seeding
    sb3 = types.ModuleType("stable_baselines3")
    sb3.PPO = object
    sys.modules["stable_baselines3"] = sb3


def _load(fname, modname):
    spec = importlib.util.spec_from_file_location(modname, os.path.join(REF_ENVS, fname))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


# --------------------------------------------------------------------------- L3
def gen_l3(mod, n_steps=1000):
    """dynamic.py: x0 from np.random.seed(s) + reset(); float32 actions."""
    # seeds 0..11 plus two seeds whose trajectories overflow to inf/NaN
    seeds = list(range(12))
    div = []
    for s in range(12, 3000):
        np.random.seed(s)
        e = mod.lorenzEnv_transient()
        e.reset()
        with np.errstate(all="ignore"):
            for _ in range(300):
                o, r, d, _i = e.step(np.zeros(3, np.float32))
        if not np.all(np.isfinite(o)):
            div.append(s)
        if len(div) == 2:
            break
    seeds += div
    n = len(seeds)
    arng = np.random.default_rng(1)
    acts = np.zeros((n, n_steps, 3), np.float32)
    kinds = []
    for i in range(n):
        if i < 4 or i >= 12:
            kinds.append("zero")
        elif i < 10:
            acts[i] = arng.uniform(-1, 1, (n_steps, 3)).astype(np.float32)
            kinds.append("u11")
        else:  # exercise the +-500 clip on the first steps, then small actions
            acts[i] = arng.uniform(-1, 1, (n_steps, 3)).astype(np.float32)
            acts[i, :3] = arng.uniform(-700, 700, (3, 3)).astype(np.float32)
            kinds.append("clip")
    obs0 = np.zeros((n, 6))
    x0 = np.zeros((n, 3))
    obs = np.zeros((n, n_steps, 6))
    rew = np.zeros((n, n_steps))
    done = np.zeros((n, n_steps), bool)
    for i, s in enumerate(seeds):
        np.random.seed(s)
        e = mod.lorenzEnv_transient()
        o = e.reset()
        obs0[i] = o
        x0[i] = e.state1
        with np.errstate(all="ignore"):
            for k in range(n_steps):
                o, r, d, _ = e.step(acts[i, k])
                obs[i, k], rew[i, k], done[i, k] = o, r, d
    # the reference's done accumulator, for the done_mode=REFERENCE emulation
    t, t_hist = 0, []
    for _ in range(1200):
        t = t + 0.01
        t_hist.append(t)
    np.savez_compressed(os.path.join(OUT, "l3.npz"), seeds=np.array(seeds), x0=x0, obs0=obs0,
                        actions=acts, obs=obs, reward=rew, done=done, t_hist=np.array(t_hist))
    print("l3", n, "envs; divergent seeds", div)


# --------------------------------------------------------------------------- L4
def gen_l4(mod, n_steps=1000):
    n = 12
    arng = np.random.default_rng(2)
    acts = arng.uniform(-2.5, 2.5, (n, n_steps, 3)).astype(np.float32)
    init = np.zeros((n, 8))
    obs0 = np.zeros((n, 8))
    obs = np.zeros((n, n_steps, 8))
    rew = np.zeros((n, n_steps))
    done = np.zeros((n, n_steps), bool)
    for i in range(n):
        np.random.seed(100 + i)
        e = mod.lorenzEnv_transient()
        o = e.reset()
        obs0[i] = o
        init[i, :4] = e.state1
        init[i, 4:] = e.state2[:4]
        with np.errstate(all="ignore"):
            for k in range(n_steps):
                o, r, d, _ = e.step(acts[i, k])
                obs[i, k], rew[i, k], done[i, k] = o, r, d
    np.savez_compressed(os.path.join(OUT, "l4.npz"), init=init, obs0=obs0, actions=acts, obs=obs,
                        reward=rew, done=done)
    print("l4", n, "envs")


# --------------------------------------------------------------------------- PMSM
def gen_pmsm(mod, n_steps=2000, n_steps2=200):
    """seed s: reset(seed=s), 2000 steps (own truncation), reset(), 200 more.
    Lambda/Adam state carries over the reset (lorenz_env_try_pmsm.py:59-75)."""
    cases = [(s, noise, alpha) for s, noise, alpha in
             [(0, False, 0.5), (1, False, 0.5), (2, True, 0.5), (3, True, 0.5),
              (4, False, 0.25), (5, True, 0.14), (6, True, 0.33), (7, False, 0.11),
              (8, True, 0.5)]]
    n = len(cases)
    T = n_steps + n_steps2
    arng = np.random.default_rng(3)
    acts = arng.uniform(-1.2, 1.2, (n, T, 2)).astype(np.float32)
    # a few envs drive hard to reach the error_sum > 1000 termination branch
    acts[1, :50] = 1.2
    init = np.zeros((n, 2, 6), np.float32)
    noise = np.zeros((n, T, 3))
    obs0 = np.zeros((n, 2, 6), np.float32)
    obs = np.zeros((n, T, 6), np.float32)
    rew = np.zeros((n, T))
    term = np.zeros((n, T), bool)
    trunc = np.zeros((n, T), bool)
    lam = np.zeros((n, T), np.float32)
    mt = np.zeros((n, T), np.float32)
    vt = np.zeros((n, T), np.float32)
    s1 = np.zeros((n, T, 3), np.float32)
    s2 = np.zeros((n, T, 3), np.float32)
    for i, (s, add_noise, alpha) in enumerate(cases):
        e = mod.PMSM_Sync_Env(alpha=alpha, add_noise=add_noise)
        replay = np.random.default_rng(s)
        o, _ = e.reset(seed=s)
        obs0[i, 0] = o
        init[i, 0, :3], init[i, 0, 3:] = e.state1, e.state2
        a = replay.uniform(-30, 30, 3).astype(np.float32)
        b = replay.uniform(-30, 30, 3).astype(np.float32)
        assert np.array_equal(a, e.state1) and np.array_equal(b, e.state2)
        if s == 8:  # CS-5 style state injection: push the slave far away so that
            # error_sum > 1000 fires the termination branch (:174-176)
            e.state2 = (e.state2 + np.array([400, -400, 300], np.float32)).astype(np.float32)
            init[i, 0, 3:] = e.state2
        for k in range(T):
            if k == n_steps:
                o, _ = e.reset()
                obs0[i, 1] = o
                init[i, 1, :3], init[i, 1, 3:] = e.state1, e.state2
                replay.uniform(-30, 30, 3)
                replay.uniform(-30, 30, 3)
            noise[i, k] = replay.normal(0, 3, 3)
            o, r, te, tr, _ = e.step(acts[i, k])
            obs[i, k], rew[i, k], term[i, k], trunc[i, k] = o, r, te, tr
            lam[i, k], mt[i, k], vt[i, k] = e.lambda_coef, e.m_t, e.v_t
            s1[i, k], s2[i, k] = e.state1, e.state2
    np.savez_compressed(os.path.join(OUT, "pmsm.npz"),
                        seeds=np.array([c[0] for c in cases]), injected=np.array([c[0] == 8 for c in cases]),
                        add_noise=np.array([c[1] for c in cases]),
                        alpha=np.array([c[2] for c in cases]), reset_at=np.array(n_steps),
                        init=init, obs0=obs0, actions=acts, noise=noise, obs=obs, reward=rew,
                        terminated=term, truncated=trunc, lambda_coef=lam, m_t=mt, v_t=vt,
                        state1=s1, state2=s2)
    print("pmsm", n, "envs; terminations", term.sum(), "truncations", trunc.sum())


# --------------------------------------------------------------------------- HR
def gen_hr(mod, n_steps=1000):
    cases = [(10, False, False, False), (11, False, False, False), (12, False, False, True),
             (13, True, False, False), (14, True, False, True), (15, True, True, False),
             (16, False, False, False), (17, True, False, True)]
    n = len(cases)
    arng = np.random.default_rng(4)
    acts = arng.uniform(-1.2, 1.2, (n, n_steps, 2)).astype(np.float32)
    acts[6] = 1.0  # drive one slave hard toward the |e|>70 termination branch
    init = np.zeros((n, 7))  # master(3), slave(3), sigma
    noise = np.zeros((n, n_steps, 3))
    obs0 = np.zeros((n, 6), np.float32)
    obs = np.zeros((n, n_steps, 6), np.float32)
    rew = np.zeros((n, n_steps))
    term = np.zeros((n, n_steps), bool)
    sm = np.zeros((n, n_steps, 3))
    ss = np.zeros((n, n_steps, 3))
    for i, (s, add_noise, eval_mode, add_filter) in enumerate(cases):
        np.random.seed(s)
        e = mod.HRSyncEnv(add_noise=add_noise, eval_mode=eval_mode, add_filter=add_filter)
        o, _ = e.reset(seed=s)
        obs0[i] = o
        init[i, :3], init[i, 3:6], init[i, 6] = e.state_master, e.state_slave, e.sigma
        # replay the global MT19937 stream to recover the per-step noise draws
        st = np.random.get_state()
        np.random.seed(s)
        np.random.uniform(-10, 20, 3)
        np.random.uniform(-10, 20, 3)
        if add_noise and not eval_mode:
            np.random.uniform(0, 2)
        for k in range(n_steps):
            if add_noise:
                noise[i, k] = np.random.normal(0, e.sigma, 3)
        np.random.set_state(st)
        with np.errstate(all="ignore"):
            for k in range(n_steps):
                o, r, te, tr, _ = e.step(acts[i, k])
                obs[i, k], rew[i, k], term[i, k] = o, r, te
                sm[i, k], ss[i, k] = e.state_master, e.state_slave
    np.savez_compressed(os.path.join(OUT, "hr.npz"), add_noise=np.array([c[1] for c in cases]),
                        eval_mode=np.array([c[2] for c in cases]),
                        add_filter=np.array([c[3] for c in cases]), init=init, obs0=obs0,
                        actions=acts, noise=noise, obs=obs, reward=rew, terminated=term,
                        state_master=sm, state_slave=ss)
    print("hr", n, "envs; terminations", term.sum())


# --------------------------------------------------------------------------- legacy
def gen_legacy(n_steps=600):
    """The four unregistered variants, each env seeded through np.random.seed(s) (they
    draw from the global MT19937 stream); per-step noise recovered by replaying it."""
    import contextlib
    import io

    out = {}
    specs = {  # key: (file, module, n envs, action dim, action range, seeds)
        "t1": ("lorenz_env_transient1.py", "ref_t1", 8, 2, 1.0, 300),
        "t2": ("lorenz_env_transient2.py", "ref_t2", 8, 3, 2.5, 310),
        "tp": ("lorenz_env_transient_pmsm.py", "ref_tp", 8, 2, 2.5, 320),
        "sc": ("lorenz_singlecontrol.py", "ref_sc", 4, 0, 0.0, 330),
    }
    for key, (fname, modname, n, adim, arange, seed0) in specs.items():
        mod = _load(fname, modname)
        arng = np.random.default_rng(seed0)
        acts = arng.uniform(-arange, arange, (n, n_steps, max(adim, 1))).astype(np.float32)
        if key == "t1":  # exercise the +-10 clip on the first steps
            acts[1, :3] = np.float32(25.0)
            acts[2, :3] = np.float32(-25.0)
        if key == "t2":  # the slave diverges under +-2 * 100 forcing: keep 6 envs gentle
            acts[:6] *= np.float32(0.02)
            acts[6, :2] = np.float32(3.0)  # clip
        O = 8 if key == "t2" else 6
        NI = {"t1": 3, "t2": 8, "tp": 6, "sc": 3}[key]
        init = np.zeros((n, NI))
        obs0 = np.zeros((n, O))
        obs = np.zeros((n, n_steps, O))
        rew = np.zeros((n, n_steps))
        done = np.zeros((n, n_steps), bool)
        noise = np.zeros((n, n_steps, 3))
        for i in range(n):
            s = seed0 + i
            np.random.seed(s)
            e = mod.lorenzEnv_transient()
            with contextlib.redirect_stdout(io.StringIO()):
                o = e.reset()
            obs0[i] = o
            if key in ("t1", "sc"):
                init[i] = np.asarray(e.state1, np.float64)
            elif key == "t2":
                init[i, :4], init[i, 4:] = e.state1, np.asarray(e.state2[:4])
            else:
                init[i, :3], init[i, 3:] = e.state1, np.asarray(e.state2[:3])
            if key in ("tp", "sc"):  # the per-step N(0,3) draws, replayed
                st = np.random.get_state()
                np.random.seed(s)
                if key == "tp":
                    np.random.uniform(-10, 10, 3)
                    np.random.uniform(-10, 10, 3)
                for k in range(n_steps):
                    noise[i, k] = np.random.normal(0, 3, 3)
                np.random.set_state(st)
            with np.errstate(all="ignore"), contextlib.redirect_stdout(io.StringIO()):
                for k in range(n_steps):
                    o, r, d, _ = e.step() if key == "sc" else e.step(acts[i, k])
                    obs[i, k], rew[i, k], done[i, k] = o, r, d
        out.update({key + "_init": init, key + "_obs0": obs0, key + "_actions": acts,
                    key + "_noise": noise, key + "_obs": obs, key + "_reward": rew,
                    key + "_done": done})
        print(key, n, "envs; done", done.sum(), "nonfinite", int((~np.isfinite(obs)).sum()))
    np.savez_compressed(os.path.join(OUT, "legacy.npz"), **out)


if __name__ == "__main__":
    _install_stubs()
    if sys.argv[1:] == ["legacy"]:
        gen_legacy()
        sys.exit(0)
    gen_l3(_load("dynamic.py", "ref_dynamic"))
    gen_l4(_load("lorenz_env_transient.py", "ref_l4"))
    gen_pmsm(_load("lorenz_env_try_pmsm.py", "ref_pmsm"))
    gen_hr(_load("lorenz_env_try.py", "ref_hr"))
