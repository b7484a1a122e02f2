"""GPU: lz_resident_step (the resident one-wave step server behind the per-env
drop-in classes) against lz_step_host -- the same step body tick for tick, so the
results must be bit-identical -- including the server's idle exit + relaunch, state
access in between (which stops it), injected noise, 64-env handles, the unsupported
cases, and that it does not hold up torch work on other streams while it waits.

The drop-in class tests in test_gpu_parity.py (test_dropin_*) run through the resident
path too (it is the default) against the reference's golden fixtures."""
import os
import time

import numpy as np
import pytest
import torch

from conftest import bits_equal

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def gl():
    import gym_lorenz

    return gym_lorenz


def _pair(system, n, dtype, **kw):
    from gym_lorenz.core import BatchedEnv

    envs = []
    for _ in range(2):
        be = BatchedEnv(system, n, dtype=dtype, seed=7, autoreset=False, compact=False,
                        max_episode_steps=0, **kw)
        be.reset()
        envs.append(be)
    return envs


def _bufs(be):
    npd = np.float64 if be.tdtype == torch.float64 else np.float32
    return (np.zeros((be.num_envs, be.obs_dim), npd), np.zeros((be.num_envs,), npd),
            np.zeros((be.num_envs,), np.uint8))


def _step(fn, be, act, noise, bufs):
    import gym_lorenz._native as nat

    o, r, d = bufs
    nat.check(fn(be._h, act.ctypes.data, None if noise is None else noise.ctypes.data,
                 o.ctypes.data, r.ctypes.data, d.ctypes.data))
    return o.copy(), r.copy(), d.copy()


@pytest.mark.parametrize("system,n,dtype,kw,noise", [
    ("lorenz3", 1, "float64", {}, False),
    ("lorenz3", 64, "float32", {}, False),
    ("pmsm", 1, "float32", {"add_noise": True}, True),
    ("pmsm", 3, "float32", {"add_noise": True}, False),
    ("hr", 1, "float64", {"add_noise": True}, True),
    ("hr", 17, "float32", {"add_noise": True, "add_filter": True}, False),
    ("lorenz4", 1, "float64", {}, False),
])
def test_resident_equals_step_host(gl, system, n, dtype, kw, noise):
    import gym_lorenz._native as nat

    a, b = _pair(system, n, dtype, **kw)
    ba, bb = _bufs(a), _bufs(b)
    rng = np.random.default_rng(3)
    A = max(a.action_dim, 1)
    for k in range(400):
        act = rng.uniform(-1, 1, (n, A)).astype(np.float32)
        nz = rng.standard_normal((n, 3)) if noise else None
        x = _step(nat.lib.lz_step_host, a, act, nz, ba)
        y = _step(nat.lib.lz_resident_step, b, act, nz, bb)
        for p, q in zip(x, y):
            assert bits_equal(p, q), (system, k)
        if k == 150:  # state access in between stops the server; the next step relaunches it
            for pl in range(2):
                assert bits_equal(a.get_state(pl).cpu().numpy(), b.get_state(pl).cpu().numpy())
    # the server's register-held state goes back to the planes
    nat.check(nat.lib.lz_resident_stop(b._h))
    for pl in range(2):
        assert bits_equal(a.get_state(pl).cpu().numpy(), b.get_state(pl).cpu().numpy())
    a.close(), b.close()


def test_resident_idle_exit_and_relaunch(gl, monkeypatch):
    """With a 300 us idle limit the server exits between spaced-out requests and is
    relaunched by the next one; the trajectory (and the RNG tick) is unchanged."""
    import gym_lorenz._native as nat

    monkeypatch.setenv("LZ_RESIDENT_IDLE_US", "300")
    a, b = _pair("pmsm", 2, "float32", add_noise=True)  # device-drawn noise: tick matters
    ba, bb = _bufs(a), _bufs(b)
    rng = np.random.default_rng(5)
    for k in range(60):
        act = rng.uniform(-1, 1, (2, 2)).astype(np.float32)
        x = _step(nat.lib.lz_step_host, a, act, None, ba)
        y = _step(nat.lib.lz_resident_step, b, act, None, bb)
        for p, q in zip(x, y):
            assert bits_equal(p, q), k
        if k % 7 == 3:
            time.sleep(0.003)  # > the idle limit: the server has exited
    a.close(), b.close()


def test_resident_then_plain_calls(gl):
    """lz_step / lz_reset after resident steps see the state and tick the server left."""
    import gym_lorenz._native as nat

    a, b = _pair("hr", 4, "float64", add_noise=True)
    ba, bb = _bufs(a), _bufs(b)
    rng = np.random.default_rng(9)
    for k in range(30):
        act = rng.uniform(-1, 1, (4, 2)).astype(np.float32)
        _step(nat.lib.lz_step_host, a, act, None, ba)
        _step(nat.lib.lz_resident_step, b, act, None, bb)
    act = torch.as_tensor(rng.uniform(-1, 1, (4, 2)).astype(np.float32), device=a.device)
    oa, ra, da = a.step(act)
    ob, rb, db = b.step(act)
    torch.cuda.synchronize()
    assert bits_equal(oa.cpu().numpy(), ob.cpu().numpy())
    a.reset(), b.reset()
    for k in range(5):
        act = rng.uniform(-1, 1, (4, 2)).astype(np.float32)
        x = _step(nat.lib.lz_step_host, a, act, None, ba)
        y = _step(nat.lib.lz_resident_step, b, act, None, bb)
        for p, q in zip(x, y):
            assert bits_equal(p, q)
    a.close(), b.close()


def test_resident_unsupported(gl):
    import gym_lorenz._native as nat
    from gym_lorenz.core import BatchedEnv

    be = BatchedEnv("lorenz3", 65, autoreset=False, compact=False)
    be.reset()
    o, r, d = _bufs(be)
    act = np.zeros((65, 3), np.float32)
    st = nat.lib.lz_resident_step(be._h, act.ctypes.data, None, o.ctypes.data, r.ctypes.data,
                                  d.ctypes.data)
    assert st == nat.LZ_ERR_UNSUPPORTED
    be.close()
    be = BatchedEnv("lorenz3", 4, autoreset=True, compact=False)
    be.reset()
    o, r, d = _bufs(be)
    st = nat.lib.lz_resident_step(be._h, act.ctypes.data, None, o.ctypes.data, r.ctypes.data,
                                  d.ctypes.data)
    assert st == nat.LZ_ERR_UNSUPPORTED
    be.close()


# Run in a fresh process with a LONG idle limit (50 ms): if torch's stream shared a
# hardware queue with the polling server, torch's kernel would wait for the server's idle
# exit (~50 ms) and the 300 us gate fails loudly.  (With the default 1 ms limit a queue-
# shared server would cost only ~1 ms and a loose gate could not tell.)
_TORCH_LATENCY_CHILD = r"""
import json, sys, time
sys.path.insert(0, %(pkg)r)
import numpy as np, torch
import gym_lorenz as gl
handles = %(handles)d
x = torch.ones(1024, device="cuda")
for _ in range(3):
    x = x + 1
torch.cuda.synchronize()
envs = []
for _ in range(handles):
    e = gl.LorenzDynamicEnv()
    e.reset()
    e.step(np.zeros(3, np.float32))  # resident and polling (50 ms idle limit)
    envs.append(e)
s = torch.cuda.current_stream()
lat = []
for _ in range(30):
    for e in envs:
        e.step(np.zeros(3, np.float32))  # the server stays resident (idle clock restarts)
    t0 = time.perf_counter()
    x = x + 1
    s.synchronize()
    lat.append(time.perf_counter() - t0)
ok = float(x[0]) == 34.0
t0 = time.perf_counter()
torch.cuda.synchronize()  # device-wide: waits for the server's idle exit (50 ms)
sync_s = time.perf_counter() - t0
envs[0].step(np.zeros(3, np.float32))  # relaunched after the exit
for e in envs:
    e.close()
print(json.dumps({"lat_us": [v * 1e6 for v in lat], "ok": ok, "sync_s": sync_s}))
"""


def _torch_latency_child(handles):
    import json
    import subprocess
    import sys

    from conftest import PKG

    env = dict(os.environ, LZ_RESIDENT_IDLE_US="50000")
    r = subprocess.run([sys.executable, "-c", _TORCH_LATENCY_CHILD % {"pkg": PKG, "handles": handles}],
                       capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    return json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])


@pytest.mark.parametrize("handles", [1, 8])
def test_resident_does_not_block_torch(handles):
    """While the server (1 handle, or 8 handles = 9 waves of one launch) waits for its next
    request, a torch kernel on torch's stream completes in <= 300 us -- it is not queued
    behind the polling launch (own non-blocking stream, own hardware queue) -- measured in a
    fresh process whose server only exits after 50 ms idle; a device-wide synchronize waits
    for that idle exit, then the next step relaunches the server."""
    d = _torch_latency_child(handles)
    lat = sorted(d["lat_us"])
    print("torch add + stream sync while %d handle(s) resident: median %.0f us, max %.0f us"
          % (handles, lat[len(lat) // 2], lat[-1]))
    assert d["ok"]
    assert lat[len(lat) // 2] <= 300, lat
    assert lat[-1] <= 5000, lat  # never the server's 50 ms idle exit
    assert 0.03 < d["sync_s"] < 1.0, d["sync_s"]  # device-wide sync did wait for the exit


def test_dropin_resident_matches_step_host(gl, monkeypatch):
    """The drop-in class with LZ_RESIDENT=0 (lz_step_host) and the default (resident)."""
    outs = []
    for flag in ("0", "1"):
        monkeypatch.setenv("LZ_RESIDENT", flag)
        env = gl.make("lorenz_pmsm-v0", alpha=0.5, add_noise=True)
        o, _ = env.reset(seed=11)
        rng = np.random.default_rng(2)
        traj = [o]
        for k in range(200):
            o, r, te, tr, _ = env.step(rng.uniform(-1, 1, 2).astype(np.float32))
            traj.append(np.concatenate([o, [r, te, tr]]).astype(np.float64))
        env.close()
        outs.append(traj)
    for p, q in zip(*outs):
        assert bits_equal(np.asarray(p), np.asarray(q))


@pytest.mark.parametrize("stepper", ["1", "0"])
@pytest.mark.parametrize("noise", [False, True])
def test_dropin_step_after_close_raises(gl, monkeypatch, stepper, noise):
    """the drop-in's fast paths (C stepper, prebuilt ctypes args) drop the
    handle on close(): a later step() raises LorenzEnvError(LZ_ERR_INVALID) instead of
    reaching the freed handle."""
    from gym_lorenz import _native as nat

    monkeypatch.setenv("LZ_STEPPER", stepper)
    env = gl.make("lorenz_pmsm-v0", alpha=0.5, add_noise=noise)
    env.reset(seed=3)
    env.step(np.zeros(2, np.float32))
    env.close()
    with pytest.raises(nat.LorenzEnvError) as ei:
        env.unwrapped.step(np.zeros(2, np.float32))
    assert ei.value.status == nat.LZ_ERR_INVALID


@pytest.mark.parametrize("close", [False, True])
def test_process_exit_with_live_server(close):
    """A script that exits while the server is resident (no close(): the atexit hook
    posts the stop command) or after close() ends cleanly."""
    import subprocess
    import sys

    from conftest import ROOT

    code = ("import sys; sys.path.insert(0, %r)\n"
            "import numpy as np, gym_lorenz as gl\n"
            "e = gl.make('lorenz_pmsm-v0'); e.reset(seed=1)\n"
            "for _ in range(100): e.step(np.zeros(2, np.float32))\n"
            "%s\n"
            "print('ok')\n" % (ROOT + "/gym-lorenz_amd", "e.close()" if close else "pass"))
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and "ok" in r.stdout, r.stderr[-2000:]


def test_resident_refused_under_capture(gl):
    """A resident step is a synchronous host round trip: refused while the handle's
    stream is being captured into a hipGraph."""
    import ctypes

    import gym_lorenz._native as nat
    from gym_lorenz.core import BatchedEnv

    be = BatchedEnv("lorenz3", 1, autoreset=False, compact=False)
    be.reset()
    torch.cuda.synchronize()
    o, r, d = _bufs(be)
    act = np.zeros((1, 3), np.float32)
    s = torch.cuda.Stream()
    nat.check(nat.lib.lz_set_stream(be._h, ctypes.c_void_p(s.cuda_stream)))
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        torch.zeros(1, device="cuda")  # keep the capture non-empty
        st = nat.lib.lz_resident_step(be._h, act.ctypes.data, None, o.ctypes.data,
                                      r.ctypes.data, d.ctypes.data)
    assert st == nat.LZ_ERR_STATE
    nat.check(nat.lib.lz_set_stream(be._h, ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)))
    _step(nat.lib.lz_resident_step, be, act, None, (o, r, d))  # fine outside the capture
    be.close()


def _plane_host(be, p):
    import gym_lorenz._native as nat

    npdt = {torch.float64: np.float64, torch.float32: np.float32, torch.int32: np.int32}
    out = np.zeros((be.num_envs,), npdt[be.plane_dtype(p)])
    nat.check(nat.lib.lz_resident_read_state(be._h, int(p), out.ctypes.data))
    return out


_MIX = [("lorenz3", "float64", {}, False), ("pmsm", "float32", {"add_noise": True}, True),
        ("hr", "float64", {"add_noise": True}, False), ("lorenz4", "float64", {}, False),
        ("lorenz4", "float32", {}, False), ("hr", "float32", {"add_noise": True, "add_filter": True}, True),
        ("lorenz3", "float32", {}, False), ("pmsm", "float32", {"add_noise": True}, False)]


def test_resident_eight_handles_round_robin(gl):
    """A DummyVecEnv of 8 drop-in envs (code/train.py:98-100 with several env fns, one
    step() call per env in turn): 8 handles of mixed systems / dtypes share ONE resident
    launch (one wave each).  Every handle stays bit-identical to its lz_step_host twin,
    and the published states (lz_resident_read_state, code/lorenz_pmsm/test_evaluate.py:
    123-125 reads them after every step) equal the twin's planes while the server runs."""
    import gym_lorenz._native as nat

    pairs = [_pair(s, 1, dt, **kw) for s, dt, kw, _ in _MIX]
    bufs = [(_bufs(a), _bufs(b)) for a, b in pairs]
    rng = np.random.default_rng(17)
    t_res, t_host = [], []
    for k in range(300):
        for i, ((a, b), (ba, bb)) in enumerate(zip(pairs, bufs)):
            act = rng.uniform(-1, 1, (1, max(a.action_dim, 1))).astype(np.float32)
            nz = rng.standard_normal((1, 3)) if _MIX[i][3] else None
            t0 = time.perf_counter()
            x = _step(nat.lib.lz_step_host, a, act, nz, ba)
            t1 = time.perf_counter()
            y = _step(nat.lib.lz_resident_step, b, act, nz, bb)
            t2 = time.perf_counter()
            if k >= 20:
                t_host.append(t1 - t0)
                t_res.append(t2 - t1)
            for p, q in zip(x, y):
                assert bits_equal(p, q), (i, k)
            if k % 25 == 7:  # published copy, no stop
                for pl in range(2):
                    assert bits_equal(a.get_state(pl).cpu().numpy(), _plane_host(b, pl)), (i, k, pl)
    print("8 handles round robin: median step lz_step_host %.1f us, resident %.1f us"
          % (1e6 * np.median(t_host), 1e6 * np.median(t_res)))
    for a, b in pairs:
        nat.check(nat.lib.lz_resident_stop(b._h))
        for pl in range(2):
            assert bits_equal(a.get_state(pl).cpu().numpy(), b.get_state(pl).cpu().numpy())
        a.close(), b.close()


def test_resident_member_churn(gl):
    """Handles joining (a restart with every state written back), a plain call on one
    member (stops the server for all), a member closing while others are served, and a
    16th and 17th handle (step through lz_step_host): all stay bit-identical to their twins."""
    import gym_lorenz._native as nat

    pairs, bufs = [], []
    rng = np.random.default_rng(23)

    def add(n):
        for _ in range(n):
            pairs.append(_pair("pmsm", 1, "float32", add_noise=True))
            bufs.append((_bufs(pairs[-1][0]), _bufs(pairs[-1][1])))

    def rounds(m):
        for k in range(m):
            for (a, b), (ba, bb) in zip(pairs, bufs):
                if a is None:
                    continue
                act = rng.uniform(-1, 1, (1, 2)).astype(np.float32)
                x = _step(nat.lib.lz_step_host, a, act, None, ba)
                y = _step(nat.lib.lz_resident_step, b, act, None, bb)
                for p, q in zip(x, y):
                    assert bits_equal(p, q), k

    add(3)
    rounds(20)
    add(5)  # joins: restart
    rounds(20)
    a, b = pairs[2]
    act = torch.zeros((1, 2), device=a.device)
    oa, _, _ = a.step(act)  # plain lz_step on a served handle: stops the server first
    ob, _, _ = b.step(act)
    assert bits_equal(oa.cpu().numpy(), ob.cpu().numpy())
    rounds(20)
    a, b = pairs[4]
    a.close(), b.close()  # a member leaves while the others are served
    pairs[4] = (None, None)
    rounds(20)
    add(10)  # 17 live handles: the 16th and 17th fall back to lz_step_host
    rounds(20)
    for a, b in pairs:
        if a is not None:
            a.close(), b.close()


def test_resident_two_threads(gl):
    """Drop-in envs stepped from two Python threads at once (ctypes releases the GIL
    during the call; the server's membership and command line are guarded by one
    mutex): every env stays bit-identical to its lz_step_host twin."""
    import threading

    import gym_lorenz._native as nat

    pairs = [_pair("pmsm", 1, "float32", add_noise=True) for _ in range(4)]
    errors = []

    def worker(idx, seed):
        try:
            rng = np.random.default_rng(seed)
            mine = pairs[idx::2]
            bufs = [(_bufs(a), _bufs(b)) for a, b in mine]
            for k in range(300):
                for (a, b), (ba, bb) in zip(mine, bufs):
                    act = rng.uniform(-1, 1, (1, 2)).astype(np.float32)
                    x = _step(nat.lib.lz_step_host, a, act, None, ba)
                    y = _step(nat.lib.lz_resident_step, b, act, None, bb)
                    for p, q in zip(x, y):
                        if not bits_equal(p, q):
                            errors.append((idx, k))
                            return
        except Exception as e:  # noqa: BLE001
            errors.append(repr(e))

    ts = [threading.Thread(target=worker, args=(j, 40 + j)) for j in range(2)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=120)
    assert not errors, errors[:3]
    for a, b in pairs:
        a.close(), b.close()


def test_read_state_after_idle_exit(gl, monkeypatch):
    """lz_resident_read_state while the server runs (its published copy) and after its
    idle exit (the planes): both equal the lz_step_host twin's state, and stepping on
    afterwards relaunches the server with the same trajectory."""
    import gym_lorenz._native as nat

    monkeypatch.setenv("LZ_RESIDENT_IDLE_US", "300")
    a, b = _pair("hr", 1, "float64", add_noise=True)
    ba, bb = _bufs(a), _bufs(b)
    rng = np.random.default_rng(8)
    for k in range(40):
        act = rng.uniform(-1, 1, (1, 2)).astype(np.float32)
        x = _step(nat.lib.lz_step_host, a, act, None, ba)
        y = _step(nat.lib.lz_resident_step, b, act, None, bb)
        for p, q in zip(x, y):
            assert bits_equal(p, q), k
        if k % 10 == 9:
            if k % 20 == 19:
                time.sleep(0.003)  # > the idle limit: the server has exited
            for pl in range(9):  # HR: master (3), slave (3), sigma, filter (2)
                assert bits_equal(a.get_state(pl).cpu().numpy(), _plane_host(b, pl)), (k, pl)
    a.close(), b.close()
