"""gym_lorenz._stepper (csrc/lz_stepper.c), the per-env drop-in classes' hot call, on the
CPU: driven with a ctypes stand-in for lz_resident_step / lz_step_host (same C signature,
include/lorenz_env.h), it must marshal exactly as SingleEnvCore.step's ctypes path does --
the action cast to float32, the injected noise as float64[3] (NULL when absent), and
(obs copy, numpy reward scalar of the env's dtype, done int) back, or the lz_status int."""
import ctypes

import numpy as np
import pytest

stepper = pytest.importorskip("gym_lorenz._stepper")
pytestmark = pytest.mark.filterwarnings("ignore:overflow encountered in cast:RuntimeWarning")

FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.POINTER(ctypes.c_float),
                      ctypes.POINTER(ctypes.c_double), ctypes.c_void_p, ctypes.c_void_p,
                      ctypes.POINTER(ctypes.c_uint8))


class Fake:
    """obs[j] = action[j % A] + j (+ noise[0] if given), reward = sum(action), done = calls."""

    def __init__(self, A, O, dtype, status=0):
        self.A, self.O, self.dt, self.status = A, O, np.dtype(dtype), status
        self.calls, self.seen = 0, []
        self.act = np.zeros((1, A), np.float32)
        self.noise = np.zeros((1, 3), np.float64)
        self.obs = np.zeros((1, O), dtype)
        self.rew = np.zeros(1, dtype)
        self.done = np.zeros(1, np.uint8)
        self.cb = FN(self._step)

    def _step(self, h, act, noise, obs, rew, done):
        self.calls += 1
        a = np.ctypeslib.as_array(act, (self.A,)).copy() if self.A else np.zeros(0, np.float32)
        nz = None if not noise else np.ctypeslib.as_array(noise, (3,)).copy()
        self.seen.append((h, a, nz))
        o = np.array([(a[j % self.A] if self.A else 0.0) + j + (nz[0] if nz is not None else 0.0)
                      for j in range(self.O)], self.dt)
        ctypes.memmove(obs, o.ctypes.data, o.nbytes)
        r = np.array([a.astype(np.float64).sum()], self.dt)
        ctypes.memmove(rew, r.ctypes.data, r.nbytes)
        done[0] = self.calls % 256
        return self.status

    def stepper(self, handle=0x1234):
        fn = ctypes.cast(self.cb, ctypes.c_void_p).value
        p = [x.ctypes.data for x in (self.act, self.noise, self.obs, self.rew, self.done)]
        return stepper.Stepper(fn, handle, *p, self.A, self.O, int(self.dt == np.float64))


@pytest.mark.parametrize("dtype", [np.float64, np.float32])
@pytest.mark.parametrize("action", [
    [0.25, -1.5, 3.0], (0.25, -1.5, 3.0), np.array([0.25, -1.5, 3.0]),
    np.array([[0.25, -1.5, 3.0]], np.float32), np.array([1, -2, 3]), [np.float32(0.1), 2, 1e40]])
def test_marshalling_matches_numpy_path(dtype, action):
    f = Fake(3, 6, dtype)
    s = f.stepper()
    obs, rew, done = s.step(action)
    want_a = np.zeros((1, 3), np.float32)
    want_a[...] = np.asarray(action).reshape(1, -1)  # the ctypes path's float32 cast
    h, a, nz = f.seen[-1]
    assert h == 0x1234 and nz is None
    assert np.array_equal(a.view(np.uint32), want_a[0].view(np.uint32))
    assert type(obs) is np.ndarray and obs.dtype == np.dtype(dtype) and obs.shape == (6,)
    assert np.array_equal(obs, f.obs[0]) and obs.ctypes.data != f.obs.ctypes.data  # a copy
    assert type(rew) is type(f.rew[0]) and rew == f.rew[0]
    assert type(done) is int and done == 1


def test_noise_and_status_and_errors():
    f = Fake(2, 6, np.float64)
    s = f.stepper()
    obs, _, _ = s.step(np.zeros(2), np.array([0.5, 0.25, -1.0]))
    assert np.array_equal(f.seen[-1][2], [0.5, 0.25, -1.0]) and obs[0] == 0.5
    s.step([1.0, 2.0], None)
    assert f.seen[-1][2] is None
    with pytest.raises(ValueError):
        s.step([1.0, 2.0, 3.0])  # wrong size: nothing called
    with pytest.raises(ValueError):
        s.step(0.5)  # a scalar (numpy would broadcast; SingleEnvCore falls back to numpy)
    assert f.calls == 2
    bad = Fake(2, 6, np.float64, status=3)
    assert bad.stepper().step([0.0, 0.0]) == 3


def test_no_action_system():
    f = Fake(0, 8, np.float32)  # LORENZ4 / singlecontrol: no action read
    obs, rew, done = f.stepper().step([])
    assert obs.shape == (8,) and rew == 0.0 and done == 1


def test_close_forgets_handle():
    """after Stepper.close() (SingleEnvCore.close, before lz_destroy) a step
    passes a NULL handle -- the library's clean LZ_ERR_INVALID -- never the freed address."""
    f = Fake(2, 6, np.float64)
    s = f.stepper()
    s.step([0.0, 1.0])
    assert f.seen[-1][0] == 0x1234
    s.close()
    s.step([0.0, 1.0])
    assert f.seen[-1][0] is None  # ctypes hands a NULL c_void_p over as None


def test_real_library_null_handle_is_invalid():
    """The real entry points answer a NULL handle with LZ_ERR_INVALID (no GPU touched)."""
    from gym_lorenz import _native as nat

    for name in ("lz_resident_step", "lz_step_host"):
        st = getattr(nat.lib, name)(None, None, None, None, None, None)
        assert st == nat.LZ_ERR_INVALID, name
