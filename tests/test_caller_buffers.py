"""The checked entry for caller-owned buffers (BatchedEnv.step_args / step_into /
rollout_args / rollout_into, core.step_io_args / rollout_io_args), on CPU through the
oracle-driven FakeBackend.

Why it exists: two round-5 measurement tools allocated
a LORENZ3 obs ring as (R, N, 3) and passed raw slot pointers to lz_step, whose obs rows
are [N, 6] (the reference's 6-D observation, dynamic.py:80-83): slot r's write covered
slots r and r + 1, the last slot wrote 12 MB past the allocation, and the first hipGraph
replay that reached it faulted (hipErrorIllegalAddress).  The C-ABI takes raw pointers
with no sizes, so the Python layer refuses such buffers before any launch."""
import numpy as np
import pytest
import torch

from fake_backend import FakeBackend
from gym_lorenz import _native as nat
from gym_lorenz.core import check_buffer, rollout_io_args, step_io_args

N, R = 64, 4


def _ring(obs_cols, n=N, r=R, be=None):
    acts = torch.rand((r, n, 3)) * 2 - 1
    obs = torch.empty((r, n, obs_cols))
    rew = torch.empty((r, n))
    done = torch.empty((r, n), dtype=torch.uint8)
    return acts, obs, rew, done


def test_l3_obs_ring_of_3_columns_is_refused():
    """The r05 fault's exact shape: a LORENZ3 (R, N, 3) obs slot is refused with
    LorenzEnvError(LZ_ERR_INVALID), and nothing is stepped."""
    be = FakeBackend("lorenz3", N, seed=1)
    be.reset()
    acts, obs, rew, done = _ring(3)
    tick = be.tick
    for r in range(R):
        with pytest.raises(nat.LorenzEnvError) as e:
            be.step_into(acts[r], obs[r], rew[r], done[r])
        assert e.value.status == nat.LZ_ERR_INVALID
        assert "obs" in str(e.value) and "need %d" % (6 * N) in str(e.value)
    assert be.tick == tick  # refused before the step


def test_l3_obs_ring_of_6_columns_steps_like_step():
    """The right ring ((R, N, 6)) is accepted slot by slot and gets exactly step()'s
    outputs (a twin backend stepped with step())."""
    a, b = FakeBackend("lorenz3", N, seed=3, max_episode_steps=3), \
        FakeBackend("lorenz3", N, seed=3, max_episode_steps=3)
    a.reset()
    b.reset()
    acts, obs, rew, done = _ring(6)
    didx = torch.empty((N,), dtype=torch.int32)
    tobs = torch.empty((N, 6))
    nd = torch.zeros((1,), dtype=torch.int32)
    for k in range(2 * R):
        r = k % R
        a.step_into(acts[r], obs[r], rew[r], done[r], didx, tobs, nd)
        o, w, d = b.step(acts[r])
        assert torch.equal(obs[r], o) and torch.equal(rew[r], w) and torch.equal(done[r], d)
        i, t = b.done_list()
        assert int(nd.item()) == len(i)
        assert np.array_equal(didx[: len(i)].numpy(), i.numpy().astype(np.int32))


@pytest.mark.parametrize("which, bad", [
    ("actions", lambda t: t.double()),                 # dtype
    ("actions", lambda t: t[:, :2].contiguous()),      # element count
    ("actions", lambda t: t.t().contiguous().t()),     # layout (not contiguous)
    ("obs", lambda t: t.reshape(-1)[: N * 6 - 1]),     # one element short
    ("obs", lambda t: torch.cat([t, t])),              # too long (layout confusion)
    ("rew", lambda t: t.double()),
    ("done", lambda t: t.bool()),                      # bool is not the uint8 done byte
    ("done", lambda t: t[: N - 1]),
    ("obs", lambda t: t.numpy()),                      # not a tensor
])
def test_every_buffer_is_checked(which, bad):
    be = FakeBackend("lorenz3", N)
    be.reset()
    acts, obs, rew, done = _ring(6, r=1)
    bufs = {"actions": acts[0], "obs": obs[0], "rew": rew[0], "done": done[0]}
    bufs[which] = bad(bufs[which])
    with pytest.raises(nat.LorenzEnvError) as e:
        be.step_into(**bufs)
    assert e.value.status == nat.LZ_ERR_INVALID and which in str(e.value)


def test_compact_list_is_a_capacity_and_pairs():
    be = FakeBackend("pmsm", N)
    be.reset()
    acts = torch.zeros((N, 2))
    obs, rew, done = torch.empty((N, 6)), torch.empty(N), torch.empty(N, dtype=torch.uint8)
    big_i, big_t = torch.empty((2 * N + 1,), dtype=torch.int32), torch.empty((2 * N, 6))
    be.step_into(acts, obs, rew, done, big_i, big_t)  # larger capacities are fine
    with pytest.raises(nat.LorenzEnvError):  # one short
        be.step_into(acts, obs, rew, done, big_i[: N - 1], big_t)
    with pytest.raises(nat.LorenzEnvError):  # int64 ids are the rollout's list, not the step's
        be.step_into(acts, obs, rew, done, big_i.long(), big_t)
    with pytest.raises(nat.LorenzEnvError):  # both or neither
        be.step_into(acts, obs, rew, done, big_i, None)
    with pytest.raises(nat.LorenzEnvError):
        be.step_into(acts, obs, rew, done, n_done=torch.zeros((1,), dtype=torch.int64))
    with pytest.raises(nat.LorenzEnvError):  # PMSM takes 2 action columns
        be.step_into(torch.zeros((N, 3)), obs, rew, done)


def test_rollout_buffers_are_checked():
    """lz_rollout's time-major buffers: [K, N, 3] obs for LORENZ3 is refused too."""
    K = 3
    be = FakeBackend("lorenz3", N, seed=4)
    be.reset()
    acts = torch.rand((K, N, 3)) * 2 - 1
    rew, done = torch.empty((K, N)), torch.empty((K, N), dtype=torch.uint8)
    with pytest.raises(nat.LorenzEnvError):
        be.rollout_into(K, acts, torch.empty((K, N, 3)), rew, done)
    with pytest.raises(nat.LorenzEnvError):  # K disagrees with the buffers
        be.rollout_into(K + 1, acts, torch.empty((K, N, 6)), rew, done)
    with pytest.raises(nat.LorenzEnvError):
        be.rollout_into(0, acts, torch.empty((K, N, 6)), rew, done)
    with pytest.raises(nat.LorenzEnvError):  # a done list needs cap >= 1
        be.rollout_into(K, acts, torch.empty((K, N, 6)), rew, done,
                        torch.empty((0,), dtype=torch.int64), torch.empty((0, 6)), 0)
    obs = torch.empty((K, N, 6))
    be.rollout_into(K, acts, obs, rew, done)
    args = rollout_io_args(be, K, acts, obs, rew, done, torch.empty((5,), dtype=torch.int64),
                           torch.empty((5, 6)), 5)
    assert args[0] == K and args[7] == 5


def test_actions_optional_only_where_the_system_reads_none():
    """LORENZ4 / SC read no actions (lz_api.cpp lz_step needs_act): None passes there only."""
    class Spec:
        num_envs, obs_dim, action_dim = 8, 8, 3
        tdtype, device, reads_actions = torch.float64, torch.device("cpu"), False
    out = (torch.empty((8, 8), dtype=torch.float64), torch.empty(8, dtype=torch.float64),
           torch.empty(8, dtype=torch.uint8))
    assert step_io_args(Spec, None, *out)[0] is None
    Spec.reads_actions = True
    with pytest.raises(nat.LorenzEnvError):
        step_io_args(Spec, None, *out)
    assert check_buffer(None, "x", torch.float32, 1, torch.device("cpu"), required=False) is None


@pytest.mark.parametrize("system", sorted({"lorenz3": 0, "lorenz4": 1, "pmsm": 2, "hr": 3,
                                           "transient1": 4, "transient2": 5, "transient_pmsm": 6,
                                           "singlecontrol": 7}))
@pytest.mark.parametrize("dtype", ["float32", "float64"])
def test_c_abi_io_sizes_agree_with_the_checker(system, dtype):
    """lz_io_sizes_for (include/lorenz_env.h: the bytes every raw buffer of lz_step /
    lz_rollout must cover, host-only) and the Python checker (core.step_io_args /
    rollout_io_args) state the same contract, for every system and precision."""
    import ctypes

    from gym_lorenz.core import SYSTEMS

    sysid = SYSTEMS[system]
    cfg = nat.config_init(sysid)
    f64 = dtype == "float64" and system != "pmsm"
    cfg.dtype = nat.F64 if f64 else nat.F32
    n, K, cap = 1000, 7, 33
    cfg.num_envs = n
    td = torch.float64 if f64 else torch.float32
    es = 8 if f64 else 4
    obs_dim = {"lorenz4": 8, "transient2": 8}.get(system, 6)
    act_dim = {"lorenz3": 3, "lorenz4": 3, "transient2": 3}.get(system, 2)
    reads = system not in ("lorenz4", "singlecontrol")

    from types import SimpleNamespace

    Spec = SimpleNamespace(num_envs=n, obs_dim=obs_dim, action_dim=act_dim, tdtype=td,
                           device=torch.device("cpu"), reads_actions=reads)
    for k in (0, K):
        sz = nat.LzIoSizes()
        nat.check(nat.lib.lz_io_sizes_for(ctypes.byref(cfg), k, cap if k else 0, ctypes.byref(sz)))
        steps = max(k, 1)
        assert sz.actions == (steps * n * act_dim * 4 if reads else 0)
        assert sz.obs == steps * n * obs_dim * es and sz.rew == steps * n * es and sz.done == steps * n
        assert sz.n_done == 4
        bufs = [torch.empty(sz.actions // 4, dtype=torch.float32) if reads else None,
                torch.empty(sz.obs // es, dtype=td), torch.empty(sz.rew // es, dtype=td),
                torch.empty(sz.done, dtype=torch.uint8)]
        if k == 0:
            assert sz.noise == n * 24 and sz.done_idx == n * 4 and sz.terminal_obs == n * obs_dim * es
            step_io_args(Spec, bufs[0], *bufs[1:], torch.empty(sz.done_idx // 4, dtype=torch.int32),
                         torch.empty(sz.terminal_obs // es, dtype=td), torch.empty(1, dtype=torch.int32),
                         noise=torch.empty(sz.noise // 8, dtype=torch.float64))
            with pytest.raises(nat.LorenzEnvError):  # one element short of the C sizes: refused
                step_io_args(Spec, bufs[0], torch.empty(sz.obs // es - 1, dtype=td), *bufs[2:])
        else:
            assert sz.noise == 0 and sz.done_idx == cap * 8 and sz.terminal_obs == cap * obs_dim * es
            rollout_io_args(Spec, k, bufs[0], *bufs[1:], torch.empty(cap, dtype=torch.int64),
                            torch.empty(sz.terminal_obs // es, dtype=td), cap)
    bad = nat.LzIoSizes()
    assert nat.lib.lz_io_sizes_for(None, 0, 0, ctypes.byref(bad)) == nat.LZ_ERR_INVALID
    cfg.num_envs = 0
    assert nat.lib.lz_io_sizes_for(ctypes.byref(cfg), 0, 0, ctypes.byref(bad)) == nat.LZ_ERR_INVALID
