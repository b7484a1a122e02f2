"""One shard as S sub-handles on S HIP streams (gym_lorenz.parallel.StreamSplitEnv, bench.py
--streams S) is the same computation as one handle of the whole shard.

The sub-handles take consecutive global_env_offset, so their Philox resets / noise draws
are keyed by the same global ids; each steps its own rows of the caller's buffers on its
own stream, concurrently.  Here S = 2 / 4 at cfg3's 131,072-env per-GPU shard (and a ragged
70,001) with TimeLimit(7) auto-reset for 20 steps, against one handle bit for bit: obs,
reward, done bytes, the done SET with its terminal obs (sub-handle ids mapped to shard
rows), every state plane; plus the same inside a captured hipGraph (the bench's launch).

Reference: dynamic.py:61-90 (LORENZ3), lorenz_env_try_pmsm.py:76-184 (PMSM, device noise)."""
import numpy as np
import pytest
import torch

pytestmark = [pytest.mark.gpu, pytest.mark.filterwarnings("ignore::RuntimeWarning")]


@pytest.fixture(scope="module")
def gl():
    import gym_lorenz

    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    return gym_lorenz


def _bits(t):
    return t.view(torch.int32) if t.dtype == torch.float32 else t


def _same(a, b):
    return a.shape == b.shape and torch.equal(_bits(a), _bits(b))


def _sorted_done(idx, tobs):
    order = torch.argsort(idx)
    return idx[order].cpu(), tobs[order].cpu()


@pytest.mark.parametrize("system, n, S, kw", [
    ("lorenz3", 131072, 2, {}), ("lorenz3", 131072, 4, {}), ("lorenz3", 70001, 4, {}),
    ("lorenz3", 65536, 3, {}), ("pmsm", 131072, 4, {"add_noise": True}),
])
def test_stream_split_equals_one_handle(gl, system, n, S, kw):
    from gym_lorenz.parallel import StreamSplitEnv

    off = 3 * n  # a rank's shard: global ids [off, off + n)
    one = gl.BatchedEnv(system, n, seed=11, global_env_offset=off, max_episode_steps=7, **kw)
    spl = StreamSplitEnv(system, n, S, global_env_offset=off, seed=11, max_episode_steps=7, **kw)
    assert len(spl.subs) == S and spl.bounds[-1][1] == n
    dev, O, A = one.device, one.obs_dim, one.action_dim
    o1, o2 = torch.empty((n, O), device=dev), torch.empty((n, O), device=dev)
    assert _same(one.reset(out=o1), spl.reset(o2))
    g = torch.Generator(device=dev).manual_seed(5)
    r2, d2 = torch.empty((n,), device=dev), torch.empty((n,), dtype=torch.uint8, device=dev)
    n_done = 0
    for k in range(20):
        a = (torch.rand((n, A), generator=g, device=dev) * 2 - 1) * (1.2 if system == "pmsm" else 1)
        ob, rw, dn = one.step(a)
        spl.step_into(a, o2, r2, d2)
        torch.cuda.synchronize()
        assert _same(ob, o2) and _same(rw, r2) and torch.equal(dn, d2), "step %d" % k
        i1, t1 = one.done_list()
        i2, t2 = spl.done_list()
        i1, t1 = _sorted_done(i1, t1)
        i2, t2 = _sorted_done(i2, t2)
        assert torch.equal(i1, i2) and _same(t1, t2), "done list, step %d" % k
        n_done += len(i1)
    assert n_done >= n  # TimeLimit(7) truncated every env at least twice in 20 steps
    planes = {"lorenz3": 4, "pmsm": 11}[system]
    for p in range(planes):
        assert _same(one.get_state(p), spl.get_state(p)), "plane %d" % p
    one.close()
    spl.close()


def test_stream_split_in_captured_graphs(gl):
    """bench.py's launch: one captured graph per sub-handle stream (20 steps, a 4-slot
    ring each), replayed concurrently, vs one handle stepped eagerly."""
    n, S, R, L = 131072, 4, 4, 20
    from gym_lorenz.parallel import sub_shards

    one = gl.BatchedEnv("lorenz3", n, seed=2, max_episode_steps=9)
    subs = [gl.BatchedEnv("lorenz3", c, seed=2, global_env_offset=o, max_episode_steps=9)
            for o, c in sub_shards(n, 0, S)]
    dev = one.device
    acts = torch.rand((R, n, 3), device=dev) * 2 - 1
    obs = torch.empty((R, n, 6), device=dev)
    rew = torch.empty((R, n), device=dev)
    done = torch.empty((R, n), dtype=torch.uint8, device=dev)
    one.reset()
    streams = [torch.cuda.Stream(dev) for _ in subs]
    import ctypes

    from gym_lorenz import _native as nat

    bounds, lo = [], 0
    for e in subs:
        bounds.append((lo, lo + e.num_envs))
        lo += e.num_envs
    graphs = []
    torch.cuda.synchronize()
    for e, st, (a, b) in zip(subs, streams, bounds):
        nat.check(nat.lib.lz_set_stream(e._h, ctypes.c_void_p(st.cuda_stream)))
        with torch.cuda.stream(st):
            e.reset()
            slots = [e.step_args(acts[r, a:b], obs[r, a:b], rew[r, a:b], done[r, a:b],
                                 e.done_idx, e.term_obs) for r in range(R)]
            gr = torch.cuda.CUDAGraph()
            with torch.cuda.graph(gr, stream=st):
                for k in range(L):
                    nat.check(nat.lib.lz_step(e._h, *slots[k % R]))
            graphs.append(gr)
    torch.cuda.synchronize()
    for gr, st in zip(graphs, streams):
        with torch.cuda.stream(st):
            gr.replay()
    ref = []
    for k in range(L):
        ob, rw, dn = one.step(acts[k % R])
        if k >= L - R:  # the ring's last R slots hold steps L - R .. L - 1
            ref.append((k % R, ob.clone(), rw.clone(), dn.clone()))
    torch.cuda.synchronize()
    for r, ob, rw, dn in ref:
        assert _same(obs[r], ob) and _same(rew[r], rw) and torch.equal(done[r], dn), "slot %d" % r
    for p in range(4):
        st = torch.cat([e.get_state(p) for e in subs])
        torch.cuda.synchronize()
        assert _same(one.get_state(p), st)
    for e in subs + [one]:
        e.close()
