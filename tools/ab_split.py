"""A/B: one lz_step launch over N envs per step vs the env axis split into S handles
on S streams inside one hipGraph (independent step chains overlap their kernel
boundaries).  HIP events on the capture-origin stream; us per full step."""
import ctypes
import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "gym-lorenz_amd"))
import gym_lorenz as gl  # noqa: E402
from gym_lorenz import _native as nat  # noqa: E402

L, R = 32, 16


def build(n, S):
    parts = []
    main = torch.cuda.Stream()
    streams = [main] + [torch.cuda.Stream() for _ in range(S - 1)]
    for s in range(S):
        m = n // S
        env = gl.BatchedEnv("lorenz3", m, global_env_offset=s * m)
        env.reset()
        acts = torch.rand((R, m, 3), device="cuda") * 2 - 1
        obs = torch.empty((R, m, 6), device="cuda")
        rew = torch.empty((R, m), device="cuda")
        done = torch.empty((R, m), dtype=torch.uint8, device="cuda")
        nat.check(nat.lib.lz_set_stream(env._h, ctypes.c_void_p(streams[s].cuda_stream)))
        parts.append((env, acts, obs, rew, done))
    torch.cuda.synchronize()

    def enqueue(k):
        for s, (env, acts, obs, rew, done) in enumerate(parts):
            r = k % R
            nat.check(nat.lib.lz_step(env._h, *env.step_args(acts[r], obs[r], rew[r], done[r],
                                                             env.done_idx, env.term_obs)))

    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(main):
        for k in range(4):
            for s in range(1, S):
                streams[s].wait_stream(main)
            enqueue(k)
            for s in range(1, S):
                main.wait_stream(streams[s])
        torch.cuda.synchronize()
        with torch.cuda.graph(g, stream=main):
            for s in range(1, S):
                streams[s].wait_stream(main)
            for k in range(L):
                enqueue(k)
            for s in range(1, S):
                main.wait_stream(streams[s])
    return g, main, parts


def timeit(g, main, reps):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    with torch.cuda.stream(main):
        g.replay()
        e0.record(main)
        for _ in range(reps):
            g.replay()
        e1.record(main)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / (reps * L)


res = {}
for n in [int(x) for x in sys.argv[1:]] or [131072, 1048576]:
    runs = {S: build(n, S) for S in (1, 2, 4)}
    reps = max(4, int(8e5 / n))
    samp = {S: [] for S in runs}
    for _ in range(7):
        for S, (g, main, _) in runs.items():
            samp[S].append(timeit(g, main, reps))
    for S in runs:
        v = sorted(samp[S])[3]
        res["n=%d split=%d" % (n, S)] = {"us_per_step": v, "GBps": 65 * n / v / 1e3,
                                         "env_steps_per_s": n / v * 1e6}
    del runs
    torch.cuda.empty_cache()
print(json.dumps(res, indent=1))
