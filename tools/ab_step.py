"""Interleaved A/B of lz_step kernel variants (one process, hipGraph-replayed steps,
HIP-event timing on the launch stream; order rotated every round, a variant listed twice
is a noise control).  Usage: AB_VARIANTS=0,32,0 [AB_SYSTEM=pmsm AB_NOISE=1]
python tools/ab_step.py [envs...]"""
import ctypes
import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "gym-lorenz_amd"))
import gym_lorenz as gl  # noqa: E402
from gym_lorenz import _native as nat  # noqa: E402


def make(variant, n, system="lorenz3", R=16):
    noise = os.environ.get("AB_NOISE")  # "1" / "0": force add_noise (default: the system's)
    kw = {} if noise is None else {"add_noise": noise == "1"}
    env = gl.BatchedEnv(system, n, dtype="float32", autoreset=True, variant=variant, **kw)
    env.reset()
    dev = env.device
    acts = torch.rand((R, n, env.action_dim), device=dev) * 2 - 1
    obs = torch.empty((R, n, env.obs_dim), device=dev)
    rew = torch.empty((R, n), device=dev)
    done = torch.empty((R, n), dtype=torch.uint8, device=dev)
    # the checked caller-buffer entry (BatchedEnv.step_args: sizes vs lz_info)
    slots = [env.step_args(acts[r], obs[r], rew[r], done[r], env.done_idx, env.term_obs)
             for r in range(R)]
    stream = torch.cuda.Stream()
    nat.check(nat.lib.lz_set_stream(env._h, ctypes.c_void_p(stream.cuda_stream)))
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(stream):
        for k in range(4):
            nat.check(nat.lib.lz_step(env._h, *slots[k % R]))
        torch.cuda.synchronize()
        with torch.cuda.graph(g, stream=stream):
            for k in range(32):
                nat.check(nat.lib.lz_step(env._h, *slots[k % R]))
    keep = (env, acts, obs, rew, done)
    return g, stream, keep


def timeit(g, stream, reps):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    with torch.cuda.stream(stream):
        g.replay()
        e0.record(stream)
        for _ in range(reps):
            g.replay()
        e1.record(stream)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / (reps * 32)  # us per step


def main():
    envs = [int(x) for x in sys.argv[1:]] or [131072, 1048576, 4194304]
    variants = [int(v) for v in os.environ.get("AB_VARIANTS", "0,1,2,3").split(",")]
    system = os.environ.get("AB_SYSTEM", "lorenz3")
    res = {}
    for n in envs:
        runs = [make(v, n, system) for v in variants]  # a variant may repeat (noise control)
        reps = max(4, int(2e5 / n * 4))
        samples = [[] for _ in variants]
        V = len(variants)
        for r in range(9):  # order rotated every round
            for j in range(V):
                k = (r + j) % V
                samples[k].append(timeit(runs[k][0], runs[k][1], reps))
        bps = runs[0][2][0].bytes_per_env_step
        for k, v in enumerate(variants):
            s = sorted(samples[k])
            med = s[len(s) // 2]
            res["%s n=%d v=%d #%d" % (system, n, v, k)] = {"us_med": med, "us_min": s[0],
                                                          "GBps": bps * n / med / 1e3}
        del runs
        torch.cuda.empty_cache()
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
