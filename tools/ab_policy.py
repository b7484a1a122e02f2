"""A/B of the fused policy rollout's launch shapes (interleaved, one process):
variant 0 = the default shape for n (E=64 / 8 waves above 131,072 envs, else E=32 /
4 waves with interleaved nets), 32 = E=32 / 8 waves serial nets, 64 = the small
shape forced (lz_config.reserved[0] bits, lz_internal.h policy_shape)."""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gym-lorenz_amd"))
import gym_lorenz as gl  # noqa: E402
from gym_lorenz.policy import ActorCriticMlp, FusedRolloutCollector  # noqa: E402


def timed(col, K, reps):
    s = torch.cuda.current_stream()
    col.collect(K)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(reps):
        col.collect(K)
    e1.record(s)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3  # us per collect


def main():
    system = sys.argv[1] if len(sys.argv) > 1 else "pmsm"
    K = int(os.environ.get("AB_K", "16"))
    variants = [int(v) for v in os.environ.get("AB_VARIANTS", "0,32").split(",")]
    out = {}
    for n in (int(v) for v in (sys.argv[2:] or ["262144", "1048576"])):
        cols = {}
        for var in variants:
            env = gl.BatchedEnv(system, n, seed=0, variant=var, add_noise=(system == "pmsm"))
            net = ActorCriticMlp(env.obs_dim, env.action_dim, seed=0)
            c = FusedRolloutCollector(env, net.state_dict())
            c.reset()
            cols[var] = c
        res = {v: [] for v in variants}
        for _ in range(5):
            for var in variants:
                res[var].append(timed(cols[var], K, max(2, 160 // K)))
        for var in variants:
            us = sorted(res[var])[len(res[var]) // 2]
            out["%s n=%d K=%d variant=%d" % (system, n, K, var)] = {
                "us_per_collect": us, "env_steps_per_s": n * K / us * 1e6}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
