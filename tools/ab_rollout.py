"""A/B of the fused rollout's tuning variants (lz_config.reserved[0] bits, see
lz_kernels.hip rollout_split / launch_all): 256 = one lane per env, 512 = two lanes
per env (small N), 1024 = DMA prefetch distance 3 instead of 7.  All envs and buffers
are allocated first; the variants then run in an order rotated every round (so no
variant always follows the same one), HIP-event timing on the launch stream; median
and min over rounds.  A variant may be listed twice (a control: the spread between the
two copies is the noise floor).
Usage: AB_VARIANTS=0,256,0 python tools/ab_rollout.py [system] [envs...]  (AB_K=2048)"""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gym-lorenz_amd"))
import gym_lorenz as gl  # noqa: E402


def timed(be, A, bufs, reps):
    s = be.stream
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(reps):
        be.rollout(A, *bufs)
    e1.record(s)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3  # us per rollout


def main():
    system = sys.argv[1] if len(sys.argv) > 1 else "lorenz3"
    K = int(os.environ.get("AB_K", "2048"))
    rounds = int(os.environ.get("AB_ROUNDS", "9"))
    variants = [int(v) for v in os.environ.get("AB_VARIANTS", "0,256,0").split(",")]
    out = {}
    for n in (int(v) for v in (sys.argv[2:] or ["16384", "32768", "65536"])):
        runs = []
        A = None
        for var in variants:
            be = gl.BatchedEnv(system, n, seed=0, variant=var, add_noise=(system in ("pmsm", "hr")))
            be.reset()
            if A is None:
                A = torch.rand((K, n, be.action_dim), device=be.device) * 2 - 1
            o = be.obs_dim
            bufs = (torch.empty((K, n, o), device=be.device), torch.empty((K, n), device=be.device),
                    torch.empty((K, n), dtype=torch.uint8, device=be.device))
            runs.append((be, bufs))
        for be, bufs in runs:  # warm
            be.rollout(A, *bufs)
        torch.cuda.synchronize()
        bps = 4 * (be.action_dim + o + 1) + 1
        res = [[] for _ in variants]
        V = len(variants)
        for r in range(rounds):
            for j in range(V):
                v = (r + j) % V
                res[v].append(timed(runs[v][0], A, runs[v][1], 2))
        for idx, var in enumerate(variants):
            t = sorted(res[idx])
            us = t[len(t) // 2]
            out["%s n=%d K=%d variant=%d #%d" % (system, n, K, var, idx)] = {
                "us_med": us, "us_min": t[0], "env_steps_per_s": n * K / us * 1e6,
                "GBps_io": n * K * bps / us * 1e-3}
        # a variant listed several times = several allocations of its buffers (placement
        # moves the time by up to ~18% at 262,144 envs): mean of their medians
        for var in sorted(set(variants)):
            meds = [sorted(res[i])[len(res[i]) // 2] for i, v in enumerate(variants) if v == var]
            out["%s n=%d K=%d variant=%d mean_of_%d" % (system, n, K, var, len(meds))] = {
                "us_mean_of_medians": sum(meds) / len(meds), "us_medians": meds}
        del runs, A
        torch.cuda.empty_cache()
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
