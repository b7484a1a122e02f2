"""VecNormalize(LorenzVecEnv).step() throughput, device-tensor path (return_tensors):
the fused lz_step_vecnorm + lz_vecnorm_apply pair against the unfused sequence of
launches (step, moments, update, normalise, returns, ...) with its per-step host sync.
Actions pre-generated on the device; each timed step is the whole Python step_wait.

  python tools/vecnorm_bench.py [system env_id n steps] ...   -> one JSON line
"""
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gym-lorenz_amd"))
import gym_lorenz as gl  # noqa: E402
from gym_lorenz.vec_normalize import LorenzVecNormalize  # noqa: E402


def run(env_id, n, steps, fused):
    v = LorenzVecNormalize(gl.make_vec(env_id, n, seed=0, max_episode_steps=2000,
                                       return_tensors=True), norm_obs=True, norm_reward=False,
                           clip_obs=10.0)
    v._fused = fused
    A = v.venv.backend.action_dim
    acts = torch.rand((16, n, A), device="cuda") * 2 - 1
    v.reset()
    for k in range(20):
        v.step(acts[k % 16])
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(steps):
        v.step(acts[k % 16])
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    v.close()
    return n * steps / dt, dt / steps * 1e6


def main():
    cases = [("lorenz_pmsm-v0", 262144, 400), ("lorenz_pmsm-v0", 1048576, 200),
             ("lorenz_dynamic-v0", 1048576, 200), ("lorenz_pmsm-v0", 4096, 1000)]
    out = {"what": "VecNormalize(norm_obs, clip_obs=10) over LorenzVecEnv(return_tensors), "
                   "env-steps/s of the whole step() incl. Python; fused vs unfused"}
    for env_id, n, steps in cases:
        for fused in ((True,) if os.environ.get("VN_FUSED_ONLY") else (True, False)):
            v, us = run(env_id, n, steps, fused)
            key = "%s_%d_%s" % (env_id, n, "fused" if fused else "unfused")
            out[key] = {"env_steps_per_s": v, "us_per_step": us}
            print(key, v, us, file=sys.stderr, flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
