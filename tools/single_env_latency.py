"""Per-env drop-in class step latency (the path of callers that keep
DummyVecEnv([lambda: gymnasium.make(...)]) unchanged): one kernel-backed env stepped
from Python, microseconds per step; next to the reference-semantics Python loop
(oracle/ref_loop.py) on the same host core for LORENZ3."""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gym-lorenz_amd"))
sys.path.insert(0, ROOT)
import gym_lorenz as gl  # noqa: E402


def timed(env, act, steps):
    for _ in range(50):
        env.step(act)
    t0 = time.perf_counter()
    for _ in range(steps):
        env.step(act)
    return (time.perf_counter() - t0) / steps * 1e6


def main():
    out = {}
    np.random.seed(0)
    e = gl.make("lorenz_dynamic-v0")
    e.reset()
    out["lorenz_dynamic-v0 (fp64)"] = timed(e, np.zeros(3, np.float32), 2000)
    e = gl.make("lorenz_try-v0")
    e.reset(seed=0)
    out["lorenz_try-v0 HR (fp64)"] = timed(e, np.zeros(2, np.float32), 2000)
    e = gl.make("lorenz_pmsm-v0")
    e.reset(seed=0)
    out["lorenz_pmsm-v0 (fp32)"] = timed(e, np.zeros(2, np.float32), 2000)
    from oracle.ref_loop import LorenzRefEnv
    r = LorenzRefEnv(np.array([1.0, 2.0, 3.0]))
    a = np.zeros(3, np.float32)
    t0 = time.perf_counter()
    for _ in range(20000):
        r.step(a)
    out["reference-semantics dynamic.py step (CPU)"] = (time.perf_counter() - t0) / 20000 * 1e6
    print(json.dumps({"us_per_step": out}, indent=1))


if __name__ == "__main__":
    main()
