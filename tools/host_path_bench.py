"""Host-buffer paths: what an SB3 caller that keeps NumPy arrays pays.

  vecenv_numpy : LorenzVecEnv.step(np actions) -> np obs/rew/done (+ lazy infos), i.e.
                 H2D actions + kernel + D2H results per step (PCIe-inclusive rate)
  vecenv_torch : LorenzVecEnv(return_tensors=True) with device actions (no PCIe)
  dropin_1env  : the per-env drop-in class (1 env = 1 launch + 1 packed D2H copy)
Prints one JSON object."""
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gym-lorenz_amd"))
import gym_lorenz  # noqa: E402


def rate(fn, n_env, steps):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        fn()
    torch.cuda.synchronize()
    return n_env * steps / (time.perf_counter() - t0)


def main():
    out = {}
    for n in (65536, 1048576):
        v = gym_lorenz.make_vec("lorenz_dynamic-v0", n)
        v.reset()
        a = np.random.default_rng(0).uniform(-1, 1, (n, 3)).astype(np.float32)
        out["vecenv_numpy_%d" % n] = rate(lambda: v.step(a), n, 50)
        vt = gym_lorenz.make_vec("lorenz_dynamic-v0", n, return_tensors=True)
        vt.reset()
        at = torch.from_numpy(a).cuda()
        out["vecenv_torch_%d" % n] = rate(lambda: vt.step(at), n, 200)
    e = gym_lorenz.LorenzDynamicEnv()
    np.random.seed(0)
    e.reset()
    act = np.zeros(3, np.float32)
    out["dropin_1env"] = rate(lambda: e.step(act), 1, 2000)
    out["unit"] = "env-steps/s"
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
