"""Is the K-step rollout's time a function of where its output buffers sit?  The same
kernel on fresh allocations of the same sizes differs by up to ~18% at 262,144 envs
(profiles/r03/done_stores/ab_rollout_262k_3.json).  Here ONE env and ONE action tensor;
the obs / reward / done outputs are views into larger allocations at chosen byte offsets
(16-B aligned), so only their placement relative to each other and to the actions
changes.  HIP-event time per 2048-step launch, median of 7 after 2 warm.

  python tools/placement_probe.py [envs] -> one JSON line per placement
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "gym-lorenz_amd"))
import gym_lorenz as gl  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 262144
    K = 2048
    be = gl.BatchedEnv("lorenz3", n, seed=0)
    be.reset()
    dev = be.device
    A = torch.rand((K, n, 3), device=dev) * 2 - 1
    O = be.obs_dim
    pad = 8 << 20  # room for offsets up to 8 MiB
    obs_raw = torch.empty(K * n * O + pad // 4, device=dev)
    rew_raw = torch.empty(K * n + pad // 4, device=dev)
    done_raw = torch.empty(K * n + pad, dtype=torch.uint8, device=dev)

    def views(oo, ro, do):
        o = obs_raw[oo // 4: oo // 4 + K * n * O].view(K, n, O)
        r = rew_raw[ro // 4: ro // 4 + K * n].view(K, n)
        d = done_raw[do: do + K * n].view(K, n)
        return o, r, d

    def timed(bufs):
        for _ in range(2):
            be.rollout(A, *bufs)
        ts = []
        for _ in range(7):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            be.rollout(A, *bufs)
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1) * 1e3)
        return sorted(ts)[3]

    base = {"obs": obs_raw.data_ptr(), "rew": rew_raw.data_ptr(), "done": done_raw.data_ptr(),
            "act": A.data_ptr()}
    print(json.dumps({"envs": n, "K": K, "bases_mod_2MiB": {k: v % (2 << 20) for k, v in base.items()}}),
          flush=True)
    offs = [0, 4096, 65536, 256 << 10, 1 << 20, (1 << 20) + 4096, 2 << 20, 3 << 20, (4 << 20) + 65536]
    for what in ("obs", "rew", "done"):
        for off in offs:
            oo, ro, do = (off if what == "obs" else 0, off if what == "rew" else 0,
                          off if what == "done" else 0)
            us = timed(views(oo, ro, do))
            print(json.dumps({"moved": what, "offset": off, "us_median": us}), flush=True)
    for rep in range(3):  # the unmoved placement again: drift control
        print(json.dumps({"moved": "none", "rep": rep, "us_median": timed(views(0, 0, 0))}), flush=True)


if __name__ == "__main__":
    main()
