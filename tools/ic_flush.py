"""Which memory level does the headline step run against?  

The LORENZ3 f32 state of 1,048,576 envs (12 MB of x, y, z) is written by step k and read
by step k + 1 with only ~68 MB of other traffic in between, so under the guide's residency
rule (MI355X_MICROARCH.md "Infinity Cache": a line stays resident while everything touched
between two of its uses fits in ~256 MiB) its reads may be served by the 256 MiB Infinity
Cache, not DRAM -- and FETCH_SIZE counts those hits too.  This A/B keeps the kernel, the
handle and its bytes per env-step unchanged and only moves the state's reuse distance:
  warm: bench.py's loop -- one handle, hipGraph-replayed lz_step over a 16-slot ring;
  cold: the same, with a 2 x 192 MiB device copy (384 MiB of other traffic) between two
        steps, so every state line the step reads comes from HBM.
The step kernel's own duration is read from `rocprofv3 --kernel-trace --stats` of each
mode (the copy is a separate kernel), so the copy's time never enters the comparison.
Usage: rocprofv3 --kernel-trace --stats -d DIR -o run --output-format csv --
python tools/ic_flush.py {warm|cold} [windows]"""
import ctypes
import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "gym-lorenz_amd"))
import gym_lorenz as gl  # noqa: E402
from gym_lorenz import _native as nat  # noqa: E402

N, R, L = 1 << 20, 16, 64
FLUSH = 192 << 20  # bytes per copy buffer


def main():
    mode = sys.argv[1]
    windows = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    assert mode in ("warm", "cold")
    env = gl.BatchedEnv("lorenz3", N, dtype="float32", seed=0, autoreset=True)
    env.reset()
    dev = env.device
    acts = torch.rand((R, N, 3), device=dev) * 2 - 1
    obs = torch.empty((R, N, 3), device=dev)
    rew = torch.empty((R, N), device=dev)
    done = torch.empty((R, N), dtype=torch.uint8, device=dev)
    src = torch.ones((FLUSH // 4,), device=dev)
    dst = torch.empty_like(src)
    P = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
    slots = [(P(acts[r]), P(obs[r]), P(rew[r]), P(done[r])) for r in range(R)]
    didx, tobs = P(env.done_idx), P(env.term_obs)
    torch.cuda.synchronize()
    stream = torch.cuda.Stream()
    nat.check(nat.lib.lz_set_stream(env._h, ctypes.c_void_p(stream.cuda_stream)))
    k = [0]

    def one():
        a, o, r_, d = slots[k[0] % R]
        k[0] += 1
        nat.check(nat.lib.lz_step(env._h, a, None, o, r_, d, didx, tobs, None))
        if mode == "cold":
            dst.copy_(src)

    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(stream):
        for _ in range(4):
            one()
        torch.cuda.synchronize()
        with torch.cuda.graph(g, stream=stream):
            for _ in range(L):
                one()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        g.replay()
        e0.record(stream)
        for _ in range(windows):
            g.replay()
        e1.record(stream)
        torch.cuda.synchronize()
    print(json.dumps({"mode": mode, "envs": N, "steps_timed": windows * L,
                      "us_per_graph_step_incl_copy": e0.elapsed_time(e1) * 1e3 / (windows * L),
                      "bytes_per_env_step": env.bytes_per_env_step,
                      "kernel": nat.launch_shape(env._h, nat.CALL_STEP)["kernel"],
                      "copy_bytes_between_steps": 2 * FLUSH if mode == "cold" else 0}))
    env.close()


if __name__ == "__main__":
    main()
