"""Which memory level does the headline step run against?  

The LORENZ3 f32 state of 1,048,576 envs (12 MB of x, y, z) is written by step k and read
by step k + 1 with only ~68 MB of other traffic in between, so under the guide's residency
rule (MI355X_MICROARCH.md "Infinity Cache": a line stays resident while everything touched
between two of its uses fits in ~256 MiB) its reads may be served by the 256 MiB Infinity
Cache, not DRAM -- and FETCH_SIZE counts those hits too.  This A/B keeps the kernel and its
bytes per env-step unchanged and only moves the state's reuse distance: H independent 1M
handles are stepped round-robin (step k runs handle k mod H), so (H - 1) x 68 MB of other
traffic separate two uses of a handle's state.  H = 1 is the bench line; H = 8 puts ~476 MB
between uses (cold: every state line comes from HBM).  Actions / outputs come from a 16-slot
ring per handle exactly as in bench.py (those are cold in both: 16 x 29 MB between reuses).

One process, hipGraph-replayed launches (64 per graph, an even count per handle: the tick
ping-pong stays valid), HIP events on the launch stream, the H values' order rotated every
round.  Usage: python tools/ic_ab.py [H...]  (default 1 2 4 8) > profiles/r05/ic_ab.json"""
import ctypes
import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "gym-lorenz_amd"))
import gym_lorenz as gl  # noqa: E402
from gym_lorenz import _native as nat  # noqa: E402

N = 1 << 20
R = 16       # ring slots per handle (bench.py --ring)
L = 64       # launches per captured graph


def make_handles(H, stream):
    P = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
    hs = []
    for j in range(H):
        env = gl.BatchedEnv("lorenz3", N, dtype="float32", seed=j, autoreset=True)
        env.reset()
        acts = torch.rand((R, N, 3), device=env.device) * 2 - 1
        obs = torch.empty((R, N, 3), device=env.device)
        rew = torch.empty((R, N), device=env.device)
        done = torch.empty((R, N), dtype=torch.uint8, device=env.device)
        nat.check(nat.lib.lz_set_stream(env._h, ctypes.c_void_p(stream.cuda_stream)))
        slots = [(P(acts[r]), P(obs[r]), P(rew[r]), P(done[r])) for r in range(R)]
        hs.append({"env": env, "keep": (acts, obs, rew, done), "slots": slots,
                   "didx": P(env.done_idx), "tobs": P(env.term_obs), "k": 0})
    return hs


def launch(h):
    a, o, r_, d = h["slots"][h["k"] % R]
    h["k"] += 1
    nat.check(nat.lib.lz_step(h["env"]._h, a, None, o, r_, d, h["didx"], h["tobs"], None))


def build(H):
    assert L % (2 * H) == 0, "an even number of launches per handle per graph"
    stream = torch.cuda.Stream()
    hs = make_handles(H, stream)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(stream):
        for k in range(2 * H):
            launch(hs[k % H])
        torch.cuda.synchronize()
        with torch.cuda.graph(g, stream=stream):
            for k in range(L):
                launch(hs[k % H])
    shape = nat.launch_shape(hs[0]["env"]._h, nat.CALL_STEP)
    return {"H": H, "g": g, "stream": stream, "hs": hs, "kernel": shape["kernel"]}


def timeit(run, reps):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    with torch.cuda.stream(run["stream"]):
        run["g"].replay()
        e0.record(run["stream"])
        for _ in range(reps):
            run["g"].replay()
        e1.record(run["stream"])
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / (reps * L)  # us per step


def main():
    Hs = [int(x) for x in sys.argv[1:]] or [1, 2, 4, 8]
    runs = [build(H) for H in Hs]
    bps = runs[0]["hs"][0]["env"].bytes_per_env_step
    samples = [[] for _ in Hs]
    for r in range(9):  # order rotated every round
        for j in range(len(Hs)):
            k = (r + j) % len(Hs)
            samples[k].append(timeit(runs[k], 40))
    out = {"envs_per_handle": N, "bytes_per_env_step": bps, "algorithmic_bytes_per_step": bps * N,
           "kernel": runs[0]["kernel"], "method": __doc__.split("\n\n")[1].replace("\n", " "),
           "runs": {}}
    for k, H in enumerate(Hs):
        s = sorted(samples[k])
        med = s[len(s) // 2]
        out["runs"]["H=%d" % H] = {
            "other_bytes_between_state_uses_MB": (H - 1) * bps * N / 1e6,
            "us_per_step_median": med, "us_per_step_min": s[0], "us_per_step_max": s[-1],
            "samples_us": s, "GBps_median": bps * N / med / 1e3,
            "frac_of_8TBps": bps * N / med / 1e3 / 8000.0}
    base = out["runs"]["H=%d" % Hs[0]]["us_per_step_median"]
    for v in out["runs"].values():
        v["vs_first"] = v["us_per_step_median"] / base
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
