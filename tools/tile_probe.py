"""Probe: is the two-tile LORENZ3 step at 262,144 envs bimodal across handles inside ONE
process (buffer placement) or only across processes (r06 stage V: 3.87 / 4.23 / 4.25 us
per step on one box, one tile 3.96 - 4.02)?  Creates H handles one after another (all
kept alive, so every handle's planes and ring sit at new addresses), each with bench.py's
16-slot ring and a captured 64-launch hipGraph, and times 60 replays per handle for the
default (two tiles) and variant 16384 (one tile).  Prints one JSON line per handle."""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "gym-lorenz_amd"))


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--envs", type=int, default=262144)
    p.add_argument("--handles", type=int, default=6)
    p.add_argument("--replays", type=int, default=60)
    a = p.parse_args()
    import torch

    import bench
    import gym_lorenz as gl
    from gym_lorenz import _native as nat

    dev = torch.device("cuda", 0)
    args = argparse.Namespace(ring=16, K=1, system="lorenz3")
    keep = []
    for hnd in range(a.handles):
        row = {"handle": hnd}
        for v in (0, 16384):
            env = gl.BatchedEnv("lorenz3", a.envs, dtype="float32", seed=0, autoreset=True, device=0,
                                variant=v)
            ln = bench._Lane(args, torch, nat, env, dev, 0, False, hnd)
            with torch.cuda.stream(ln.stream):
                for _ in range(8):
                    ln.one()
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g, stream=ln.stream):
                    for _ in range(64):
                        ln.one()
            torch.cuda.synchronize(dev)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            with torch.cuda.stream(ln.stream):
                for _ in range(5):
                    g.replay()
                e0.record(ln.stream)
                for _ in range(a.replays):
                    g.replay()
                e1.record(ln.stream)
            torch.cuda.synchronize(dev)
            us = e0.elapsed_time(e1) * 1e3 / (a.replays * 64)
            shape = nat.launch_shape(env._h, nat.CALL_STEP)
            row["v%d_us" % v] = round(us, 3)
            row["v%d_kernel" % v] = shape["kernel"]
            row["v%d_ring_mod2M" % v] = [t.data_ptr() % (1 << 21) for t in ln.buf]
            keep.append((env, ln, g))
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
