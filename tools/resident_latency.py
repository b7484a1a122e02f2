"""Resident step server latency with several live handles (C calls only, no Python
class overhead): microseconds per lz_resident_step for
  * N = 1, 2, 4, 8, 16 one-env LORENZ3 fp64 handles stepped round robin;
  * N handles registered, only handle 0 stepped (the others' waves poll idle);
  * N handles stepped in runs of 8 calls each;
next to lz_step_host.  Separates the cost of idle polling waves from the cost of
switching between handles.  At 8 handles also: a small torch kernel + synchronize on
torch's stream with and without the server resident."""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gym-lorenz_amd"))
import gym_lorenz._native as nat  # noqa: E402
from gym_lorenz.core import BatchedEnv  # noqa: E402


def handles(n):
    out = []
    for _ in range(n):
        be = BatchedEnv("lorenz3", 1, dtype="float64", autoreset=False, compact=False)
        be.reset()
        a = np.zeros((1, 3), np.float32)
        o, r, d = np.zeros((1, 6)), np.zeros(1), np.zeros(1, np.uint8)
        out.append((be, (be._h, a.ctypes.data, None, o.ctypes.data, r.ctypes.data, d.ctypes.data),
                    (a, o, r, d)))
    return out


def run(fn, hs, order, reps):
    f = getattr(nat.lib, fn)
    for i in order[:200]:
        f(*hs[i][1])
    t0 = time.perf_counter()
    for _ in range(reps):
        for i in order:
            f(*hs[i][1])
    return (time.perf_counter() - t0) / (reps * len(order)) * 1e6


def torch_latency(hs):
    """Median microseconds of one small torch kernel + stream synchronize on torch's own
    stream: with no server, then while the server polls for the live handles."""
    import torch

    x = torch.ones(1024, device="cuda")
    s = torch.cuda.current_stream()

    def med(live):
        ts = []
        for _ in range(300):
            if live:
                nat.lib.lz_resident_step(*hs[0][1])  # keeps the server resident
            t0 = time.perf_counter()
            x.add_(1.0)
            s.synchronize()
            ts.append(time.perf_counter() - t0)
        return float(np.median(ts)) * 1e6

    for be, _, _ in hs:
        nat.check(nat.lib.lz_resident_stop(be._h))
    idle = med(False)
    for be, args, _ in hs:
        nat.lib.lz_resident_step(*args)
    return {"torch kernel + sync, no server": idle,
            "torch kernel + sync, server live for %d handles" % len(hs): med(True)}


def main():
    res = {}
    for n in (1, 2, 4, 8, 16):
        hs = handles(n)
        row = {}
        for fn in ("lz_step_host", "lz_resident_step"):
            rr = list(range(n)) * max(1, 64 // n)
            row[fn + " round robin"] = run(fn, hs, rr, 100)
            if fn == "lz_resident_step":
                row[fn + " handle 0 only"] = run(fn, hs, [0] * 64, 100)
                row[fn + " runs of 8"] = run(fn, hs, [i for i in range(n) for _ in range(8)], 50)
        if n == 8:
            row.update(torch_latency(hs))
        res["%d handles" % n] = row
        for be, _, _ in hs:
            be.close()
    print(json.dumps({"us_per_step": res}, indent=1))


if __name__ == "__main__":
    main()
