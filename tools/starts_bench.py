"""Episode-starts of one collect: the three torch launches collect() used to run
(compare, convert + copy, row copy) against the single lz_episode_starts kernel, timed
in one process with HIP events on the current stream.

  python tools/starts_bench.py [n] [K] [reps]     (default 262,144 envs x 16 steps)
"""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gym-lorenz_amd"))

import torch  # noqa: E402

from gym_lorenz import _native as nat  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 262144
    K = int(sys.argv[2]) if len(sys.argv) > 2 else 16
    reps = int(sys.argv[3]) if len(sys.argv) > 3 else 200
    dev = torch.device("cuda:0")
    done = torch.randint(0, 4, (K, n), device=dev, dtype=torch.uint8)
    last = torch.ones(n, device=dev)
    s = torch.cuda.current_stream(dev)
    p = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731

    def torch_path():
        starts = torch.empty((K, n), dtype=torch.float32, device=dev)
        starts[0] = last
        starts[1:] = (done[:-1] != 0).to(torch.float32)
        return starts, (done[-1] != 0).to(torch.float32)

    def kernel_path():
        starts = torch.empty((K, n), dtype=torch.float32, device=dev)
        out = torch.empty((n,), dtype=torch.float32, device=dev)
        nat.check(nat.lib.lz_episode_starts(n, K, p(done), p(last), p(starts), p(out), 0,
                                            ctypes.c_void_p(s.cuda_stream)))
        return starts, out

    a, b = torch_path(), kernel_path()
    assert torch.equal(a[0], b[0]) and torch.equal(a[1], b[1])
    res = {"n": n, "K": K}
    for name, f in (("torch", torch_path), ("kernel", kernel_path)) * 2:
        for _ in range(10):
            f()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        e0.record(s)
        for _ in range(reps):
            f()
        e1.record(s)
        torch.cuda.synchronize()
        res[name + "_us"] = e0.elapsed_time(e1) * 1e3 / reps
    print(json.dumps(res))


if __name__ == "__main__":
    main()
