"""Time lz_gae alone (RolloutBuffer.compute_returns_and_advantage) on device buffers.

  python tools/gae_bench.py [n] [K] [reps]      (default cfg5's 32,768 envs x 2048 steps)

Prints one JSON line: average launch time (HIP events on the launch stream), the
algorithmic bytes (4 B reward + 4 B value + 1 B done read, 8 B written per env-step)
and a checksum of the outputs so A/B builds (LZ_LIB_AB) can be compared bit-for-bit.
"""
import ctypes
import hashlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gym-lorenz_amd"))

import torch  # noqa: E402

from gym_lorenz import _native as nat  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 32768
    K = int(sys.argv[2]) if len(sys.argv) > 2 else 2048
    reps = int(sys.argv[3]) if len(sys.argv) > 3 else 50
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(0)
    rew = torch.randn(K, n, device=dev, generator=g)
    val = torch.randn(K, n, device=dev, generator=g)
    done = (torch.rand(K, n, device=dev, generator=g) < 0.01).to(torch.uint8)
    last = torch.randn(n, device=dev, generator=g)
    adv = torch.empty_like(rew)
    ret = torch.empty_like(rew)
    s = torch.cuda.current_stream(dev)
    p = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731

    def call():
        nat.check(nat.lib.lz_gae(n, K, p(rew), p(val), p(done), p(last), 0.99, 0.95, p(adv),
                                 p(ret), 0, ctypes.c_void_p(s.cuda_stream)))

    for _ in range(5):
        call()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record(s)
    for _ in range(reps):
        call()
    e1.record(s)
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / reps
    h = hashlib.sha256(adv.cpu().numpy().tobytes() + ret.cpu().numpy().tobytes()).hexdigest()
    nbytes = 17 * n * K
    print(json.dumps({"n": n, "K": K, "avg_launch_us": us, "GB_per_s": nbytes / us / 1e3,
                      "lib": os.environ.get("LZ_LIB_AB", "default"), "sha256": h[:16]}))


if __name__ == "__main__":
    main()
