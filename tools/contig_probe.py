"""Rollout time (LORENZ3, K = 2048) vs how its buffers were allocated: torch's caching
allocator (what bench.py uses), plain hipMalloc, and hipExtMallocWithFlags with
hipDeviceMallocContiguous (physically contiguous: large page-table fragments).  Three
fresh allocations per kind (placement varies between allocations of the same size by up
to ~18%, tools/placement_probe.py shows offsets inside one allocation do not matter).
HIP-event time per launch on the env's stream, median of 5 after 2 warm.

  python tools/contig_probe.py [envs] -> one JSON line per allocation
"""
import ctypes
import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "gym-lorenz_amd"))
import gym_lorenz as gl  # noqa: E402
from gym_lorenz import _native as nat  # noqa: E402

hip = ctypes.CDLL("libamdhip64.so")
hip.hipExtMallocWithFlags.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t, ctypes.c_uint]
hip.hipMalloc.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t]
hip.hipFree.argtypes = [ctypes.c_void_p]
hip.hipMemset.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t]
CONTIG = 0x4


def raw(nbytes, kind):
    p = ctypes.c_void_p()
    st = hip.hipExtMallocWithFlags(ctypes.byref(p), nbytes, CONTIG) if kind == "contig" else \
        hip.hipMalloc(ctypes.byref(p), nbytes)
    if st != 0:
        raise RuntimeError("alloc %s %d: %d" % (kind, nbytes, st))
    hip.hipMemset(p, 0, nbytes)
    return p


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 262144
    K = 2048
    be = gl.BatchedEnv("lorenz3", n, seed=0)
    be.reset()
    stream = torch.cuda.Stream()
    nat.check(nat.lib.lz_set_stream(be._h, ctypes.c_void_p(stream.cuda_stream)))
    # raw (non-torch) buffers cannot go through BatchedEnv.rollout_args: size them from
    # lz_info here (actions [K, N, A] f32, obs [K, N, O] f32, rew [K, N] f32, done [K, N] u8)
    sizes = (K * n * be.action_dim * 4, K * n * be.obs_dim * 4, K * n * 4, K * n)

    def timed(ptrs):
        a, o, r, d = (ctypes.c_void_p(p.value if isinstance(p, ctypes.c_void_p) else p) for p in ptrs)
        run = lambda: nat.check(nat.lib.lz_rollout(be._h, K, a, o, r, d, None, None, 0, None))  # noqa: E731
        with torch.cuda.stream(stream):
            for _ in range(2):
                run()
            ts = []
            for _ in range(5):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(stream)
                run()
                e1.record(stream)
                stream.synchronize()
                ts.append(e0.elapsed_time(e1) * 1e3)
        return sorted(ts)[2]

    for rep in range(3):
        for kind in ("torch", "hipMalloc", "contig"):
            if kind == "torch":
                ts = [torch.zeros(s // 4 if i < 3 else s, dtype=torch.float32 if i < 3 else torch.uint8,
                                  device=be.device) for i, s in enumerate(sizes)]
                us = timed([t.data_ptr() for t in ts])
                del ts
                torch.cuda.empty_cache()
            else:
                try:
                    ps = [raw(s, kind) for s in sizes]
                except RuntimeError as e:
                    print(json.dumps({"kind": kind, "rep": rep, "error": str(e)}), flush=True)
                    continue
                us = timed(ps)
                for p in ps:
                    hip.hipFree(p)
            print(json.dumps({"envs": n, "kind": kind, "rep": rep, "us_median": us,
                              "env_steps_per_s": n * K / us * 1e6}), flush=True)


if __name__ == "__main__":
    main()
