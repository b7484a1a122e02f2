"""Env-step throughput of the MI355X-native Lorenz env (the reference's dynamic.py env,
BASELINE.json metric: env-steps/s at 1M parallel Lorenz envs on 1/2/4/8 MI355X, plus
fp32 drift vs the fp64 reference arithmetic).

One "step" = one batched lz_step over every env of the shard: clip -> Euler ->
derivative -> obs -> reward -> done (+ auto-reset / done compaction), reading the
actions from and writing obs / reward / done into a 16-slot on-device rollout ring
(PPO-style rollout buffer, > 256 MiB Infinity Cache, so the I/O streams from HBM).

  python bench.py [--gpus N --steps K --warmup W]
  python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 \\
         --master-port P bench.py --gpus N ...

Multi-GPU: one process per GPU, contiguous shard of the global env axis per rank, no
collective on the step path (barrier + max-over-ranks timing only).  Default
scaling is "weak" (1,048,576 envs per GPU: N=1 is exactly the BASELINE 1M-env
config); --scaling strong splits a fixed global env count instead.
Rank 0 prints one JSON line.
"""
import argparse
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "gym-lorenz_amd"))

METRIC = "env-steps/sec at 1M parallel Lorenz envs, 1/2/4/8 MI355X; fp32 drift vs CPU"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
KERNEL = "_ZN2lz6k_stepINS_5SysL3IfEEfLi0EEEvNS_5KArgsE"


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=4000)
    p.add_argument("--warmup", type=int, default=400)
    p.add_argument("--envs", type=int, default=1 << 20, help="per-GPU env count (weak) or "
                   "global env count (strong)")
    p.add_argument("--scaling", choices=["strong", "weak"], default="weak")
    p.add_argument("--launch", choices=["graph", "eager"], default="graph")
    p.add_argument("--graph-len", type=int, default=64, help="steps per captured hipGraph")
    p.add_argument("--ring", type=int, default=16, help="rollout-ring slots for actions/obs")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--no-drift", action="store_true")
    p.add_argument("--cpu-seconds", type=float, default=12.0)
    return p.parse_args()


def cpu_baseline(seconds):
    """The oracle's scalar C port of dynamic.py's step (fp32, 1 thread) on a bounded
    sample: 65,536 envs x S steps, S calibrated to ~`seconds` of CPU work."""
    import numpy as np

    import oracle

    n = 65536
    st = oracle.reset_draw("l3", np.float32, n, 0, 0, 0).copy()
    acts = np.random.default_rng(0).uniform(-1, 1, (8, n, 3)).astype(np.float32)
    with np.errstate(all="ignore"):
        t0 = time.perf_counter()
        for k in range(4):
            oracle.l3_step(st, acts[k % 8])
        per = (time.perf_counter() - t0) / 4
        steps = max(8, int(seconds / max(per, 1e-9)))
        t0 = time.perf_counter()
        for k in range(steps):
            oracle.l3_step(st, acts[k % 8])
        dt = time.perf_counter() - t0
    return {"value": n * steps / dt, "unit": "env-steps/s", "cores": 1, "kind": "port",
            "sample": "oracle/lz_oracle.c orc_l3_step_float (scalar C restatement of "
                      "dynamic.py:86-115), 65,536 envs x %d steps = %.2e env-steps in %.1f s, "
                      "1 thread, GPU box host CPU" % (steps, n * steps, dt)}


def fp32_drift(gl, torch, device):
    """fp32 kernel vs the fp64 kernel (bit-identical to dynamic.py, see
    tests/test_gpu_parity.py::test_l3_f64_golden_bitexact), same x0 and actions:
    (a) per-step teacher-forced relative error (the BASELINE gate, < 1e-5),
    (b) the free-running max abs error curve (chaotic growth; reported only)."""
    import numpy as np

    n, T = 4096, 200
    f64 = gl.BatchedEnv("lorenz3", n, dtype="float64", seed=99, autoreset=False, device=device)
    f32 = gl.BatchedEnv("lorenz3", n, dtype="float32", seed=99, autoreset=False, device=device)
    f64.reset()
    x0 = torch.stack([f64.get_state(j) for j in range(3)], 1)
    f32.reset(init=x0.float())
    g = torch.Generator(device=device).manual_seed(7)
    acts = torch.rand((T, n, 3), generator=g, device=device) * 2 - 1
    o64, _, _ = f64.rollout(acts)
    o32, _, _ = f32.rollout(acts)
    prev = torch.cat([x0[None], o64[:-1, :, :3]], 0).reshape(T * n, 3)
    nxt = o64[:, :, :3].reshape(T * n, 3)
    # SURVEY 8d protocol: ~0.8% of U(-30,30)^3 inits overflow under Euler dt=0.01;
    # they are excluded from the error statistics (bounded states only)
    fin = (torch.isfinite(prev).all(1) & torch.isfinite(nxt).all(1)
           & (prev.abs() < 1e6).all(1) & (nxt.abs() < 1e6).all(1))
    prev, nxt, a = prev[fin], nxt[fin], acts.reshape(T * n, 3)[fin]
    tf = gl.BatchedEnv("lorenz3", prev.shape[0], dtype="float32", autoreset=False, device=device)
    tf.reset(init=prev.float().contiguous())
    o, _, _ = tf.step(a.contiguous())
    rel = ((o[:, :3].double() - nxt).abs() / nxt.abs().clamp_min(1.0)).max().item()
    err = (o32[:, :, :3].double() - o64[:, :, :3]).abs()
    bounded = ((o64[:, :, :3].abs() < 1e6).all(-1).all(0)
               & (o32[:, :, :3].abs() < 1e6).all(-1).all(0))  # envs bounded all horizon
    nonfin_agree = bool(torch.equal(torch.isfinite(o64).all(-1).all(0),
                                    torch.isfinite(o32).all(-1).all(0)))
    curve = {}
    for k in (1, 10, 50, 100, 200):
        e = err[k - 1][bounded]
        curve[str(k)] = float(e.max().item()) if e.numel() else None
    for e in (f64, f32, tf):
        e.close()
    return {"per_step_rel_max": rel, "gate": 1e-5, "pass": bool(rel < 1e-5),
            "free_running_max_abs": curve, "bounded_envs": int(bounded.sum().item()),
            "divergence_agrees": nonfin_agree,
            "vs": "fp64 kernel (bit-identical to reference dynamic.py)",
            "sample": "%d envs x %d steps, actions U(-1,1)^3" % (n, T)}


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        if world == 1 and args.gpus > 1:
            raise SystemExit("--gpus %d needs torch.distributed.run with %d processes"
                             % (args.gpus, args.gpus))
    torch.cuda.set_device(local)
    device = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", device_id=device)

    import gym_lorenz as gl
    from gym_lorenz import _native as nat
    from gym_lorenz.parallel import shard_bounds

    if args.scaling == "strong":
        total = args.envs
        start, n = shard_bounds(total, rank, world)
    else:
        n = args.envs
        total = n * world
        start = rank * n
    env = gl.BatchedEnv("lorenz3", n, dtype="float32", seed=0, global_env_offset=start,
                        autoreset=True, device=local)
    R = args.ring
    g = torch.Generator(device=device).manual_seed(1000 + rank)
    acts = torch.rand((R, n, 3), generator=g, device=device) * 2 - 1
    obs = torch.empty((R, n, 6), device=device)
    rew = torch.empty((R, n), device=device)
    done = torch.empty((R, n), dtype=torch.uint8, device=device)
    env.reset()

    h = env._h
    P = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
    slots = [(P(acts[r]), P(obs[r]), P(rew[r]), P(done[r])) for r in range(R)]
    didx, tobs = P(env.done_idx), P(env.term_obs)
    lz_step = nat.lib.lz_step

    def one(k):
        a, o, r_, d = slots[k % R]
        st = lz_step(h, a, None, o, r_, d, didx, tobs, None)
        if st:
            nat.check(st)

    stream = torch.cuda.Stream(device)
    graph = None
    L = max(2, args.graph_len - args.graph_len % 2)  # even: keeps the ping-pong parity
    if L % R and R % L:
        L = R
    with torch.cuda.stream(stream):
        nat.check(nat.lib.lz_set_stream(h, ctypes.c_void_p(stream.cuda_stream)))
        for k in range(max(args.warmup, 2)):
            one(k)
        if args.launch == "graph":
            graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(graph, stream=stream):
                for k in range(L):
                    one(k)
        torch.cuda.synchronize(device)

        def run(nsteps):
            if graph is None:
                for k in range(nsteps):
                    one(k)
                return nsteps
            reps = max(1, nsteps // L)
            for _ in range(reps):
                graph.replay()
            return reps * L

        run(max(args.warmup, L))  # warm the graph path too
        torch.cuda.synchronize(device)
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize(device)
        ev0 = torch.cuda.Event(enable_timing=True)
        ev1 = torch.cuda.Event(enable_timing=True)
        t0 = time.perf_counter()
        ev0.record(stream)
        K = run(args.steps)
        ev1.record(stream)
        torch.cuda.synchronize(device)
        if world > 1:
            dist.barrier()
        t1 = time.perf_counter()
    elapsed = t1 - t0
    ev_ms = ev0.elapsed_time(ev1)
    if world > 1:
        t = torch.tensor([elapsed, ev_ms], device=device, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, ev_ms = float(t[0]), float(t[1])

    bytes_step = env.bytes_per_env_step  # 65 B/env-step (12 state in, 12 out, 12 act, 24 obs, 4 rew, 1 done)
    launch_s = ev_ms / 1e3 / K
    achieved = bytes_step * n / launch_s / 1e9
    out = {
        "metric": METRIC,
        "value": total * K / elapsed,
        "unit": "env-steps/s",
        "n_gpus": world,
        "steps": K,
        "warmup": args.warmup,
        "ms_per_step": elapsed * 1e3 / K,
        "higher_is_better": True,
        "scaling": args.scaling,
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic: x0 ~ U(-30,30)^3 on-device Philox keyed by global env id; "
                "actions ~ U(-1,1)^3 f32 pre-generated on device",
        "config": {
            "workload": "dynamic.py 3-state Lorenz env step (lz_step, LORENZ3 fp32), "
                        "%d envs total, %d per GPU, actions/obs/reward/done in a %d-slot "
                        "on-device rollout ring" % (total, n, R),
            "system": "lorenz3", "envs_total": total, "envs_per_gpu": n,
            "parallelism": "env shard x%d (contiguous global ids, no collective on step)" % world,
            "launch": "hipGraph of %d lz_step launches" % L if graph is not None else "eager",
        },
        "roofline": {
            "bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": achieved / HBM_PEAK_GBS, "traffic": None,
            "kernel": KERNEL, "avg_launch_us": launch_s * 1e6,
            "bytes_per_env_step": bytes_step,
            "note": "achieved = algorithmic bytes per launch (bytes_per_env_step x envs_per_gpu) "
                    "/ HIP-event average launch time on the launch stream",
        },
    }
    traffic = load_traffic(n)
    if traffic is not None:
        out["roofline"]["traffic"] = traffic["bytes_per_launch"]
        out["roofline"]["traffic_source"] = traffic["source"]
    if rank == 0 and world == 1 and not args.no_drift:
        out["fp32_drift"] = fp32_drift(gl, torch, device)
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(args.cpu_seconds)
    env.close()
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    if rank == 0:
        print(json.dumps(out), flush=True)


def load_traffic(n):
    """HBM bytes per launch from the committed rocprofv3 PMC summary of this workload
    (profiles/<round>/*pmc_summary.json, written by tools/pmc_summary.py from separate
    rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes, gfx950-calibrated), if one matches
    this kernel and shard size; otherwise null."""
    import glob

    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "**", "*pmc_summary.json"),
                              recursive=True), reverse=True):  # newest round first
        try:
            d = json.load(open(f))
        except Exception:  # noqa: BLE001
            continue
        if d.get("kernel") == KERNEL and d.get("envs_per_gpu") == n:
            return {"bytes_per_launch": d["hbm_bytes_per_launch"],
                    "source": os.path.relpath(f, ROOT)}
    return None


if __name__ == "__main__":
    main()
