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
collective on the step path (barrier + max-over-ranks timing only).  `--gpus N` without
a torch.distributed.run environment (no WORLD_SIZE) spawns the N rank processes itself
(child processes started before anything touches the GPU; rank r pins cuda:r).  Default
scaling is "strong": BASELINE's 1,048,576 envs in total, split over the N GPUs
(configs[2]: 131,072 per GPU at N = 8; N = 1 is the 1M-env config itself); for N > 1
the line also carries the weak 1M-per-GPU run and the step + RCCL gather of obs /
reward / done to rank 0 (north_star's optional learner gather) in `extra_lines`.
--scaling weak makes the weak run the headline.  Rank 0 prints one JSON line.
"""
import argparse
import math
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "gym-lorenz_amd"))

METRIC = "env-steps/sec at 1M parallel Lorenz envs, 1/2/4/8 MI355X; fp32 drift vs CPU"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
MFMA_BF16_PEAK_TFLOPS = 2500.0  # MI355X_MICROARCH.md: dense bf16 MFMA (no sparsity)
MFMA_F32_PEAK_TFLOPS = 157.3  # dense f32-input MFMA (= the f32 vector peak), MI355X_MICROARCH.md


def parse(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=4000)
    p.add_argument("--warmup", type=int, default=400)
    p.add_argument("--envs", type=int, default=1 << 20, help="per-GPU env count (weak) or "
                   "global env count (strong)")
    p.add_argument("--scaling", choices=["strong", "weak"], default="strong",
                   help="strong (default): --envs is the global env count split over the GPUs "
                        "(BASELINE configs[2]); weak: --envs per GPU")
    p.add_argument("--launch", choices=["graph", "eager"], default="graph")
    p.add_argument("--graph-len", type=int, default=64, help="steps per captured hipGraph")
    p.add_argument("--ring", type=int, default=16, help="rollout-ring slots for actions/obs")
    p.add_argument("--head-eager", type=int, default=0,
                   help="step mode: launch each timed window's first E (even) steps eagerly, the "
                        "rest from graphs (0 = off)")
    p.add_argument("--head-graph", type=int, default=0,
                   help="step mode: launch each timed window's first H (even) steps as a graph of "
                        "their own, so the GPU starts on them while the host submits the rest "
                        "(0 = off)")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--no-drift", action="store_true")
    p.add_argument("--no-extras", action="store_true",
                   help="skip the extra lines of the headline run (fp64 reference precision)")
    p.add_argument("--cpu-seconds", type=float, default=12.0)
    p.add_argument("--system", choices=["lorenz3", "lorenz4", "pmsm", "hr"], default="lorenz3",
                   help="lorenz3 = the BASELINE headline (dynamic.py env); pmsm = cfg4")
    p.add_argument("--mode", choices=["step", "rollout", "policy", "vecnorm"], default="step",
                   help="rollout = cfg5's fused K-step on-device rollout; policy = the fused "
                        "SB3 actor-critic rollout (lz_rollout_policy + VecNormalize + GAE); "
                        "vecnorm = VecNormalize(VecEnv).step fused (lz_step_vecnorm + "
                        "lz_vecnorm_apply), 1 GPU")
    p.add_argument("--K", type=int, default=2048, help="rollout length (--mode rollout)")
    p.add_argument("--dtype", choices=["float32", "float64"], default="float32",
                   help=argparse.SUPPRESS)  # A/B: the env arithmetic of the main line
    p.add_argument("--add-noise", type=int, choices=[0, 1], default=None,
                   help=argparse.SUPPRESS)  # A/B: the process-noise flag (default: the config's)
    p.add_argument("--precision", choices=["fp32", "bf16", "i8x4"], default="fp32",
                   help="--mode policy --policy mlp: fp32 = SB3's float32 forward "
                        "(lz_rollout_policy_f32), bf16 = the bf16-MFMA kernel")
    p.add_argument("--vecnorm-update", choices=["step", "rollout"], default="step",
                   help="--mode policy --policy mlp fp32: step = SB3's VecNormalize order (obs_rms "
                        "updated by every step's batch before it is normalised; one launch per "
                        "step, lz_rollout_policy_f32_vn); rollout = one K-step launch with the "
                        "rollout-start statistics and a pooled update (opt-in, not SB3's order)")
    p.add_argument("--policy", choices=["mlp", "attn", "attn_ln"], default="mlp",
                   help="--mode policy: mlp = SB3 MlpPolicy behind VecNormalize (the PMSM A2C "
                        "learner, code/lorenz_pmsm/train.py); attn = code/train.py's PPO policy "
                        "with the AttentionFeaturesExtractor (no VecNormalize, as there); "
                        "attn_ln = code/lorenz_filter/train.py's residual + LayerNorm extractor "
                        "on VecFrameStack(4)")
    p.add_argument("--ic-flush-mib", type=int, default=0,
                   help="A/B only (profiles/r05/ic/): after every lz_step copy a buffer of this many "
                        "MiB on the step's stream, so two uses of a state line are more than the "
                        "256 MiB Infinity Cache apart; the step kernel's own time comes from "
                        "rocprofv3 --kernel-trace (this line's value includes the copies)")
    p.add_argument("--ic-flush-kind", choices=["copy", "read"], default="copy",
                   help="--ic-flush-mib: copy the buffer (reads + writes) or only read it (a sum)")
    p.add_argument("--variant", type=int, default=0,
                   help="step-kernel tuning variant (lz_config.reserved[0]; A/B only, e.g. "
                        "16384 / 32768 / 49152 force 1 / 2 / 4 tiles per PMSM / HR workgroup)")
    p.add_argument("--max-episode-steps", type=int, default=0,
                   help="TimeLimit truncation (auto-reset inside the kernel); 0 = none")
    p.add_argument("--integrator", choices=["euler", "rk4"], default="euler",
                   help="euler = the reference's (dynamic.py:70-75); rk4 = the opt-in RK4 mode "
                        "of lorenz3 / lorenz4 (lz_config.integrator)")
    p.add_argument("--streams", type=int, default=0,
                   help="step mode: split each rank's shard into S sub-handles of consecutive "
                        "global env ids, each stepping on its own HIP stream with its own "
                        "captured graphs, so the S dependent-launch chains overlap (1..4: "
                        "GPU_MAX_HW_QUEUES is 4); 0 = auto (default_streams)")
    p.add_argument("--no-gather", action="store_true",
                   help="N > 1: skip the step + gather-to-rank-0 extra line")
    p.add_argument("--probe-ranks", action="store_true", help=argparse.SUPPRESS)
    return p.parse_args(argv)


def _cpu_worker(kind, seconds):
    """One host core's share of the CPU baseline (run in a spawned process): returns
    (env-steps, seconds) of `kind` = "ref" (oracle/ref_loop.py, the reference's own per-env
    NumPy step in a DummyVecEnv loop) or "port" (the oracle's scalar C step)."""
    import numpy as np

    sys.path.insert(0, ROOT)
    if kind == "ref":
        from oracle.ref_loop import LorenzRefEnv, dummy_vec_step

        n = 1024
        envs = [LorenzRefEnv(x) for x in np.random.default_rng(0).uniform(-30, 30, (n, 3))]
        acts = np.random.default_rng(1).uniform(-1, 1, (n, 3)).astype(np.float32)
        bo, br = np.zeros((n, 6), np.float32), np.zeros(n, np.float32)
        step = lambda k: dummy_vec_step(envs, acts, bo, br)  # noqa: E731
    else:
        import oracle

        n = 65536
        st = oracle.reset_draw("l3", np.float32, n, 0, 0, 0).copy()
        acts = np.random.default_rng(0).uniform(-1, 1, (8, n, 3)).astype(np.float32)
        step = lambda k: oracle.l3_step(st, acts[k % 8])  # noqa: E731
    with np.errstate(all="ignore"):
        t0 = time.perf_counter()
        k = 0
        while time.perf_counter() - t0 < seconds:
            step(k)
            k += 1
        dt = time.perf_counter() - t0
    return n * k, dt


def _cpu_run(kind, seconds, cores):
    if cores == 1:
        steps, dt = _cpu_worker(kind, seconds)
        return steps / dt, steps, dt
    import multiprocessing as mp

    with mp.get_context("spawn").Pool(cores) as pool:
        res = pool.starmap(_cpu_worker, [(kind, seconds)] * cores)
    steps = sum(r[0] for r in res)
    dt = max(r[1] for r in res)
    return steps / dt, steps, dt


def host_cores():
    """Host cores of this process's share: the affinity mask, at most 16 (a one-GPU box's
    CPU share; os.cpu_count() there shows the whole machine)."""
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    return max(1, min(n, 16))


def cpu_baseline(seconds):
    """The reference's own cost model on the host: dynamic.py's step() per env object in
    a DummyVecEnv-style loop (oracle/ref_loop.py, pinned bit-exact to the reference's
    outputs; the reference itself does not travel to the GPU box), one process per host
    core (spawned before the GPU is initialised) and on one core; beside it the oracle's
    scalar C port.  Bounded samples: ~`seconds` / 4 of wall time per measurement."""
    cores = host_cores()
    w = max(1.0, seconds / 4)
    ref_all, ref_steps, ref_dt = _cpu_run("ref", w, cores)
    ref_one, one_steps, one_dt = _cpu_run("ref", w, 1)
    port_all, port_steps, port_dt = _cpu_run("port", w, cores)
    port_one, p1_steps, p1_dt = _cpu_run("port", w, 1)
    return {
        "value": ref_all, "unit": "env-steps/s", "cores": cores, "kind": "port",
        "sample": "oracle/ref_loop.py (dynamic.py:61-90 step() with the reference's per-call "
                  "NumPy work: 3 np.clip, 4 list - int64 array observations, generator-sum "
                  "reward; bit-exact vs the reference fixture) driving 1024 envs per process "
                  "in a DummyVecEnv-style loop, %d processes (one per host core) for %.1f s: "
                  "%.2e env-steps; GPU box host CPU" % (cores, ref_dt, ref_steps),
        "one_core": {"value": ref_one, "cores": 1,
                     "sample": "the same loop, 1 process, %.2e env-steps in %.1f s"
                               % (one_steps, one_dt)},
        "c_port": {"value": port_all, "cores": cores, "one_core": port_one, "kind": "port",
                   "sample": "oracle/lz_oracle.c orc_l3_step_float (scalar C restatement of "
                             "dynamic.py:61-90, fp32), 65,536 envs per process, %d processes "
                             "%.2e env-steps in %.1f s; 1 process %.2e env-steps in %.1f s"
                             % (cores, port_steps, port_dt, p1_steps, p1_dt)},
    }


def fp32_drift(gl, torch, device):
    """fp32 kernel vs the fp64 kernel (bit-identical to dynamic.py, see
    tests/test_gpu_parity.py::test_l3_f64_golden_bitexact), same x0 and actions:
    (a) per-step teacher-forced relative error (the BASELINE gate, < 1e-5),
    (b) the free-running max abs error curve (chaotic growth; reported only)."""
    import numpy as np

    n, T = 4096, 1000  # north_star's horizon: 1000 steps
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
    for k in (1, 10, 50, 100, 200, 500, 1000):
        e = err[k - 1][bounded]
        curve[str(k)] = float(e.max().item()) if e.numel() else None
    for e in (f64, f32, tf):
        e.close()
    return {"per_step_rel_max": rel, "gate": 1e-5, "pass": bool(rel < 1e-5),
            "free_running_max_abs": curve, "bounded_envs": int(bounded.sum().item()),
            "divergence_agrees": nonfin_agree,
            "vs": "fp64 kernel (bit-identical to reference dynamic.py)",
            "sample": "%d envs x %d steps, actions U(-1,1)^3" % (n, T)}


SYSTEM_INFO = {  # system -> (reference env, mangled k_step / k_rollout names, action range)
    "lorenz3": ("dynamic.py 3-state Lorenz env", "SysL3IfEEf", 1.0),
    "lorenz4": ("lorenz_env_transient.py 4-state master/slave env", "SysL4IfEEf", 2.0),
    "pmsm": ("lorenz_env_try_pmsm.py PMSM sync env (add_noise=True, alpha=0.5)", "SysPMSMEf", 1.2),
    "hr": ("lorenz_env_try.py Hindmarsh-Rose RK4 env", "SysHRIfEEf", 1.2),
}


def step_tiles(system, n, f64=False, num_cus=256, variant=0, integrator="euler"):
    """Tiles per workgroup of the step launch: lz_kernels.hip step_tiles (variant bits
    14-15 force 1 / 2 / 4) and step_tiles_balanced (LORENZ3 / PMSM / HR float32: 4 where
    that grid puts exactly 4 -- LORENZ3 / PMSM: or 3 -- workgroups on every CU, else 1)."""
    if system not in ("pmsm", "hr", "lorenz3") or f64 or integrator == "rk4":
        return 1
    forced = (variant >> 14) & 3
    if forced:
        return {1: 1, 2: 2, 3: 4}[forced]
    # step_tiles_balanced: exactly 4 (LORENZ3 / PMSM: or 3) workgroups of 1,024 envs per CU
    groups = -(-n // 1024)
    return 4 if groups == 4 * num_cus or (system != "hr" and groups == 3 * num_cus) else 1


def kernel_name(system, mode, n, f64=False, no_done=False, num_cus=256, variant=0,
                integrator="euler", noise=None):
    """Mangled name of the dominant kernel (lz_kernels.hip launch_all / launch_rollout_d).
    no_done: a rollout launch that cannot produce a done (LORENZ3 without a TimeLimit)
    runs the done-free instantiation (kNoDone = true).  integrator "rk4": SysL3RK4 /
    SysL4RK4 (lz_systems.h), which take the generic launcher bounds.  noise: the launch
    draws process noise (default: PMSM, as this bench configures it) -- the one-wave
    rollout then runs with a noise-producer wave (k_rollout kNP)."""
    tag = SYSTEM_INFO[system][1]
    if f64:
        tag = tag.replace("IfEEf", "IdEEd")
    rk4 = integrator == "rk4" and system in ("lorenz3", "lorenz4")
    if rk4:
        tag = tag.replace("I", "RK4I", 1)
    name = tag[: tag.index("I")] if "I" in tag else tag[: tag.index("E")]
    sysname = str(len(name)) + tag
    if mode != "rollout":
        tiles = step_tiles(system, n, f64, num_cus, variant, integrator)
        if tiles > 1:  # k_step_multi<Sys, T, E, kDoneT = false>
            return "_ZN2lz12k_step_multiINS_%sLi%dELb0EEEvNS_5KArgsE" % (sysname, tiles)
        return "_ZN2lz6k_stepINS_%sLi0EEEvNS_5KArgsE" % sysname
    D = 7  # kDmaDist
    # lz_kernels.hip rollout_pair: PMSM where its 32-env waves are 2 < waves / CU <= 4
    force_other = variant & (256 | 512 | (1 << 23) | (1 << 24) | (1 << 25) | (1 << 26))
    if system == "pmsm" and not variant & (1 << 28) and (
            variant & (1 << 27) or (not force_other and 2 * num_cus < -(-n // 32) <= 4 * num_cus)):
        # the lane-pair rollout: k_rollout_pair<SysPMSM, float, D>
        return "_ZN2lz14k_rollout_pairINS_7SysPMSMEfLi%dEEEvNS_5KArgsE" % D
    b = "Lb%dE" % int(no_done and system == "lorenz3")  # (SysL3RK4 never terminates either)
    # lz_kernels.hip launch_rollout_d: one-wave workgroups below 256 x CUs envs for
    # LORENZ3 f32 (3/4 of that for LORENZ4 f32, 131,072 for the others); two lanes per env for LORENZ3
    # f32 from 32,768; temporal done stores by default (split SV = 1, k_rollout kDoneT = true)
    one_wave_below = (256 * num_cus if system == "lorenz3" and not f64 and not rk4
                      else 256 * num_cus * 3 // 4 if system == "lorenz4" and not f64 and not rk4
                      else 2 * 256 * 256)
    if n < one_wave_below:
        # rollout_split: variant 256 / 512 force one / two lanes per env (every system's
        # obs width is even), else LORENZ3 f32 (Euler) from 32,768
        if not variant & 256 and (variant & 512 or (system == "lorenz3" and not f64 and not rk4
                                                   and n >= 32768)):
            return "_ZN2lz15k_rollout_splitINS_%sLi2ELi%dE%sLi1EEEvNS_5KArgsE" % (sysname, D, b)
        if (system == "pmsm" if noise is None else noise) and system in ("pmsm", "hr") \
                and variant & (1 << 25):  # opt-in noise-producer wave
            return "_ZN2lz12k_rollout_npINS_%sLi%dEEEvNS_5KArgsE" % (sysname, D)
    # k_rollout<Sys, T, B, D, kNoDone, kDoneT = true, kZN>: kZN (variant bit 1<<26) = the next
    # step's normals drawn during this step, noisy systems only
    zn = "Lb%dE" % int(bool(variant & (1 << 26)) and system in ("pmsm", "hr")
                       and bool(system == "pmsm" if noise is None else noise))
    if n < one_wave_below:
        return "_ZN2lz9k_rolloutINS_%sLi64ELi%dE%sLb1E%sEEvNS_5KArgsE" % (sysname, D, b, zn)
    return "_ZN2lz9k_rolloutINS_%sLi256ELi%dE%sLb1E%sEEvNS_5KArgsE" % (sysname, D, b, zn)


def bench_vecnorm(args, gl, nat, torch, env, device, world, total, n):
    """--mode vecnorm: one SB3 VecNormalize(norm_obs, norm_reward, clip_obs=10) step per
    step (code/lorenz_pmsm/train.py:170), fused: lz_step_vecnorm (step + float64 moment
    partials) and lz_vecnorm_apply (fixed-order reduction, RunningMeanStd updates + normalised
    obs / reward / terminal rows, bool dones); actions / outputs in a 16-slot ring, a
    hipGraph of 64 steps.  Per-rank statistics (the all-reduce of the multi-GPU path,
    LZ_VN_DEFER, is not captured here)."""
    A, O = env.action_dim, env.obs_dim
    R, L = 16, 64
    g = torch.Generator(device=device).manual_seed(1000)
    arange = SYSTEM_INFO[args.system][2]
    acts = (torch.rand((R, n, A), generator=g, device=device) * 2 - 1) * arange
    raw_o = torch.empty((R, n, O), device=device)
    raw_r = torch.empty((R, n), device=device)
    done = torch.empty((R, n), dtype=torch.uint8, device=device)
    obs_n = torch.empty((R, n, O), device=device)
    rew_n = torch.empty((R, n), device=device)
    dones = torch.empty((R, n), dtype=torch.uint8, device=device)
    didx = torch.empty((n + 1,), dtype=torch.int32, device=device)
    tobs, tn = torch.empty((n, O), device=device), torch.empty((n, O), device=device)
    from gym_lorenz.vec_normalize import DeviceRunningMeanStd

    stream = torch.cuda.Stream(device)
    obs_rms = DeviceRunningMeanStd(O, device, stream=stream)
    ret_rms = DeviceRunningMeanStd(1, device, stream=stream)
    returns = torch.zeros((n,), dtype=torch.float64, device=device)
    vn = nat.LzVecNorm()
    vn.obs_rms, vn.ret_rms = obs_rms._h.value, ret_rms._h.value
    vn.returns = returns.data_ptr()
    vn.gamma, vn.epsilon, vn.clip_obs, vn.clip_reward = 0.99, 1e-8, 10.0, 10.0
    vn.flags = nat.VN_TRAINING | nat.VN_NORM_OBS | nat.VN_NORM_REWARD
    h = env._h
    env.reset()
    nd = didx.data_ptr() + 4 * n
    for r in range(R):  # lz_step_vecnorm takes lz_step's buffers: the same checked entry
        env.step_args(acts[r], raw_o[r], raw_r[r], done[r], didx[:n], tobs, didx[n:])
        env.step_args(acts[r], obs_n[r], rew_n[r], dones[r])

    def one(k):
        r = k % R
        nat.check(nat.lib.lz_step_vecnorm(h, vn, acts[r].data_ptr(), raw_o[r].data_ptr(),
                                          raw_r[r].data_ptr(), done[r].data_ptr(), didx.data_ptr(),
                                          tobs.data_ptr(), nd))
        nat.check(nat.lib.lz_vecnorm_apply(h, vn, raw_o[r].data_ptr(), raw_r[r].data_ptr(),
                                           done[r].data_ptr(), obs_n[r].data_ptr(),
                                           rew_n[r].data_ptr(), dones[r].data_ptr(),
                                           tobs.data_ptr(), nd, tn.data_ptr()))

    with torch.cuda.stream(stream):
        nat.check(nat.lib.lz_set_stream(h, ctypes.c_void_p(stream.cuda_stream)))
        for k in range(4):
            one(k)
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph, stream=stream):
            for k in range(L):
                one(k)
        for _ in range(max(1, args.warmup // L)):
            graph.replay()
        torch.cuda.synchronize(device)
        reps = max(1, args.steps // L)
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        while True:  # whole graphs of L steps; re-timed with more replays until >= 200 ms
            t0 = time.perf_counter()
            ev0.record(stream)
            for _ in range(reps):
                graph.replay()
            ev1.record(stream)
            torch.cuda.synchronize(device)
            t1 = time.perf_counter()
            if t1 - t0 >= 0.2 or reps >= 1 << 16:
                break
            reps = int(reps * min(64.0, 0.25 / max(t1 - t0, 1e-6))) + 1
    steps = reps * L
    elapsed = t1 - t0
    step_s = ev0.elapsed_time(ev1) / 1e3 / steps
    info = env.info
    es = 4
    bytes_step = info.bytes_per_env_step + 16 + 2 * (O * es + es + 1)
    achieved = bytes_step * n / step_s / 1e9
    obs_rms.close()
    ret_rms.close()
    # PMC bytes of the two kernels (tools/pmc_vecnorm.sh summaries), when committed for
    # this system and size
    tr = [load_traffic(k, n) for k in (
        "_ZN2lz9k_step_vnINS_7SysPMSMEfLi24EEEvNS_5KArgsENS_5VArgsE",
        "_ZN12_GLOBAL__N_110k_vn_applyIfLi6ELb1EEEvNS_11VnApplyArgsE")] if args.system == "pmsm" else [None]
    traffic = sum(t["bytes_per_launch"] for t in tr) if all(tr) else None
    return {
        "metric": METRIC, "value": total * steps / elapsed, "unit": "env-steps/s",
        "n_gpus": world, "steps": steps, "warmup": args.warmup,
        "ms_per_step": elapsed * 1e3 / steps, "higher_is_better": True,
        "timing": {"requested_steps": args.steps, "timed_steps": steps,
                   "timed_seconds": elapsed, "graph_steps": L,
                   "method": "hipGraph replays of L fused steps, the count raised until the "
                             "timed region is >= 200 ms"},
        "scaling": args.scaling, "vs_baseline": None, "dtype": "f32 env, f64 statistics",
        "data": "synthetic: on-device Philox initial states; actions ~ U(-%g,%g) f32 "
                "pre-generated on device" % (arange, arange),
        "config": {
            "workload": "VecNormalize(norm_obs, norm_reward, clip_obs=10) over %s, fused step "
                        "(lz_step_vecnorm + lz_vecnorm_apply: 2 kernels, no host sync), %d envs"
                        % (SYSTEM_INFO[args.system][0], n),
            "system": args.system, "envs_total": total, "envs_per_gpu": n, "mode": "vecnorm",
            "parallelism": "env shard x%d (per-rank statistics)" % world,
            "launch": "hipGraph of %d steps" % L},
        "roofline": {
            "bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
            "traffic_source": [t["source"] for t in tr] if traffic else None,
            "kernel": "k_step_vn + k_vn_apply (one fused VecNormalize step)",
            "avg_launch_us": step_s * 1e6, "bytes_per_env_step": bytes_step,
            "note": "achieved = algorithmic bytes of the whole fused step (lz_step's + 16 B of "
                    "float64 returns + the normalise pass: raw obs/reward/done read, normalised "
                    "obs/reward/dones written) / HIP-event time per step"},
    }


def policy_flops(O, A, H=128):
    """Useful FLOP per env-step of the SB3 MlpPolicy forward (pi and vf nets)."""
    return 2 * (O * H + H * H + H * A) + 2 * (O * H + H * H + H)


def attn_policy_flops(O, A, H=128, F=64):
    """Useful FLOP per env-step of code/train.py's attention actor-critic as SB3 runs it:
    fc1, in_proj (8 tokens x 48 x 16), scores and weights @ v (4 heads, 8 x 8 x 4),
    out_proj (8 x 16 x 16), post_attention_fc (128 -> 64), then the pi and vf nets on
    the 64 features."""
    ext = 2 * (O * H + 8 * 48 * 16 + 2 * 4 * 8 * 8 * 4 + 8 * 16 * 16 + H * F)
    return ext + 2 * (F * H + H * H + H * A) + 2 * (F * H + H * H + H)


def bench_policy(args, gl, nat, torch, env, device, world, rank, total, n):
    """--mode policy: the reference's PMSM learner loop (code/lorenz_pmsm/train.py:155-178:
    A2C MlpPolicy pi/vf [128,128] Tanh, VecNormalize(norm_obs, clip_obs=10), n_steps=16)
    collected on the GPU: per rollout one lz_rollout_policy launch (K steps of policy
    forward + sample + env step + bootstrap), the obs_rms update from its moments, and
    lz_gae.  One "step" = one env step of every env (policy forward included)."""
    import torch.distributed as dist

    from gym_lorenz.policy import ActorCriticAttn, ActorCriticMlp, FusedRolloutCollector
    from gym_lorenz.vec_normalize import DeviceRunningMeanStd

    K = args.K
    O, A = env.obs_dim, env.action_dim
    attn = args.policy in ("attn", "attn_ln")
    ln = args.policy == "attn_ln"
    stack = 4 if ln else 1
    # SB3 init (orthogonal, log_std 0): random weights
    net = (ActorCriticAttn(stack * O, A, seed=0, layer_norm=ln) if attn
           else ActorCriticMlp(O, A, seed=0))
    rms = None if attn else DeviceRunningMeanStd(O, device)
    f32 = args.precision in ("fp32", "i8x4")
    i8 = args.precision == "i8x4"
    if i8 and not attn and args.vecnorm_update == "step":
        raise SystemExit("--precision i8x4 --policy mlp runs the fused rollout: add --vecnorm-update "
                         "rollout (the per-step VecNormalize collect is float32 only)")
    per_step = f32 and not attn and args.vecnorm_update == "step"
    col = FusedRolloutCollector(env, net.state_dict(), gamma=0.99, gae_lambda=0.95, obs_rms=rms,
                                clip_obs=10.0, training=True, bootstrap=True, frame_stack=stack,
                                group=dist.group.WORLD if world > 1 else None,
                                precision=args.precision,
                                vecnorm_update=("step" if per_step else "rollout")
                                if f32 and not attn else None)
    assert col.per_step_vecnorm == per_step
    stream = torch.cuda.Stream(device)
    with torch.cuda.stream(stream):
        nat.check(nat.lib.lz_set_stream(env._h, ctypes.c_void_p(stream.cuda_stream)))
        if rms is not None:
            nat.check(nat.lib.lz_rms_set_stream(rms._h, ctypes.c_void_p(stream.cuda_stream)))
        col.reset()
        launches = max(2, args.steps // K)
        warm = 2

        def one():
            b = col.collect(K)
            col.compute_returns_and_advantage(b)

        for _ in range(warm):
            one()
        torch.cuda.synchronize(device)
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize(device)
        t0 = time.perf_counter()
        for _ in range(launches):
            one()
        torch.cuda.synchronize(device)
        t1 = time.perf_counter()  # this rank's K steps; the job's time is the MAX over ranks
        if world > 1:
            dist.barrier()
        # the dominant kernel alone (k_rollout_policy), HIP events on its stream
        evs = [torch.cuda.Event(enable_timing=True) for _ in range(2 * launches)]
        for j in range(launches):
            evs[2 * j].record(stream)
            col.collect(K)
            evs[2 * j + 1].record(stream)
        torch.cuda.synchronize(device)
    elapsed = t1 - t0
    steps = launches * K
    # collect() = lz_rollout_policy + moments-final + rms update (tiny): per-launch time
    launch_s = sum(evs[2 * j].elapsed_time(evs[2 * j + 1]) for j in range(launches)) / launches / 1e3
    if world > 1:
        t = torch.tensor([elapsed, launch_s], device=device, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, launch_s = float(t[0]), float(t[1])
    fl = attn_policy_flops(stack * O, A) if attn else policy_flops(O, A)
    achieved = fl * n * K / launch_s / 1e12
    peak = MFMA_F32_PEAK_TFLOPS if f32 else MFMA_BF16_PEAK_TFLOPS
    # the MlpPolicy fused rollout's kernel as its launcher chooses it (lz_get_launch_shape:
    # size, LZ_POL_F32_WAVES and the variant bits included; i8x4 runs the same shape)
    f32_shape = (nat.launch_shape(env._h, nat.CALL_ROLLOUT_POLICY_F32)
                 if f32 and not attn and not per_step else None)
    mangled = {"pmsm": "7SysPMSME", "lorenz3": "5SysL3IfEE", "lorenz4": "5SysL4IfEE",
               "hr": "5SysHRIfEE"}[args.system]
    sf = scaling_fields(args, world, total, n, "no collective on step" + (
        "" if attn else "; obs_rms moments all-reduced once per rollout"))
    return {
        "metric": METRIC,
        "value": total * steps / elapsed,
        "unit": "env-steps/s",
        "n_gpus": sf["n_gpus"],
        "steps": steps,
        "warmup": warm * K,
        "ms_per_step": elapsed * 1e3 / steps,
        "higher_is_better": True,
        "scaling": sf["scaling"],
        "vs_baseline": None,
        "dtype": ("f32 MFMA extractor + int8 MFMA nets (truncated 4-digit fixed point: digit levels >= 3 "
                  "summed exactly in int32, two float32 roundings), f32 env" if i8 else
                  "f32 MFMA (f32 accumulate), f32 env" if f32 else "bf16 MFMA (fp32 accumulate), f32 env"),
        "precision_note": ("opt-in i8x4: the nets' wide layers as truncated 4-digit fixed-point products "
                           "(levels >= 3 summed exactly, recombined with two float32 roundings), float32-"
                           "level accuracy, bit-exact vs the C oracle (orc_attn_i8x4 / orc_mlp_i8x4); "
                           "frac = useful "
                           "FLOP against the f32 MFMA peak, like the fp32 line" if i8 else
                           "float32 end to end, bit-exact vs the C oracle (SB3's own precision)"
                           if f32 else "bf16 operands (opt-in, ~1e-2 off SB3's float32)"),
        "data": "synthetic: on-device Philox initial states and Gaussian action samples; "
                "SB3-initialised (orthogonal) random policy weights",
        "config": {
            "workload": ("%s with code/lorenz_filter/train.py's PPO actor-critic on "
                         "VecFrameStack(4) (attention + residual + LayerNorm extractor, pi/vf "
                         "[128,128] Tanh): %d-step fused rollout (lz_rollout_policy_attn_stack" +
                         ("_f32 + LZ_POLICY_I8X4, int8 fixed-point nets" if i8 else "_f32, float32 as SB3"
                          if f32 else ", bf16 MFMA") + ": "
                         "frame stack + extractor + nets + sample + clip + env step + bootstrap), "
                         "GAE (lz_gae); %d envs total, %d per GPU" if ln else
                         "%s with code/train.py's PPO actor-critic (AttentionFeaturesExtractor "
                         "fc1 + 4-head self-attention over 8 tokens + post_fc 64, then pi/vf "
                         "[128,128] Tanh) in the loop: %d-step fused rollout "
                         "(lz_rollout_policy_attn" + ("_f32 + LZ_POLICY_I8X4, int8 fixed-point nets" if i8 else
                                                      "_f32, float32 as SB3" if f32 else ", bf16 MFMA")
                         + ": extractor + nets + DiagGaussian sample + clip "
                         "+ env step + truncation bootstrap), GAE (lz_gae); %d envs total, %d per "
                         "GPU" if attn else
                         "%s with the SB3 A2C/PPO MlpPolicy (pi/vf [128,128] Tanh) in the loop: "
                         + ("%d-step collect in SB3's VecNormalize order (lz_rollout_policy_f32_vn: "
                            "per step one launch of VecNormalize obs with the statistics updated by "
                            "the previous step's batch + float32 policy forward + DiagGaussian sample "
                            "+ clip + env step + float64 tile moments, then the obs_rms update; "
                            "truncation bootstraps valued with their step's statistics), GAE "
                            "(lz_gae); %d envs total, %d per GPU" if per_step else
                            "%d-step fused rollout (lz_rollout_policy" + (
                                "_f32 + LZ_POLICY_I8X4, layer 2 as int8 fixed-point products" if i8 else
                                "_f32, float32 as SB3" if f32 else ", bf16 MFMA")
                            + ": policy forward + DiagGaussian "
                            "sample + clip + env step + truncation bootstrap + VecNormalize obs with "
                            "the rollout-start statistics), pooled obs_rms update, GAE (lz_gae); "
                            "%d envs total, %d per GPU"))
                        % (SYSTEM_INFO[args.system][0], K, total, n),
            "system": args.system, "mode": "policy",
            "policy": args.policy, "precision": args.precision,
            "vecnorm_update": None if attn else ("step (SB3 order)" if per_step
                                                 else "rollout (pooled, opt-in)"),
            "K": K, **sf["config"],
        },
        "roofline": {
            "bound": "mfma", "achieved": achieved, "peak": peak,
            "unit": "TFLOP/s", "frac": achieved / peak, "traffic": None,
            "kernel": (("_ZN2lz25k_rollout_policy_attn_f32INS_%sLb1ELi4ELi8ELb" + "01"[i8] + "EEEvNS_5KArgsENS_5PArgsE")
                       if ln and f32 else
                       ("_ZN2lz25k_rollout_policy_attn_f32INS_%sLb0ELi1ELi8ELb" + "01"[i8] + "EEEvNS_5KArgsENS_5PArgsE")
                       if attn and f32 else
                       "_ZN2lz16k_rollout_policyINS_%sLi4ELi32ELi4ELi4EEEvNS_5KArgsENS_5PArgsE"
                       if ln else
                       "_ZN2lz16k_rollout_policyINS_%sLi4ELi32ELi3EEEvNS_5KArgsENS_5PArgsE"
                       if attn else
                       "_ZN2lz17k_policy_step_f32INS_%sLi8EEEvNS_5KArgsENS_5PArgsENS_9PStepArgsE"
                       if per_step else
                       (("_ZN2lz16k_rollout_policyINS_%sLi" + str(f32_shape["waves"]) + "ELi32ELi"
                         + "56"[i8] + "ELi1EEEvNS_5KArgsENS_5PArgsE")
                        if f32_shape["kernel"] == "policy" else
                        ("_ZN2lz26k_rollout_policy_f32_splitINS_%sLb" + "01"[i8] + "EEEvNS_5KArgsENS_5PArgsE"))
                       if f32 else "_ZN2lz16k_rollout_policyINS_%sLi8EEEvNS_5KArgsENS_5PArgsE")
                      % mangled,
            "avg_launch_us": launch_s * 1e6, "flop_per_env_step": fl,
            "note": ("achieved = useful FLOP of the attention actor-critic as SB3 computes it "
                     "(extractor + pi + vf, %d per env-step) x envs x K / HIP-event time of one "
                     "collect() (one policy-rollout launch)" if attn else
                     "achieved = useful MLP FLOP (pi + vf, %d per env-step) x envs x K / HIP-event "
                     "time of one collect() (K + 1 policy-step launches + K statistics updates)"
                     if per_step else
                     "achieved = useful MLP FLOP (pi + vf, %d per env-step) x envs x K / HIP-event "
                     "time of one collect() (policy kernel + a 1-block moments reduction + the "
                     "obs_rms update)") % fl,
        },
    }


def describe_launches(tm, rollout):
    """What one timed window of measure_steps actually launched: hipGraph replays and
    eager launches (the driver's --steps 20 is 0 replays of a 64-step graph + 20 eager)."""
    S = tm.get("streams", 1)
    if S > 1:
        one = describe_launches(dict(tm, streams=1), rollout)
        return one.replace("per timed window: ", "per timed window, on each of %d streams "
                           "(one sub-handle of 1/%d of the shard each, concurrently): " % (S, S))
    per_win = tm["launches"] // tm["windows"]
    if rollout:
        return ("per timed window: %d eager %d-step lz_rollout launches (x%d windows)"
                % (per_win, tm["T"], tm["windows"]))
    if tm["graph"]:
        L, G, H = tm["graph_len"], tm.get("graph_rem", 0), tm.get("graph_head", 0)
        E = tm.get("head_eager", 0)
        head = ("1 hipGraph replay of %d lz_step launches (the head graph) + " % H) if H else \
            ("%d eager lz_step launches (the head) + " % E) if E else ""
        body = per_win - H - E
        rem = body % L
        extra = ("1 hipGraph replay of %d lz_step launches + " % G) if G and rem >= G else ""
        return ("per timed window: %s%d hipGraph replays of %d lz_step launches + %s%d eager "
                "lz_step launches (x%d windows)"
                % (head, body // L, L, extra, rem - (G if extra else 0), tm["windows"]))
    return "per timed window: %d eager lz_step launches (x%d windows)" % (per_win, tm["windows"])


def fp64_line(args, gl, nat, torch, dist, device, n):
    """The same step benchmark at the reference's precision: float64 LORENZ3, the kernel
    that is bit-identical to dynamic.py (tests/test_gpu_parity.py::
    test_l3_f64_golden_bitexact), 1M envs, HIP events on the launch stream."""
    env = gl.BatchedEnv("lorenz3", n, dtype="float64", seed=0, autoreset=True, device=device.index)
    tm = measure_steps(args, torch, dist, nat, env, device, 1, 0, False)
    bytes_step = env.info.bytes_per_env_step
    launch_s = tm["ev_ms"] / 1e3 / tm["launches"]
    achieved = bytes_step * n / launch_s / 1e9
    env.close()
    kname = kernel_name("lorenz3", "step", n, f64=True)
    line = {
        "metric": METRIC + " (fp64: the reference's arithmetic, bit-exact)",
        "value": n * tm["steps"] * tm["windows"] / tm["elapsed"], "unit": "env-steps/s",
        "steps": tm["steps"], "ms_per_step": tm["elapsed"] * 1e3 / (tm["steps"] * tm["windows"]),
        "dtype": "f64",
        "config": {"workload": "dynamic.py 3-state Lorenz env step (lz_step, float64, "
                               "bit-identical to the reference), %d envs on 1 GPU" % n,
                   "launch": describe_launches(tm, False)},
        "timing": tm["timing"],
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": None, "kernel": kname,
                     "avg_launch_us": launch_s * 1e6, "bytes_per_env_step": bytes_step},
    }
    traffic = load_traffic(kname, n)
    if traffic is not None:
        line["roofline"]["traffic"] = traffic["bytes_per_launch"]
        line["roofline"]["traffic_source"] = traffic["source"]
    return line


# FLOP per env-step of the RK4 mode (lz_systems.h SysL3RK4 / SysL4RK4): 4 RHS evaluations
# (L3: 9 FLOP, L4: 4 x 12 = 2 systems), 3 stage inputs, 2 stage accumulations and the final
# combination per component, then the observation RHS, the reward (and L3's clip + action)
RK4_FLOP = {"lorenz3": 4 * 9 + 3 * 6 + 2 * 6 + 3 * 4 + 9 + 6 + 6,
            "lorenz4": 2 * (4 * 12 + 3 * 8 + 2 * 8 + 4 * 3) + 2 * 12 + 8 + 8}


def rk4_line(args, gl, nat, torch, dist, device, n):
    """The headline step with the opt-in RK4 integrator (lz_config.integrator = RK4;
    north_star's "RK4 substages in registers"): the same 65 B per env-step, ~4x the FLOP
    (still < 2 FLOP/B: HBM-bound).  Bit-exact vs the oracle restatement (the reference
    has no RK4 Lorenz: parity unpinned, tests/test_gpu_rk4.py)."""
    env = gl.BatchedEnv("lorenz3", n, dtype="float32", seed=0, autoreset=True,
                        device=device.index, integrator="rk4")
    tm = measure_steps(args, torch, dist, nat, env, device, 1, 0, False)
    bytes_step = env.info.bytes_per_env_step
    launch_s = tm["ev_ms"] / 1e3 / tm["launches"]
    achieved = bytes_step * n / launch_s / 1e9
    kname = kernel_name("lorenz3", "step", n, integrator="rk4")
    env.close()
    line = {
        "metric": METRIC + " (integrator=rk4, opt-in mode)",
        "value": n * tm["steps"] * tm["windows"] / tm["elapsed"], "unit": "env-steps/s",
        "steps": tm["steps"], "ms_per_step": tm["elapsed"] * 1e3 / (tm["steps"] * tm["windows"]),
        "dtype": "f32",
        "config": {"workload": "dynamic.py 3-state Lorenz env step with the RK4 integrator "
                               "(lz_step, float32, 4 RHS stages in registers), %d envs on 1 GPU" % n,
                   "integrator": "rk4", "launch": describe_launches(tm, False)},
        "timing": tm["timing"],
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": None, "kernel": kname,
                     "avg_launch_us": launch_s * 1e6, "bytes_per_env_step": bytes_step,
                     "flop_per_env_step": RK4_FLOP["lorenz3"]},
    }
    traffic = load_traffic(kname, n)
    if traffic is not None:
        line["roofline"]["traffic"] = traffic["bytes_per_launch"]
        line["roofline"]["traffic_source"] = traffic["source"]
    return line


def default_streams(system, mode, n):
    """--streams 0 (auto): how many concurrent sub-handle chains a rank's per-step loop
    uses for an n-env shard (see make_subs)."""
    return 1


def make_subs(args, gl, n, start, local, kw):
    """--streams S > 1 (step mode): the rank's shard as S BatchedEnv sub-handles of
    consecutive global ids (gym_lorenz.parallel.sub_shards), else None."""
    from gym_lorenz.parallel import sub_shards

    S = args.streams or default_streams(args.system, args.mode, n)
    S = max(1, min(int(S), 4, n))
    if S == 1:
        return None
    return [gl.BatchedEnv(args.system, c, dtype=args.dtype, seed=0, global_env_offset=o,
                          autoreset=True, device=local, max_episode_steps=args.max_episode_steps,
                          variant=args.variant, **kw) for o, c in sub_shards(n, start, S)]


def scaling_line(args, gl, nat, torch, dist, device, world, rank):
    """N > 1: the headline step in the other scaling mode (the weak 1,048,576-per-GPU run
    next to the strong 1M-total headline, or the reverse with --scaling weak)."""
    from gym_lorenz.parallel import shard_bounds

    if args.scaling == "strong":
        mode, n = "weak", args.envs
        total, start = n * world, rank * n
    else:
        mode, total = "strong", args.envs
        start, n = shard_bounds(total, rank, world)
    env = gl.BatchedEnv("lorenz3", n, dtype="float32", seed=0, global_env_offset=start,
                        autoreset=True, device=device.index)
    subs = make_subs(args, gl, n, start, device.index, {})
    tm = measure_steps(args, torch, dist, nat, env, device, world, rank, False, subs=subs)
    launch_s = tm["ev_ms"] / 1e3 / tm["launches"]
    achieved = env.info.bytes_per_env_step * n / launch_s / 1e9
    sub_n = subs[0].num_envs if subs else n
    for e in [env] + (subs or []):
        e.close()
    return {
        "metric": METRIC + " (%s scaling)" % mode,
        "value": total * tm["steps"] * tm["windows"] / tm["elapsed"], "unit": "env-steps/s",
        "n_gpus": world, "scaling": mode, "steps": tm["steps"],
        "ms_per_step": tm["elapsed"] * 1e3 / (tm["steps"] * tm["windows"]), "dtype": "f32",
        "config": {"workload": "dynamic.py env step (lz_step, fp32), %d envs total, %d per GPU"
                               % (total, n), "envs_total": total, "envs_per_gpu": n,
                   "launch": describe_launches(tm, False)},
        "timing": tm["timing"],
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "avg_launch_us": launch_s * 1e6,
                     "kernel": kernel_name("lorenz3", "step", sub_n)},
    }


XGMI_LINKS = 7  # point-to-point xGMI links per MI355X (MI355X_MICROARCH.md)


def gather_accounting(world, nbytes, steps, seconds):
    """Bytes and rates of `steps` gathers of `nbytes` per rank into rank 0.  Rank 0's own
    shard never leaves its HBM, so (world - 1) x nbytes cross xGMI per gather; each peer
    sends its shard over its own point-to-point link into rank 0 (a full mesh of 8), so
    the per-link figure divides by the min(world - 1, 7) links rank 0 receives on."""
    xgmi = (world - 1) * nbytes
    links = max(1, min(world - 1, XGMI_LINKS))
    return {"us_per_step": seconds * 1e6 / steps, "bytes_per_step_xgmi": xgmi,
            "bytes_per_step_rank0_local": nbytes,
            "GB_per_s": xgmi * steps / seconds / 1e9,
            "links": links, "GB_per_s_per_link": xgmi * steps / seconds / 1e9 / links}


def check_devices(gpus, backend, device_count):
    """RCCL runs one rank per GPU: more ranks than visible GPUs would share cards (rank r
    takes cuda:(r mod count)) and report a 'strong' number that is not one -- refuse."""
    if backend == "nccl" and gpus > 1 and gpus > device_count:
        raise SystemExit("bench.py: --gpus %d but only %d GPU(s) visible; the nccl (RCCL) backend "
                         "needs one GPU per rank (LZ_BENCH_BACKEND=gloo rehearses ranks sharing a "
                         "GPU)" % (gpus, device_count))


def gather_line(args, gl, nat, torch, dist, device, world, rank, total, n, start, backend,
                steps=200):
    """N > 1: north_star's optional learner gather -- every step, lz_step on each rank's
    shard, then ONE dist.gather of the shard's packed obs | reward | done bytes into rank
    0 (RCCL over xGMI with the default backend: send / recv pairs into rank 0's links).
    Timed as `steps` whole steps (barrier + synchronize on both sides, MAX over ranks);
    the gather alone is timed the same way for its bytes/s."""
    from gym_lorenz.parallel import shard_counts

    counts = shard_counts(total, world)
    if len(set(counts)) != 1:
        return {"metric": "step + gather to rank 0", "skipped": "unequal shards %s" % counts}
    env = gl.BatchedEnv("lorenz3", n, dtype="float32", seed=0, global_env_offset=start,
                        autoreset=True, device=device.index, compact=False)
    env.reset()
    a = torch.rand((n, 3), device=device) * 2 - 1
    host = backend != "nccl"  # gloo rehearsal: the collective runs on host copies
    src = env.packed if not host else torch.empty(env.packed.shape, dtype=torch.uint8)
    bufs = [torch.empty_like(src) for _ in range(world)] if rank == 0 else None
    nbytes = env.packed.numel()

    def gather():
        if host:
            src.copy_(env.packed)
        dist.gather(src, gather_list=bufs, dst=0)

    def timed(fn, k):
        dist.barrier()
        torch.cuda.synchronize(device)
        t0 = time.perf_counter()
        for _ in range(k):
            fn()
        torch.cuda.synchronize(device)
        t1 = time.perf_counter()
        dist.barrier()
        t = torch.tensor([t1 - t0], dtype=torch.float64, device=device if not host else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    def both():
        env.step(a, want_n_done=False)
        gather()

    timed(both, 10)
    t_both = timed(both, steps)
    t_gather = timed(gather, steps)
    env.close()
    return {
        "metric": "env-steps/s with the per-step gather of obs | reward | done to rank 0",
        "value": total * steps / t_both, "unit": "env-steps/s", "n_gpus": world, "steps": steps,
        "ms_per_step": t_both * 1e3 / steps, "dtype": "f32",
        "gather": dict(gather_accounting(world, nbytes, steps, t_gather), **{
                   "backend": "RCCL (xGMI)" if not host else "%s on host copies (rehearsal)" % backend,
                   "collective": "one torch.distributed.gather of each rank's packed obs|reward|done "
                                 "(%d B) into rank 0; GB_per_s counts the (world - 1) shards that "
                                 "cross xGMI" % nbytes}),
        "config": {"workload": "dynamic.py env step (lz_step, fp32) + gather to rank 0, %d envs "
                               "total, %d per GPU" % (total, n),
                   "envs_total": total, "envs_per_gpu": n},
    }


class _Lane:
    """One handle of a rank's shard with its own on-device ring, HIP stream and captured
    hipGraphs (measure_steps drives 1 lane, or S with --streams S)."""

    def __init__(self, args, torch, nat, env, device, rank, rollout, lane):
        A, O = env.action_dim, env.obs_dim
        arange = SYSTEM_INFO[args.system][2]
        self.R = R = args.ring if not rollout else 1
        self.T = T = args.K if rollout else 1
        tdt = env.tdtype
        g = torch.Generator(device=device).manual_seed(1000 + rank + 7919 * lane)
        n = env.num_envs
        self.buf = (
            (torch.rand((R, T, n, A), generator=g, device=device) * 2 - 1) * arange,
            torch.empty((R, T, n, O), device=device, dtype=tdt),
            torch.empty((R, T, n), device=device, dtype=tdt),
            torch.empty((R, T, n), dtype=torch.uint8, device=device))
        acts, obs, rew, done = self.buf
        env.reset()
        self.env, self.h, self.rollout, self.counter = env, env._h, rollout, 0
        # every ring slot through the checked caller-buffer entry once (dtype / device /
        # contiguity / element count vs lz_info), then its pointer tuple is launched as is
        if rollout:
            self.slots = [env.rollout_args(T, acts[r], obs[r], rew[r], done[r]) for r in range(R)]
        else:
            self.slots = [env.step_args(acts[r, 0], obs[r, 0], rew[r, 0], done[r, 0],
                                        env.done_idx, env.term_obs) for r in range(R)]
        self.fn = nat.lib.lz_rollout if rollout else nat.lib.lz_step
        self.nat = nat
        self.stream = torch.cuda.Stream(device)
        nat.check(nat.lib.lz_set_stream(self.h, ctypes.c_void_p(self.stream.cuda_stream)))
        self.graph = self.graph_rem = None
        self.flush = None

    def one(self):
        sl = self.slots[self.counter % self.R]
        self.counter += 1
        st = self.fn(self.h, *sl)
        if st:
            self.nat.check(st)
        if self.flush is not None:
            self.flush()


def measure_steps(args, torch, dist, nat, env, device, world, rank, rollout, min_window_s=0.2,
                  subs=None):
    """Time EXACTLY K env steps (K = --steps; rollout mode: --steps rounded down to whole
    --K launches), each timed window bracketed by a barrier + torch.cuda.synchronize()
    on both sides.  When one window is shorter than `min_window_s` (e.g. the driver's
    --steps 20 is 0.24 ms at 1M envs), back-to-back windows of the same K steps are timed
    until their sum reaches it; value = windows x K x envs / summed window time (the
    MAX over ranks).  Step mode replays a hipGraph of L lz_step launches and launches
    the K mod L remainder eagerly; an odd remainder is followed by one untimed step so
    the captured graph's ping-pong parity stays valid.

    subs (--streams S): the shard as S sub-handles of consecutive global_env_offset
    (bit-identical to one handle: tests/test_gpu_streams.py), each with its own ring,
    stream and graphs; every window runs all S chains of K steps concurrently, bracketed
    by one device synchronize.  The HIP-event time is the span from the first stream's
    start event to the last stream's end event."""
    lanes = [_Lane(args, torch, nat, e, device, rank, rollout, j)
             for j, e in enumerate(subs or [env])]
    R, T = lanes[0].R, lanes[0].T
    flush = getattr(args, "ic_flush_mib", 0)
    if flush:  # A/B only: evict the Infinity Cache between steps (see --ic-flush-mib)
        fsrc = torch.ones((flush << 18,), device=device)
        fdst = torch.empty_like(fsrc) if args.ic_flush_kind == "copy" else None
        fsum = torch.empty((), device=device)
        if args.ic_flush_kind == "read":  # the same bytes read as the copy moves in total
            fsrc = torch.ones((flush << 19,), device=device)
        lanes[0].flush = ((lambda: fdst.copy_(fsrc)) if args.ic_flush_kind == "copy"
                          else (lambda: torch.sum(fsrc, dim=0, out=fsum)))

    L = max(2, args.graph_len - args.graph_len % 2)  # even: keeps the ping-pong parity
    if R > 1 and L % R and R % L:
        L = R
    launches = args.steps if not rollout else max(1, args.steps // T)
    warm = args.warmup if not rollout else 2
    if rollout:
        L = 1
    use_graph = args.launch == "graph" and not rollout
    # --head-graph H: the window's first H launches as a short graph of their own (H even:
    # the captured ping-pong parity)
    H = getattr(args, "head_graph", 0)
    H = H - H % 2 if use_graph and 0 < H <= launches else 0
    E = getattr(args, "head_eager", 0)
    E = E - E % 2 if use_graph and not H and 0 < E <= launches else 0
    H = H or E  # (the remainder graph covers what follows the head either way)
    # the window's (K - H) mod L remainder as a graph too (its even part: the captured
    # ping-pong parity), so that a short window (the driver's --steps 20) is not
    # paced by one Python launch per step
    rem_n = ((launches - H) % L) - ((launches - H) % L) % 2 if use_graph else 0
    for ln in lanes:
        with torch.cuda.stream(ln.stream):
            for _ in range(max(warm, 2)):
                ln.one()
            if use_graph:
                ln.graph = torch.cuda.CUDAGraph()
                with torch.cuda.graph(ln.graph, stream=ln.stream):
                    for _ in range(L):
                        ln.one()
                if rem_n:
                    ln.graph_rem = torch.cuda.CUDAGraph()
                    with torch.cuda.graph(ln.graph_rem, stream=ln.stream):
                        for _ in range(rem_n):
                            ln.one()
                if H and not E:
                    ln.graph_head = torch.cuda.CUDAGraph()
                    with torch.cuda.graph(ln.graph_head, stream=ln.stream):
                        for _ in range(H):
                            ln.one()
    torch.cuda.synchronize(device)

    def run(nlaunch):  # exactly nlaunch launches on every lane, the lanes interleaved
        if not use_graph:
            for _ in range(nlaunch):
                for ln in lanes:
                    with torch.cuda.stream(ln.stream):
                        ln.one()
            return
        if E and nlaunch >= E:
            for _ in range(E):
                for ln in lanes:
                    with torch.cuda.stream(ln.stream):
                        ln.one()
            nlaunch -= E
        elif H and nlaunch >= H:
            for ln in lanes:
                with torch.cuda.stream(ln.stream):
                    ln.graph_head.replay()
            nlaunch -= H
        for _ in range(nlaunch // L):
            for ln in lanes:
                with torch.cuda.stream(ln.stream):
                    ln.graph.replay()
        r = nlaunch % L
        if rem_n and r >= rem_n:
            for ln in lanes:
                with torch.cuda.stream(ln.stream):
                    ln.graph_rem.replay()
            r -= rem_n
        for _ in range(r):
            for ln in lanes:
                with torch.cuda.stream(ln.stream):
                    ln.one()

    def fix_parity(nlaunch):  # untimed: an odd eager remainder flipped the parity
        if use_graph and nlaunch % 2:  # (H, L and the remainder graph are all even)
            for ln in lanes:
                with torch.cuda.stream(ln.stream):
                    ln.one()

    if use_graph:
        run(max(warm, L))  # warm the graph path too
        fix_parity(max(warm, L))
    torch.cuda.synchronize(device)

    def window():
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize(device)
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
              for _ in lanes]
        t0 = time.perf_counter()
        for ln, (e0, _) in zip(lanes, ev):
            e0.record(ln.stream)
        run(launches)
        for ln, (_, e1) in zip(lanes, ev):
            e1.record(ln.stream)
        torch.cuda.synchronize(device)
        # stop before the closing barrier: a collective's latency is not part of the K
        # steps (the path has none); the job's time is the MAX over ranks below
        t1 = time.perf_counter()
        if world > 1:
            dist.barrier()
        fix_parity(launches)
        base = ev[0][0]
        span = (max(base.elapsed_time(e1) for _, e1 in ev)
                - min(0.0, min(base.elapsed_time(e0) for e0, _ in ev)))
        return t1 - t0, span

    first = window()
    # windows until min_window_s are timed in total: batches sized from the windows
    # so far (the first window after warm-up runs slower than the rest), every rank
    # running the same count (MAX over ranks)
    wins, per = [], first[0]
    while True:
        left = min_window_s - sum(w[0] for w in wins)
        need = max(1, min(math.ceil(left / max(per, 1e-9)), 5000 - len(wins)))
        if world > 1:
            t = torch.tensor([need if left > 0 else 0], device=device, dtype=torch.int64)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            need = int(t.item())
        elif left <= 0:
            need = 0
        if need == 0 or len(wins) >= 5000:
            break
        wins += [window() for _ in range(need)]
        per = sum(w[0] for w in wins) / len(wins)
    need = len(wins)
    elapsed = sum(w[0] for w in wins)
    ev_ms = sum(w[1] for w in wins)
    if world > 1:
        t = torch.tensor([elapsed, ev_ms], device=device, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, ev_ms = float(t[0]), float(t[1])
    wms = sorted(w[0] * 1e3 for w in wins)
    K = launches * T
    return {
        "steps": K, "T": T, "ring": R, "graph_len": L, "graph": use_graph,
        "graph_rem": rem_n, "graph_head": 0 if E else H, "head_eager": E, "streams": len(lanes),
        "warmup": warm, "launches": launches * need, "windows": need,
        "elapsed": elapsed, "ev_ms": ev_ms,
        "timing": {
            "requested_steps": args.steps, "steps_per_window": K, "windows": need,
            "timed_steps_total": K * need, "timed_seconds": elapsed,
            "window_ms_min": wms[0], "window_ms_median": wms[len(wms) // 2],
            "method": "each window = exactly `steps` env steps of every env, bracketed by "
                      "barrier + torch.cuda.synchronize() on both sides (the clock stops "
                      "after the closing synchronize, before the closing barrier); windows repeated "
                      "until >= %.0f ms are timed; value = windows x steps x envs / summed "
                      "window time (MAX over ranks)" % (min_window_s * 1e3),
        },
    }


def free_port():
    import socket

    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def rank_envs(n, port, base=None):
    """The torch.distributed.run environment of each of n rank processes on one node."""
    base = dict(os.environ if base is None else base)
    out = []
    for r in range(n):
        e = dict(base)
        e.update({"RANK": str(r), "LOCAL_RANK": str(r), "WORLD_SIZE": str(n),
                  "LOCAL_WORLD_SIZE": str(n), "GROUP_RANK": "0", "MASTER_ADDR": "127.0.0.1",
                  "MASTER_PORT": str(port), "TORCHELASTIC_RUN_ID": "bench-self-spawn"})
        out.append(e)
    return out


def spawn_ranks(n, argv):
    """`--gpus N` without a launcher: run this script as N child processes (rank r on
    cuda:r), the same arguments, before this process touches torch or the GPU.  Children
    inherit stdout / stderr (rank 0 prints the JSON line); if one fails the others are
    terminated (their exact PIDs).  Returns the exit status."""
    import subprocess

    envs = rank_envs(n, free_port())
    procs = [subprocess.Popen([sys.executable, os.path.abspath(__file__)] + list(argv), env=e)
             for e in envs]
    status = 0
    try:
        while True:
            codes = [p.poll() for p in procs]
            bad = [c for c in codes if c not in (None, 0)]
            if bad:
                status = bad[0]
                break
            if all(c == 0 for c in codes):
                break
            time.sleep(0.05)
    finally:
        for p in procs:
            if p.poll() is None:
                p.terminate()
        for p in procs:
            try:
                p.wait(timeout=30)
            except Exception:  # noqa: BLE001
                p.kill()
    return status


def shard_plan(args, world, rank):
    """(envs_total, first global env id, envs on this rank): --scaling strong splits the
    --envs total over the ranks (gym_lorenz.parallel.shard_bounds: contiguous ids, the first
    N mod W ranks one more), weak gives every rank --envs."""
    from gym_lorenz.parallel import shard_bounds

    if args.scaling == "strong":
        start, n = shard_bounds(args.envs, rank, world)
        return args.envs, start, n
    return args.envs * world, rank * args.envs, args.envs


def scaling_fields(args, world, total, n, collective):
    """The line's scaling statement (every mode): n_gpus, scaling, and in config the job's
    and one rank's env counts and what crosses ranks (`collective`)."""
    return {"n_gpus": world, "scaling": args.scaling,
            "config": {"envs_total": total, "envs_per_gpu": n,
                       "parallelism": "env shard x%d (contiguous global ids; %s)" % (world, collective)}}


def main():
    args = parse()
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(spawn_ranks(args.gpus, sys.argv[1:]))
    if args.probe_ranks:  # launcher test: this rank's environment, nothing else
        if os.environ.get("LZ_BENCH_PROBE_FAIL_RANK") == os.environ.get("RANK"):
            sys.exit(3)
        if os.environ.get("LZ_BENCH_PROBE_FAIL_RANK") is not None:
            time.sleep(60)  # a healthy rank still running when another fails
        print(json.dumps({k: os.environ.get(k) for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE",
                                                          "MASTER_ADDR", "MASTER_PORT")}), flush=True)
        return
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit("--gpus %d but WORLD_SIZE=%d" % (args.gpus, world))
    headline = args.system == "lorenz3" and args.mode == "step"
    cpu = None
    if rank == 0 and world == 1 and headline and not args.no_cpu_baseline:
        cpu = cpu_baseline(args.cpu_seconds)  # first: its worker processes start before
        #                                       anything initialises the GPU
    # LZ_BENCH_BACKEND=gloo + ranks sharing a GPU: rehearsal of the multi-rank path on a
    # 1-GPU box (the driver's 8-GPU runs use the default: RCCL, one GPU per rank)
    backend = os.environ.get("LZ_BENCH_BACKEND", "nccl")
    check_devices(world, backend, torch.cuda.device_count())
    local = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    device = torch.device("cuda", local)
    if world > 1:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=device)
        else:
            dist.init_process_group(backend)

    import gym_lorenz as gl
    from gym_lorenz import _native as nat

    total, start, n = shard_plan(args, world, rank)
    kw = {"add_noise": True, "alpha": 0.5} if args.system == "pmsm" else {}
    if args.integrator == "rk4" and args.system in ("lorenz3", "lorenz4"):
        kw["integrator"] = "rk4"
    if args.add_noise is not None:
        kw["add_noise"] = bool(args.add_noise)
    env = gl.BatchedEnv(args.system, n, dtype=args.dtype, seed=0, global_env_offset=start,
                        autoreset=True, device=local, max_episode_steps=args.max_episode_steps,
                        variant=args.variant, **kw)
    if args.mode == "policy":
        out = bench_policy(args, gl, nat, torch, env, device, world, rank, total, n)
        env.close()
        if world > 1:
            dist.barrier()
            dist.destroy_process_group()
        if rank == 0:
            print(json.dumps(out), flush=True)
        return
    if args.mode == "vecnorm":
        out = bench_vecnorm(args, gl, nat, torch, env, device, world, total, n)
        env.close()
        if world > 1:
            dist.barrier()
            dist.destroy_process_group()
        if rank == 0:
            print(json.dumps(out), flush=True)
        return
    rollout = args.mode == "rollout"
    subs = make_subs(args, gl, n, start, local, kw) if not rollout else None
    tm = measure_steps(args, torch, dist, nat, env, device, world, rank, rollout, subs=subs)
    sub_n = subs[0].num_envs if subs else n
    for e in subs or []:
        e.close()
    K, L, R, T = tm["steps"], tm["graph_len"], tm["ring"], tm["T"]
    elapsed, ev_ms, nl = tm["elapsed"], tm["ev_ms"], tm["launches"]
    warm = tm["warmup"]
    graph = tm["graph"]
    arange = SYSTEM_INFO[args.system][2]

    info = env.info
    if rollout:  # state planes once per launch, per-step I/O every step
        bytes_step = info.bytes_per_env_step - info.state_io_bytes + info.state_io_bytes / T
    else:
        bytes_step = info.bytes_per_env_step  # LORENZ3 f32: 65 B (24 state + 12 act + 29 out)
    launch_s = ev_ms / 1e3 / nl
    achieved = bytes_step * n * T / launch_s / 1e9
    ref_env = SYSTEM_INFO[args.system][0]
    launch_desc = describe_launches(tm, rollout)
    integ = " [integrator=rk4: the opt-in RK4 mode, not the reference's Euler]" if "integrator" in kw else ""
    if rollout:
        workload = ("%s%s: %d-step fused on-device rollout (lz_rollout, fp32, state in VGPRs), "
                    "%d envs total, %d per GPU, time-major [K,N,.] rollout buffers"
                    % (ref_env, integ, T, total, n))
    else:
        workload = ("%s%s step (lz_step, fp32), %d envs total, %d per GPU, actions/obs/reward/"
                    "done in a %d-slot on-device rollout ring" % (ref_env, integ, total, n, R))
    sf = scaling_fields(args, world, total, n, "no collective on step")
    out = {
        "metric": METRIC,
        "value": total * K * tm["windows"] / elapsed,
        "unit": "env-steps/s",
        "n_gpus": sf["n_gpus"],
        "steps": K,
        "warmup": warm,
        "ms_per_step": elapsed * 1e3 / (K * tm["windows"]),
        "higher_is_better": True,
        "scaling": sf["scaling"],
        "vs_baseline": None,
        "dtype": "f64" if args.dtype == "float64" else "f32",
        "data": "synthetic: initial states from on-device Philox keyed by global env id "
                "(reference distributions); actions ~ U(-%g,%g) f32 pre-generated on device"
                % (arange, arange),
        "config": dict({"workload": workload, "system": args.system, "mode": args.mode,
                        "launch": launch_desc}, **sf["config"]),
        "timing": tm["timing"],
        "roofline": {
            "bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": achieved / HBM_PEAK_GBS, "traffic": None,
            "kernel": kernel_name(args.system, args.mode, sub_n, f64=args.dtype == "float64",
                                  no_done=args.max_episode_steps == 0,
                                  num_cus=torch.cuda.get_device_properties(device).multi_processor_count,
                                  variant=args.variant, integrator=kw.get("integrator", "euler"),
                                  noise=bool(env.config.flags & nat.FLAG_ADD_NOISE)),
            "avg_launch_us": launch_s * 1e6,
            "bytes_per_env_step": bytes_step,
            "note": "achieved = algorithmic bytes per launch (bytes_per_env_step x envs_per_gpu"
                    " x steps per launch) / HIP-event average launch time on the launch stream",
        },
    }
    traffic = load_traffic(out["roofline"]["kernel"], n) if not subs else None
    if subs:
        out["config"]["streams"] = len(subs)
        out["roofline"]["note"] += ("; --streams %d: the launch time is the span of one step of "
                                    "all %d concurrent sub-handle chains (%d envs each)"
                                    % (len(subs), len(subs), sub_n))
    if traffic is not None:
        out["roofline"]["traffic"] = traffic["bytes_per_launch"]
        out["roofline"]["traffic_source"] = traffic["source"]
        out["roofline"]["traffic_kernel_sha256"] = traffic["kernel_code_sha256"]
    else:
        out["roofline"]["traffic_note"] = ("null: no committed PMC summary for this kernel "
                                           "build (code hash) and shard size")
    if "integrator" in kw:
        out["config"]["integrator"] = "rk4"
        out["roofline"]["flop_per_env_step"] = RK4_FLOP[args.system]
    headline = args.system == "lorenz3" and not rollout and "integrator" not in kw
    env.close()
    if rank == 0 and world == 1 and headline and args.dtype == "float32" and not args.no_extras:
        cs = cold_state_probe(gl, nat, torch, device, n)
        cs["frac_cold_scaled"] = out["roofline"]["frac"] * cs["us_per_launch_warm"] / cs["us_per_launch_cold"]
        out["roofline"]["cold_state"] = cs
        out["roofline"]["memory_level_note"] = (
            "the state the step reads was written by the previous step ~68 MB of traffic earlier, "
            "so in this loop it is served from the 256 MiB Infinity Cache, not DRAM "
            "(profiles/r05/ic/): with the state evicted before every step the same launch takes "
            "cold_over_warm x as long; frac_cold_scaled = frac x warm / cold is the fraction of "
            "8 TB/s the kernel reaches when every byte comes from DRAM")
    extras = []
    if rank == 0 and world == 1 and headline and not args.no_drift:
        out["fp32_drift"] = fp32_drift(gl, torch, device)
    if world == 1 and headline and not args.no_extras:
        extras.append(fp64_line(args, gl, nat, torch, dist, device, n))
        extras.append(rk4_line(args, gl, nat, torch, dist, device, n))
    if world > 1 and headline and not args.no_extras:
        # the other scaling mode at the same N, then the learner gather (every rank runs
        # these: they time collectively)
        extras.append(scaling_line(args, gl, nat, torch, dist, device, world, rank))
        if not args.no_gather:
            extras.append(gather_line(args, gl, nat, torch, dist, device, world, rank, total, n,
                                      start, backend))
    if extras and rank == 0:
        out["extra_lines"] = extras
    if cpu is not None:
        out["cpu_baseline"] = cpu
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    if rank == 0:
        print(json.dumps(out), flush=True)


def cold_state_probe(gl, nat, torch, device, n, reps=96, flush_mib=384):
    """Which memory level the headline's state reads come from.  The
    12 MB of LORENZ3 state is written by step k and read by step k + 1 with ~68 MB of other
    traffic between, so the Infinity Cache (256 MiB, MI355X_MICROARCH.md "Infinity Cache")
    can serve those reads, and FETCH_SIZE counts such hits as traffic.  Here the same
    handle / ring / kernel is timed per launch (HIP events around each lz_step on its
    stream, a spin kernel queued first so the GPU never waits for Python) in two loops:
    `warm` = back-to-back steps as in the bench; `cold` = a read of `flush_mib` MiB (a sum)
    before every step, so nothing of the state survives in the Infinity Cache.  Returns
    the two per-launch times and the HBM fraction of the cold one."""
    import ctypes

    env = gl.BatchedEnv("lorenz3", n, dtype="float32", seed=0, autoreset=True, device=device.index)
    env.reset()
    R, A, O = 16, env.action_dim, env.obs_dim
    acts = torch.rand((R, n, A), device=device) * 2 - 1
    obs = torch.empty((R, n, O), device=device)
    rew = torch.empty((R, n), device=device)
    done = torch.empty((R, n), dtype=torch.uint8, device=device)
    big = torch.ones((flush_mib << 18,), device=device)
    out = torch.empty((), device=device)
    slots = [env.step_args(acts[r], obs[r], rew[r], done[r], env.done_idx, env.term_obs)
             for r in range(R)]  # the checked caller-buffer entry (core.step_io_args)
    stream = torch.cuda.Stream(device)
    nat.check(nat.lib.lz_set_stream(env._h, ctypes.c_void_p(stream.cuda_stream)))
    k = [0]

    def step():
        sl = slots[k[0] % R]
        k[0] += 1
        nat.check(nat.lib.lz_step(env._h, *sl))

    res = {}
    with torch.cuda.stream(stream):
        for _ in range(8):
            step()
        torch.cuda.synchronize(device)
        for mode in ("warm", "cold", "warm2", "cold2"):
            evs = []
            torch.cuda._sleep(int(5e7))  # the queue fills while the GPU spins
            for _ in range(reps):
                if mode.startswith("cold"):
                    torch.sum(big, dim=0, out=out)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(stream)
                step()
                e1.record(stream)
                evs.append((e0, e1))
            torch.cuda.synchronize(device)
            ts = sorted(e0.elapsed_time(e1) * 1e3 for e0, e1 in evs[4:])
            res.setdefault(mode.rstrip("2"), []).append(ts[len(ts) // 2])
    env.close()
    del big
    torch.cuda.empty_cache()
    warm, cold = min(res["warm"]), min(res["cold"])
    alg = env.bytes_per_env_step * n
    return {"us_per_launch_warm": warm, "us_per_launch_cold": cold, "cold_over_warm": cold / warm,
            "frac_cold": alg / (cold * 1e-6) / 1e9 / HBM_PEAK_GBS,
            "method": "per-launch HIP events (median of %d, best of 2 loops), the same 1M LORENZ3 "
                      "handle and 16-slot ring; cold = a %d MiB read (torch.sum) before every step "
                      "evicts the state from the 256 MiB Infinity Cache" % (reps - 4, flush_mib)}


def load_traffic(kernel, n):
    """HBM bytes per launch from the committed rocprofv3 PMC summary of this workload
    (profiles/<round>/*pmc_summary.json, written by tools/pmc_summary.py from separate
    rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes, gfx950-calibrated), if one matches
    this kernel and shard size AND was measured on the same build of the kernel: the
    summary's kernel_code_sha256 (tools/kernel_hash.py: the kernel's gfx950 machine code
    + descriptor) must equal the running library's -- a changed kernel reports null
    until it is re-measured."""
    import glob

    sys.path.insert(0, os.path.join(ROOT, "tools"))
    from kernel_hash import kernel_code_sha256

    live = kernel_code_sha256(kernel)
    if live is None:
        return None
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "**", "*pmc_summary.json"),
                              recursive=True), reverse=True):  # newest round first
        try:
            d = json.load(open(f))
        except Exception:  # noqa: BLE001
            continue
        if (d.get("kernel") == kernel and d.get("envs_per_gpu") == n
                and d.get("kernel_code_sha256") == live):
            return {"bytes_per_launch": d["hbm_bytes_per_launch"],
                    "source": os.path.relpath(f, ROOT), "kernel_code_sha256": live}
    return None


if __name__ == "__main__":
    main()
