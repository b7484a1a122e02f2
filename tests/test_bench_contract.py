"""bench.py's output contract (the driver parses its one JSON line): the CPU baseline
leg on the host (no GPU), and on the GPU the whole line at the driver's own short
setting (--steps 20): the BASELINE metric, whole-job value, exactly K timed steps per
window, the roofline object with frac = achieved / peak, and a launch description that
says what ran."""
import json
import os
import subprocess
import sys
import time

import pytest

from conftest import ROOT


def test_cpu_baseline_leg():
    """The bounded CPU sample: the reference-cost loop on every host core and on one,
    plus the C port; kind 'port', cores stated."""
    sys.path.insert(0, ROOT)
    import bench

    cb = bench.cpu_baseline(2.0)
    assert cb["unit"] == "env-steps/s" and cb["kind"] == "port"
    assert cb["value"] > 0 and cb["cores"] >= 1 and "ref_loop.py" in cb["sample"]
    assert cb["one_core"]["cores"] == 1 and cb["one_core"]["value"] > 0
    assert cb["c_port"]["value"] > cb["value"]  # the C port is far cheaper per step


def test_launcher_rank_environment():
    """`python bench.py --gpus N` outside torch.distributed.run spawns N rank processes
    itself: each gets RANK = LOCAL_RANK = r, WORLD_SIZE = N and a 127.0.0.1 rendezvous;
    the spawning process touches neither torch nor the GPU (--probe-ranks makes each rank
    print its environment and exit; no GPU needed)."""
    sys.path.insert(0, ROOT)
    import bench

    envs = bench.rank_envs(3, 29500, base={"PATH": "/bin", "HSA_ENABLE_IPC_MODE_LEGACY": "0"})
    assert [e["RANK"] for e in envs] == ["0", "1", "2"]
    assert all(e["LOCAL_RANK"] == e["RANK"] and e["WORLD_SIZE"] == "3" for e in envs)
    assert all(e["MASTER_ADDR"] == "127.0.0.1" and e["MASTER_PORT"] == "29500" for e in envs)
    assert all(e["HSA_ENABLE_IPC_MODE_LEGACY"] == "0" and e["PATH"] == "/bin" for e in envs)
    a = bench.parse(["--gpus", "4"])
    assert a.scaling == "strong" and a.envs == 1 << 20 and a.integrator == "euler"
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, "-c",
                        "import sys, runpy; sys.argv = ['bench.py', '--gpus', '2', '--probe-ranks'];"
                        "runpy.run_path('bench.py', run_name='__main__');"
                        "print('torch imported:', 'torch' in sys.modules)"],
                       capture_output=True, text=True, timeout=120, cwd=ROOT, env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [json.loads(ln) for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert sorted(int(d["RANK"]) for d in lines) == [0, 1]
    assert all(d["WORLD_SIZE"] == "2" and d["MASTER_ADDR"] == "127.0.0.1" for d in lines)
    assert len({d["MASTER_PORT"] for d in lines}) == 1
    # sys.exit(status) ends the parent before the print: the parent never imported torch
    assert "torch imported" not in r.stdout


def test_launcher_propagates_a_failed_rank():
    """A rank that fails (rank 1 exits 3 while rank 0 is still running) makes the launcher
    terminate the other rank and exit with the failure's status, promptly."""
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK")}
    env["LZ_BENCH_PROBE_FAIL_RANK"] = "1"
    t0 = time.time()
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--probe-ranks"],
                       capture_output=True, text=True, timeout=120, cwd=ROOT, env=env)
    assert r.returncode == 3, (r.returncode, r.stderr[-2000:])
    assert time.time() - t0 < 40  # rank 0 (sleeping 60 s) was terminated, not waited for


def test_gather_accounting_counts_xgmi_bytes_only():
    """rank 0's own shard never crosses xGMI -- the gather line
    counts (world - 1) shards, and per link over the min(world - 1, 7) links into rank 0."""
    sys.path.insert(0, ROOT)
    import bench

    nb, steps, secs = 1_000_000, 100, 0.5
    g = bench.gather_accounting(8, nb, steps, secs)
    assert g["bytes_per_step_xgmi"] == 7 * nb and g["bytes_per_step_rank0_local"] == nb
    assert g["links"] == 7
    assert abs(g["GB_per_s"] - 7 * nb * steps / secs / 1e9) < 1e-12
    assert abs(g["GB_per_s_per_link"] - nb * steps / secs / 1e9) < 1e-12
    assert abs(g["us_per_step"] - secs * 1e6 / steps) < 1e-9
    g2 = bench.gather_accounting(2, nb, steps, secs)
    assert g2["bytes_per_step_xgmi"] == nb and g2["links"] == 1
    assert g2["GB_per_s_per_link"] == g2["GB_per_s"]
    g4 = bench.gather_accounting(4, nb, steps, secs)
    assert g4["links"] == 3 and g4["bytes_per_step_xgmi"] == 3 * nb


def test_refuses_more_rccl_ranks_than_gpus():
    """`--gpus N` with the nccl (RCCL) backend and fewer than N visible GPUs exits non-zero
    with a clear message (ranks would share cards and report a false 'strong' number);
    gloo rehearsals and one-rank runs are not refused."""
    sys.path.insert(0, ROOT)
    import bench

    with pytest.raises(SystemExit) as ei:
        bench.check_devices(8, "nccl", 1)
    assert "only 1 GPU" in str(ei.value.code)
    bench.check_devices(8, "nccl", 8)
    bench.check_devices(2, "gloo", 1)
    bench.check_devices(1, "nccl", 1)
    # end to end on this GPU-less host: both spawned ranks refuse, the launcher fails
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK",
                                                             "LZ_BENCH_BACKEND")}
    env["HIP_VISIBLE_DEVICES"] = ""  # no GPU visible even on a GPU box
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "2"],
                       capture_output=True, text=True, timeout=300, cwd=ROOT, env=env)
    assert r.returncode != 0 and "GPU(s) visible" in r.stderr, (r.returncode, r.stderr[-2000:])
    assert not [ln for ln in r.stdout.splitlines() if ln.startswith("{")]


@pytest.mark.gpu
def test_bench_line_contract_steps20():
    base = json.load(open(os.path.join(ROOT, "BASELINE.json")))
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "20", "--warmup", "5",
                        "--no-cpu-baseline", "--no-extras", "--no-drift"],
                       capture_output=True, text=True, timeout=300, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    d = json.loads(lines[0])
    assert d["metric"] == base["metric"] and d["unit"] == "env-steps/s"
    assert d["n_gpus"] == 1 and d["steps"] == 20 and d["warmup"] == 5
    assert d["higher_is_better"] is True and d["scaling"] == "strong" and d["vs_baseline"] is None
    assert d["dtype"] == "f32" and d["data"].startswith("synthetic")
    assert d["config"]["envs_per_gpu"] == 1 << 20 and "workload" in d["config"]
    t = d["timing"]
    assert t["steps_per_window"] == 20 and t["timed_steps_total"] == 20 * t["windows"]
    assert t["timed_seconds"] >= 0.2
    assert abs(d["value"] - (1 << 20) * t["timed_steps_total"] / t["timed_seconds"]) < 1e-6 * d["value"]
    assert abs(d["ms_per_step"] - t["timed_seconds"] * 1e3 / t["timed_steps_total"]) < 1e-9
    rf = d["roofline"]
    assert rf["bound"] == "hbm" and rf["unit"] == "GB/s" and rf["peak"] == 8000.0
    assert abs(rf["frac"] - rf["achieved"] / rf["peak"]) < 1e-12
    assert 0.3 < rf["frac"] < 1.0 and "traffic" in rf
    assert rf["achieved"] == pytest.approx(65 * (1 << 20) / (rf["avg_launch_us"] * 1e-6) / 1e9)
    assert "hipGraph replay of 20 lz_step launches" in d["config"]["launch"]


@pytest.mark.parametrize("mode,extra", [("rollout", ["--K", "2048"]),
                                        ("policy", ["--policy", "attn", "--K", "2048"]),
                                        ("step", [])])
def test_multi_rank_line_shape(mode, extra):
    """the N > 1 lines of cfg5's modes state the scaling and the per-GPU
    env count correctly.  Strong (default): --envs is the job's total, split over the
    ranks in contiguous global ids (BASELINE configs[4]: 262,144 envs on 8 GPUs = 32,768
    per GPU); weak: --envs per rank.  Every rank's shard together covers [0, total) once."""
    sys.path.insert(0, ROOT)
    import bench

    for world, envs in ((2, 65536), (8, 262144), (3, 100001)):
        args = bench.parse(["--gpus", str(world), "--mode", mode, "--envs", str(envs)] + extra)
        assert args.scaling == "strong"
        plan = [bench.shard_plan(args, world, r) for r in range(world)]
        assert all(p[0] == envs for p in plan)
        assert [p[1] for p in plan] == [sum(q[2] for q in plan[:r]) for r in range(world)]
        assert sum(p[2] for p in plan) == envs and max(p[2] for p in plan) - min(p[2] for p in plan) <= 1
        total, _, n = plan[0]
        sf = bench.scaling_fields(args, world, total, n, "no collective on step")
        assert sf["n_gpus"] == world and sf["scaling"] == "strong"
        assert sf["config"]["envs_total"] == envs and sf["config"]["envs_per_gpu"] == -(-envs // world)
        assert ("x%d" % world) in sf["config"]["parallelism"]
        wk = bench.parse(["--gpus", str(world), "--mode", mode, "--envs", "32768", "--scaling", "weak"] + extra)
        wplan = [bench.shard_plan(wk, world, r) for r in range(world)]
        assert all(p == (32768 * world, 32768 * r, 32768) for r, p in enumerate(wplan))
        wsf = bench.scaling_fields(wk, world, *wplan[1][::2], "x")
        assert wsf["scaling"] == "weak" and wsf["config"]["envs_per_gpu"] == 32768
        assert wsf["config"]["envs_total"] == 32768 * world
    if mode == "rollout":  # cfg5's per-GPU shard at 8 GPUs
        a8 = bench.parse(["--gpus", "8", "--mode", "rollout", "--envs", "262144"])
        assert bench.shard_plan(a8, 8, 7) == (262144, 7 * 32768, 32768)


def test_launch_description_and_sub_shards():
    """describe_launches states what a window ran (the driver's --steps 20: one 20-launch
    remainder graph; --streams S: per stream); sub_shards tiles a rank's shard with
    consecutive global ids (StreamSplitEnv, bench.py --streams)."""
    sys.path.insert(0, ROOT)
    import bench
    from gym_lorenz.parallel import sub_shards

    tm = {"launches": 20 * 3, "windows": 3, "graph": True, "graph_len": 64, "graph_rem": 20,
          "graph_head": 0, "head_eager": 0, "streams": 1}
    d = bench.describe_launches(tm, False)
    assert "1 hipGraph replay of 20 lz_step launches" in d and "0 eager" in d and "x3 windows" in d
    tm2 = dict(tm, launches=4000, windows=1, graph_rem=32)
    d2 = bench.describe_launches(tm2, False)
    assert "62 hipGraph replays of 64" in d2 and "1 hipGraph replay of 32" in d2
    d3 = bench.describe_launches(dict(tm, streams=4), False)
    assert d3.startswith("per timed window, on each of 4 streams")
    for n, off, S in ((131072, 0, 4), (70001, 3 * 70001, 4), (5, 10, 3)):
        subs = sub_shards(n, off, S)
        assert len(subs) == S and subs[0][0] == off
        assert all(a[0] + a[1] == b[0] for a, b in zip(subs, subs[1:]))
        assert sum(c for _, c in subs) == n
