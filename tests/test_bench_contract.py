"""bench.py's output contract (the driver parses its one JSON line): the CPU baseline
leg on the host (no GPU), and on the GPU the whole line at the driver's own short
setting (--steps 20): the BASELINE metric, whole-job value, exactly K timed steps per
window, the roofline object with frac = achieved / peak, and a launch description that
says what ran."""
import json
import os
import subprocess
import sys

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
    assert d["higher_is_better"] is True and d["scaling"] == "weak" and d["vs_baseline"] is None
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
