"""A/B of several builds of libgym_lorenz_amd.so on one bench command: every round runs
each build in its own process (order rotated per round, so clock and placement drift
hit all alike; "default" = the product library, others via LZ_LIB_AB).

  python tools/ab_libs.py <rounds> <lib|default>... -- bench.py args...

Prints one JSON object: per build the bench values, HIP-event launch times and medians."""
import json
import os
import statistics
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def run(lib, args):
    env = dict(os.environ)
    env.pop("LZ_LIB_AB", None)
    if lib != "default":
        env["LZ_LIB_AB"] = os.path.abspath(lib)
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, env=env,
                         capture_output=True, text=True, timeout=400)
    if out.returncode != 0:
        sys.stderr.write(out.stderr[-3000:])
        raise SystemExit(out.returncode)
    d = json.loads([ln for ln in out.stdout.splitlines() if ln.startswith("{")][-1])
    return d["value"], d["roofline"]["avg_launch_us"], d["ms_per_step"] * 1e3


def main():
    sep = sys.argv.index("--")
    rounds, libs, args = int(sys.argv[1]), sys.argv[2:sep], sys.argv[sep + 1:]
    res = {"args": args, "builds": {}}
    for lib in libs:
        res["builds"][lib] = {"values": [], "launch_us": [], "step_us": []}
    for r in range(rounds):
        for j in range(len(libs)):
            lib = libs[(r + j) % len(libs)]
            v, us, st = run(lib, args)
            b = res["builds"][lib]
            b["values"].append(v)
            b["launch_us"].append(us)
            b["step_us"].append(st)
            print(r, lib, v, us, st, file=sys.stderr, flush=True)
    for lib, b in res["builds"].items():
        b["median_value"] = statistics.median(b["values"])
        b["median_launch_us"] = statistics.median(b["launch_us"])
        b["median_step_us"] = statistics.median(b["step_us"])
    print(json.dumps(res))


if __name__ == "__main__":
    main()
