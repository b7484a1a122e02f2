"""A/B of two builds of libgym_lorenz_amd.so on the same bench command, alternated
(A B A B ...) in separate processes so clocks and placement drift hit both alike.

  python tools/ab_lib.py <libA.so|default> <libB.so|default> <rounds> -- bench.py args...

Prints one JSON object: per-variant bench values per round and their medians.
"""
import json
import os
import statistics
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def run(lib, args):
    env = dict(os.environ)
    if lib != "default":
        env["LZ_LIB_AB"] = os.path.abspath(lib)
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, env=env,
                         capture_output=True, text=True, timeout=400)
    if out.returncode != 0:
        sys.stderr.write(out.stderr[-3000:])
        raise SystemExit(out.returncode)
    line = [ln for ln in out.stdout.splitlines() if ln.startswith("{")][-1]
    d = json.loads(line)
    return d["value"], d.get("roofline", {}).get("avg_launch_us")


def main():
    sep = sys.argv.index("--")
    a, b, rounds = sys.argv[1], sys.argv[2], int(sys.argv[3])
    args = sys.argv[sep + 1:]
    res = {"A": a, "B": b, "args": args, "A_values": [], "B_values": [], "A_us": [], "B_us": []}
    for r in range(rounds):
        for tag, lib in (("A", a), ("B", b)) if r % 2 == 0 else (("B", b), ("A", a)):
            v, us = run(lib, args)
            res[tag + "_values"].append(v)
            res[tag + "_us"].append(us)
            print(tag, r, v, us, file=sys.stderr, flush=True)
    for t in "AB":
        res[t + "_median"] = statistics.median(res[t + "_values"])
    res["B_over_A"] = res["B_median"] / res["A_median"]
    print(json.dumps(res))


if __name__ == "__main__":
    main()
