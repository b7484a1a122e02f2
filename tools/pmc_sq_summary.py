"""Issue / wait accounting of one kernel from the passes tools/step_counters.sh takes:
kernel trace (--stats), FETCH_SIZE, WRITE_SIZE, two SQ passes.  Writes
<out>_pmc_summary.json with the HBM bytes per launch (gfx950 calibration of
tools/pmc_generic.py) and the derived issue split.

  python tools/pmc_sq_summary.py <dir prefix> <kernel substring> <mangled> <envs>
                                 <alg bytes per launch> <out.json> [note]

Units: SQ_WAVE_CYCLES / SQ_WAIT_* / SQ_ACTIVE_INST_* / SQ_BUSY_CYCLES count quad-cycles
(x4 = shader cycles), summed over all waves (SQ_*) or all SIMDs (busy); GRBM_GUI_ACTIVE is
summed over the 8 XCDs (MI355X_MICROARCH.md "rocprofv3 PMC slots", "DVFS give-back").
"""
import csv
import glob
import json
import os
import sys

from kernel_hash import kernel_code_sha256  # noqa: E402  (tools/)

FETCH_FACTOR = 0.5000092188517252  # tools/pmc_generic.py (r01 calibration)
SIMDS = 1024


def counters(d, match):
    acc = {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            if match not in row["Kernel_Name"]:
                continue
            acc.setdefault(row["Counter_Name"], []).append(float(row["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in acc.items()}


def trace_avg_ns(d, match):
    for f in glob.glob(os.path.join(d, "**", "*kernel_stats.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            if match in row["Name"]:
                return float(row["AverageNs"]), int(row["Calls"]), float(row["MinNs"])
    raise SystemExit("kernel %r not in the trace of %s" % (match, d))


def main():
    pre, match, mangled, envs, alg, out = sys.argv[1:7]
    note = sys.argv[7] if len(sys.argv) > 7 else ""
    envs, alg = int(envs), float(alg)
    avg_ns, calls, min_ns = trace_avg_ns(pre + ".trace", match)
    c = {}
    for p in ("sq1", "sq2"):
        c.update(counters(pre + "." + p, match))
    fetch = counters(pre + ".FETCH_SIZE", match)["FETCH_SIZE"] * 1024 / FETCH_FACTOR
    write = counters(pre + ".WRITE_SIZE", match)["WRITE_SIZE"] * 1024
    waves = c["SQ_WAVES"]
    wave_cyc = 4 * c["SQ_WAVE_CYCLES"]
    # GRBM_GUI_ACTIVE / 8 over the kernel time reads high below ~0.3 ms dispatches
    # (MI355X_MICROARCH.md "DVFS give-back"): busy fractions use the 2.4 GHz peak clock,
    # so they are LOWER bounds
    clk_grbm = c["GRBM_GUI_ACTIVE"] / 8 / (avg_ns * 1e-9) / 1e9
    kernel_cycles = avg_ns * 1e-9 * 2.4e9
    d = {
        "grbm_clock_ghz_profiled": clk_grbm,
        "busy_fractions_at_ghz": 2.4,
        "valu_busy_frac": 4 * c["SQ_ACTIVE_INST_VALU"] / (SIMDS * kernel_cycles),
        "simd_busy_frac": 4 * c["SQ_BUSY_CYCLES"] / (SIMDS * kernel_cycles) if "SQ_BUSY_CYCLES" in c else None,
        "wave_cycles_split": {
            "active_issue": 4 * c["SQ_ACTIVE_INST_ANY"] / wave_cyc,
            "issue_stall": 4 * c["SQ_WAIT_INST_ANY"] / wave_cyc,
            "waitcnt_parked": 4 * c["SQ_WAIT_ANY"] / wave_cyc,
        },
        "valu_insts_per_wave": c["SQ_INSTS_VALU"] / waves,
        "trans_insts_per_wave": c.get("SQ_INSTS_VALU_TRANS_F", 0.0) / waves,
        "salu_insts_per_wave": c.get("SQ_INSTS_SALU", 0.0) / waves,
        "lds_insts_per_wave": c.get("SQ_INSTS_LDS", 0.0) / waves,
        "resident_waves_avg": wave_cyc / kernel_cycles,
        "hbm_frac_of_8TBs": (fetch + write) / (avg_ns * 1e-9) / 8e12,
    }
    res = {
        "kernel": mangled, "envs_per_gpu": envs,
        "avg_kernel_ns_kernel_trace": avg_ns, "min_kernel_ns": min_ns, "calls": calls,
        "hbm_bytes_per_launch": fetch + write, "read_bytes": fetch, "write_bytes": write,
        "algorithmic_bytes": alg, "traffic_over_algorithmic": (fetch + write) / alg,
        "counters_per_dispatch": c, "derived": d, "note": note,
        "method": "rocprofv3 kernel trace + separate --pmc passes (FETCH_SIZE; WRITE_SIZE; "
                  "SQ issue/wait set; SQ instruction mix + GRBM_GUI_ACTIVE), kernel trace only; "
                  "averages over the profiled dispatches (tools/step_counters.sh)",
    }
    # the traffic is valid for exactly this build of the kernel (bench.py load_traffic)
    res["kernel_code_sha256"] = kernel_code_sha256(res["kernel"])
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps({"kernel": match, "avg_us": avg_ns / 1e3, "traffic_x": res["traffic_over_algorithmic"],
                      **{k: v for k, v in d.items() if k != "wave_cycles_split"},
                      **d["wave_cycles_split"]}, indent=1))


if __name__ == "__main__":
    main()
