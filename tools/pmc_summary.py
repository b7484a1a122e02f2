"""Turn rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes into HBM bytes per launch.

Calibration (MI355X_MICROARCH.md "HBM": FETCH_SIZE under-reports 16-B/lane streams
by 2x on gfx950; other widths uncalibrated): tools/pmc_calib moves known bytes with
4-B, 16-B and 1-B lanes; measured/known gives a factor per width.  The step kernel's
raw counters are divided by the algorithmic-byte-weighted factor of its own mix of
widths (reads: 12 B/env of 4-B plane loads + 12 B/env of 16-B staged actions;
writes: 16 B/env of 4-B plane + reward stores, 24 B/env of 16-B staged obs,
1 B/env done flags).

usage: python tools/pmc_summary.py <prof_dir_fetch> <prof_dir_write> <envs> <out.json>
"""
import csv
import glob
import json
import os
import sys

from kernel_hash import kernel_code_sha256  # noqa: E402  (tools/)

GIB = 1 << 30
STEP = "k_step<lz::SysL3<float>, float, 0>"
STEP_MANGLED = "_ZN2lz6k_stepINS_5SysL3IfEEfLi0EEEvNS_5KArgsE"


def per_kernel(d, counter):
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    acc = {}
    for f in files:
        for row in csv.DictReader(open(f)):
            if row.get("Counter_Name") != counter:
                continue
            k = row["Kernel_Name"]
            acc.setdefault(k, []).append(float(row["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in acc.items()}


def find(m, key):
    for k, v in m.items():
        if key in k:
            return v
    raise KeyError(key)


def main():
    dfetch, dwrite, envs, out = sys.argv[1], sys.argv[2], int(sys.argv[3]), sys.argv[4]
    F = per_kernel(dfetch, "FETCH_SIZE")
    W = per_kernel(dwrite, "WRITE_SIZE")
    r4 = find(F, "copy4") * 1024 / GIB
    r16 = find(F, "copy16") * 1024 / GIB
    w4 = find(W, "copy4") * 1024 / GIB
    w16 = find(W, "copy16") * 1024 / GIB
    w1 = find(W, "store1") * 1024 / GIB
    fr = (12 * r4 + 12 * r16) / 24
    fw = (16 * w4 + 24 * w16 + 1 * w1) / 41
    raw_f = find(F, STEP) * 1024
    raw_w = find(W, STEP) * 1024
    rd, wr = raw_f / fr, raw_w / fw
    alg_rd, alg_wr = 24 * envs, 41 * envs
    res = {
        "kernel": STEP_MANGLED, "envs_per_gpu": envs,
        "hbm_bytes_per_launch": rd + wr,
        "read_bytes": rd, "write_bytes": wr,
        "algorithmic_bytes": alg_rd + alg_wr,
        "traffic_over_algorithmic": (rd + wr) / (alg_rd + alg_wr),
        "raw": {"FETCH_SIZE_KB": raw_f / 1024, "WRITE_SIZE_KB": raw_w / 1024},
        "calibration": {"fetch_4B": r4, "fetch_16B": r16, "write_4B": w4, "write_16B": w16,
                        "write_1B": w1, "fetch_factor_mix": fr, "write_factor_mix": fw},
        "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes; "
                  "measured/known factors from tools/pmc_calib (1 GiB streams)",
    }
    # the traffic is valid for exactly this build of the kernel (bench.py load_traffic)
    res["kernel_code_sha256"] = kernel_code_sha256(res["kernel"])
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
