"""HBM traffic per launch of any lz kernel from separate rocprofv3 --pmc FETCH_SIZE /
WRITE_SIZE passes, against its algorithmic bytes (the *_pmc_summary.json format that
bench.py's `traffic` field reads; tools/pmc_summary.py is the calibrated headline case).

Calibration: the gfx950 factors tools/pmc_calib measured on 1 GiB streams
(profiles/r01/lz_step_1M_pmc_summary.json): FETCH_SIZE reports 0.500x the bytes moved
for 4-B and 16-B lanes alike, WRITE_SIZE 1.0x for 1-, 4- and 16-B lanes.  The
counters see traffic leaving the XCD L2s; a working set under the 256 MB MALL is
partly served from there, so below ~100 MB the figure is an upper bound on DRAM bytes.

usage: python tools/pmc_generic.py <fetch_dir> <write_dir> <kernel_mangled> <match>
                                   <envs> <alg_bytes_per_launch> <out.json>
  <match>: a substring of the demangled kernel name as rocprofv3 writes it
"""
import json
import sys

from pmc_summary import per_kernel

from kernel_hash import kernel_code_sha256  # noqa: E402  (tools/)

FETCH_FACTOR = 0.5000092188517252
WRITE_FACTOR = 1.0


def main():
    dfetch, dwrite, mangled, match, envs, alg, out = sys.argv[1:8]
    envs, alg = int(envs), float(alg)
    F = {k: v for k, v in per_kernel(dfetch, "FETCH_SIZE").items() if match in k}
    W = {k: v for k, v in per_kernel(dwrite, "WRITE_SIZE").items() if match in k}
    if len(F) != 1 or len(W) != 1:
        raise SystemExit("kernel match %r ambiguous or absent: %s / %s" % (match, list(F), list(W)))
    raw_f, raw_w = next(iter(F.values())) * 1024, next(iter(W.values())) * 1024
    rd, wr = raw_f / FETCH_FACTOR, raw_w / WRITE_FACTOR
    res = {
        "kernel": mangled, "envs_per_gpu": envs,
        "hbm_bytes_per_launch": rd + wr, "read_bytes": rd, "write_bytes": wr,
        "algorithmic_bytes": alg, "traffic_over_algorithmic": (rd + wr) / alg,
        "raw": {"FETCH_SIZE_KB": raw_f / 1024, "WRITE_SIZE_KB": raw_w / 1024},
        "calibration": {"fetch_factor": FETCH_FACTOR, "write_factor": WRITE_FACTOR,
                        "source": "profiles/r01/lz_step_1M_pmc_summary.json"},
        "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes, "
                  "kernel-trace only; average over the profiled launches",
    }
    # the traffic is valid for exactly this build of the kernel (bench.py load_traffic)
    res["kernel_code_sha256"] = kernel_code_sha256(res["kernel"])
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps({k: res[k] for k in ("kernel", "hbm_bytes_per_launch", "algorithmic_bytes",
                                          "traffic_over_algorithmic")}))


if __name__ == "__main__":
    main()
