#!/bin/bash
# One GPU-box session: parity tests, smoke, bench variants.  Stops at the first
# crash / timeout (exit codes 124, 134, 137, 139) so nothing else touches the GPU.
set -u
mkdir -p gpurun_out
crashed() { case "$1" in 124|134|137|139) return 0;; esac; return 1; }
run() {  # run <name> <timeout_s> cmd...
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc" | tee -a gpurun_out/summary.txt
  if crashed $rc; then echo "STOP after $name (rc=$rc)" | tee -a gpurun_out/summary.txt; exit $rc; fi
  return 0
}
: > gpurun_out/summary.txt
for step in "$@"; do
  case "$step" in
    tests) run gpu_tests 900 python -m pytest tests -q -m gpu -p no:cacheprovider ;;
    smoke) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) run bench 600 python bench.py ;;
    bench_quick) run bench_quick 300 python bench.py --steps 2000 --warmup 200 --no-cpu-baseline ;;
    sweep)
      for e in 65536 131072 262144 1048576 4194304; do
        run "sweep_graph_$e" 200 python bench.py --envs $e --steps 4000 --warmup 200 --no-cpu-baseline --no-drift
        run "sweep_eager_$e" 200 python bench.py --envs $e --steps 2000 --warmup 200 --no-cpu-baseline --no-drift --launch eager
      done ;;
    prof)
      export TMPDIR=/tmp
      run prof 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python bench.py --steps 2000 --warmup 200 --no-cpu-baseline --no-drift ;;
    ab) run ab_step 600 python tools/ab_step.py 131072 1048576 4194304 ;;
    ab_pmsm) AB_SYSTEM=pmsm run ab_pmsm 600 python tools/ab_step.py 262144 1048576 ;;
    counters) run counters 120 rocprofv3 -L ;;
    pmc)
      export TMPDIR=/tmp
      run pmc_f_calib 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch -o calib --output-format csv -- ./tools/pmc_calib
      run pmc_w_calib 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_write -o calib --output-format csv -- ./tools/pmc_calib
      run pmc_f_step 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch -o step --output-format csv -- python bench.py --steps 256 --warmup 64 --no-cpu-baseline --no-drift --launch eager
      run pmc_w_step 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_write -o step --output-format csv -- python bench.py --steps 256 --warmup 64 --no-cpu-baseline --no-drift --launch eager
      run pmc_summary 60 python tools/pmc_summary.py gpurun_out/pmc_fetch gpurun_out/pmc_write 1048576 gpurun_out/pmc_summary.json ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
