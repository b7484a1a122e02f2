#!/bin/bash
# Round 4 GPU runs.  usage: tools/gpu_r04.sh <stage> [out-dir]
#   new   : the round's new / changed GPU tests (RK4 mode, cfg2 LORENZ4 f32, resident
#           latency in fresh processes, odd-K collect, bench contract)
#   full  : every -m gpu test + smoke()
#   bench : default bench line, the driver's --steps 20, --integrator rk4, and the
#           2-rank self-spawned launcher over gloo on this one GPU (cfg3's strong split)
set -o pipefail
export TMPDIR=/tmp
STAGE=${1:-new}
O=${2:-gpurun_out/r04_$STAGE}
mkdir -p $O
PYT="python -u -m pytest -v --timeout 170 --timeout-method thread -p no:cacheprovider"
case $STAGE in
new)
  timeout -k 10 1100 $PYT -m gpu --maxfail=8 tests/test_gpu_rk4.py tests/test_gpu_vecnorm_step.py \
    tests/test_gpu_resident.py tests/test_bench_contract.py \
    "tests/test_gpu_parity.py::test_l4_f32_vs_oracle_cfg2" > $O/new_tests.txt 2>&1
  ;;
full)
  timeout -k 10 1000 $PYT -x -m gpu tests > $O/gpu_tests.txt 2>&1 || exit 1
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('SMOKE OK')" > $O/smoke.txt 2>&1
  ;;
bench)
  timeout -k 10 400 python bench.py > $O/bench_default.json 2> $O/bench_default.err || exit 1
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 > $O/bench_steps20.json 2> $O/bench_steps20.err || exit 1
  timeout -k 10 200 python bench.py --integrator rk4 --no-cpu-baseline > $O/bench_rk4.json 2> $O/bench_rk4.err || exit 1
  LZ_BENCH_BACKEND=gloo timeout -k 10 300 python bench.py --gpus 2 > $O/bench_gpus2_gloo.json 2> $O/bench_gpus2_gloo.err
  ;;
esac
