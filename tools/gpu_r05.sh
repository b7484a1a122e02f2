#!/bin/bash
# Round 5 GPU runs.  usage: tools/gpu_r05.sh <stage> [out-dir]
#   new   : the round's new / changed GPU tests (default step launches at their selecting
#           sizes, step-after-close, step_multi injected-noise cases, resident server)
#   full  : every -m gpu test + smoke()
#   bench : default bench line, the driver's --steps 20, and the 2-rank self-spawned
#           launcher over gloo on this one GPU (cfg3's strong split + gather accounting)
set -o pipefail
export TMPDIR=/tmp
STAGE=${1:-new}
O=${2:-gpurun_out/r05_$STAGE}
mkdir -p $O
PYT="python -u -m pytest -v --timeout 170 --timeout-method thread -p no:cacheprovider"
BQ="--no-cpu-baseline --no-drift --no-extras"
case $STAGE in
new)
  timeout -k 10 900 $PYT -m gpu --maxfail=8 tests/test_gpu_default_launch.py tests/test_gpu_step_multi.py \
    tests/test_gpu_resident.py tests/test_gpu_policy_branches.py > $O/new_tests.txt 2>&1 || exit 1
  LZ_BENCH_BACKEND=gloo timeout -k 10 300 python bench.py --gpus 2 > $O/bench_gpus2_gloo.json 2> $O/bench_gpus2_gloo.err
  ;;
full)
  timeout -k 10 1000 $PYT -x -m gpu tests > $O/gpu_tests.txt 2>&1 || exit 1
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('SMOKE OK')" > $O/smoke.txt 2>&1
  ;;
bench)
  timeout -k 10 400 python bench.py > $O/bench_default.json 2> $O/bench_default.err || exit 1
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 > $O/bench_steps20.json 2> $O/bench_steps20.err || exit 1
  LZ_BENCH_BACKEND=gloo timeout -k 10 300 python bench.py --gpus 2 > $O/bench_gpus2_gloo.json 2> $O/bench_gpus2_gloo.err
  ;;
esac
