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
ic)  # the headline state's reuse distance: warm (bench) vs cold (384 MiB copy between steps)
  KN="k_step_multi<lz::SysL3<float>, float, 4"
  for r in 1 2 3; do for m in warm cold; do
    timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/${m}_$r -o run --output-format csv \
      -- python tools/ic_flush.py $m 20 > $O/${m}_$r.json 2> $O/${m}_$r.err || exit 1
  done; done
  ;;
diag)  # graph replays of lz_step: eager, k_step graph, then the default (k_step_multi) graph
  timeout -k 10 200 python bench.py --launch eager $BQ > $O/eager.json 2> $O/eager.err || exit 1
  timeout -k 10 200 python bench.py --variant 16384 $BQ > $O/kstep_graph.json 2> $O/kstep_graph.err || exit 1
  timeout -k 10 200 python bench.py $BQ > $O/default.json 2> $O/default.err || exit 1
  ;;
i8)  # the default bench path first, then the i8x4 attention policies: parity, then A/B vs fp32
  timeout -k 10 200 python bench.py $BQ > $O/default.json 2> $O/default.err || exit 1
  timeout -k 10 900 $PYT -m gpu --maxfail=6 tests/test_gpu_policy_i8x4.py > $O/i8_tests.txt 2>&1 || exit 1
  PB="--mode policy --system hr --envs 32768 --K 2048 --steps 4096 $BQ"
  for r in 1 2; do for pr in fp32 i8x4; do for po in attn attn_ln; do
    timeout -k 10 300 python bench.py $PB --policy $po --precision $pr > $O/${po}_${pr}_$r.json 2>> $O/bench.err || exit 1
  done; done; done
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
