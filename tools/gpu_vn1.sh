#!/bin/bash
# single-launch VecNormalize step: parity vs the two-call form, then bench both forms
# (PMSM 262,144) and a kernel trace of the single launch
set -u
export TMPDIR=/tmp
O=gpurun_out/vn1
mkdir -p $O
ok() { local s=$1; [ $s -eq 0 ] || [ $s -eq 1 ] || exit $s; }
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread \
  tests/test_gpu_vecnorm.py tests/test_gpu_multirank.py -s > $O/tests.txt 2>&1; ok $?
B="python bench.py --mode vecnorm --system pmsm --envs 262144 --steps 2048 --warmup 128 --no-cpu-baseline"
for L in one two; do
  timeout -k 10 300 $B --vn-launch $L > $O/bench_$L.json 2> $O/bench_$L.log || exit 1
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace_one -o run --output-format csv -- $B --vn-launch one > $O/trace_one.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --mode vecnorm --system lorenz3 --envs 262144 --steps 2048 --warmup 128 --no-cpu-baseline > $O/bench_l3_one.json 2> $O/bench_l3_one.log || exit 1
