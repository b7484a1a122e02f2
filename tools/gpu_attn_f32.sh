#!/bin/bash
# Round 3: float32 attention actor-critics -- parity tests and a first throughput line
# (HR 32,768 envs x K = 2,048, code/train.py's and code/lorenz_filter/train.py's shapes)
# -- plus the multi-handle resident server tests.  A test FAILURE (pytest exit 1) lets
# the next step run; anything else (timeout, abort, fault) ends the script.
set -u
export TMPDIR=/tmp
O=gpurun_out/r03_attn
mkdir -p $O
ok() { local s=$1; [ $s -eq 0 ] || [ $s -eq 1 ] || exit $s; }
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
  tests/test_gpu_resident.py tests/test_gpu_state_index.py -s > $O/tests_resident.txt 2>&1; ok $?
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_policy_attn_f32.py tests/test_gpu_vecnorm_step.py -s > $O/tests.txt 2>&1; ok $?
timeout -k 10 300 python bench.py --mode policy --policy attn --system hr --envs 32768 --K 2048 --steps 4096 > $O/bench_attn_32k.json 2> $O/bench_attn_32k.log || exit 1
timeout -k 10 300 python bench.py --mode policy --policy attn_ln --system hr --envs 32768 --K 2048 --steps 4096 > $O/bench_attn_ln_32k.json 2> $O/bench_attn_ln_32k.log || exit 1
