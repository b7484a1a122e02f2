#!/bin/bash
# Round 3: SB3-exact VecNormalize in the fused float32 rollout -- parity tests, the
# throughput of both update modes at PMSM 262,144 envs K=16 (code/lorenz_pmsm/train.py's
# A2C shape), and a kernel trace of the per-step collect.  -> gpurun_out/r03_vn/
set -u
export TMPDIR=/tmp
O=gpurun_out/r03_vn
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_vecnorm_step.py tests/test_gpu_policy_f32.py tests/test_gpu_multirank.py -s > $O/tests.txt 2>&1 || exit 1
B="python bench.py --mode policy --system pmsm --envs 262144 --K 16 --steps 512"
timeout -k 10 300 $B --vecnorm-update step > $O/bench_step.json 2> $O/bench_step.log || exit 1
timeout -k 10 300 $B --vecnorm-update rollout > $O/bench_rollout.json 2> $O/bench_rollout.log || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace_step -o run --output-format csv -- $B --vecnorm-update step > $O/trace_step.log 2>&1 || exit 1
