#!/bin/bash
# resident server (doorbell) + RCCL single rank + f32 attention (distributed LN stack)
# tests, latency tables, LN attention bench with 4 vs 8 waves per workgroup
set -u
export TMPDIR=/tmp
O=gpurun_out/r03e
mkdir -p $O
ok() { local s=$1; [ $s -eq 0 ] || [ $s -eq 1 ] || exit $s; }
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread \
  tests/test_gpu_resident.py tests/test_gpu_rccl.py tests/test_gpu_policy_attn_f32.py -s > $O/tests.txt 2>&1; ok $?
timeout -k 10 200 python -u tools/resident_latency.py > $O/resident_latency.json 2> $O/resident_latency.log || exit 1
timeout -k 10 240 python -u tools/single_env_latency.py > $O/single_env_latency.json 2> $O/single_env_latency.log || exit 1
for W in 4 8; do
  LZ_ATTN_F32_WAVES=$W timeout -k 10 300 python bench.py --mode policy --policy attn_ln --system hr --envs 32768 --K 2048 --steps 4096 > $O/bench_attn_ln_w$W.json 2> $O/bench_attn_ln_w$W.log || exit 1
done
