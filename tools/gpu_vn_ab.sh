#!/bin/bash
# VecNormalize fused step (PMSM 262,144 envs): parity tests, then A/B of the step
# workgroup size (LZ_VN_BLOCK) and the normalise-pass row workgroups (LZ_VN_APPLY_BLOCKS),
# then a kernel trace of the default.
set -e
out=gpu_vn_ab
mkdir -p gpurun_out/$out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gpu_vecnorm.py tests/test_gpu_multirank.py tests/test_gpu_parity.py > gpurun_out/$out/tests.txt 2>&1
for cfg in "1024 512" "256 512" "1024 256" "1024 1024" "1024 128"; do
  set -- $cfg
  LZ_VN_BLOCK=$1 LZ_VN_APPLY_BLOCKS=$2 timeout -k 10 120 python bench.py --mode vecnorm \
    --system pmsm --envs 262144 --steps 2048 --warmup 256 > gpurun_out/$out/b_$1_$2.json
done
timeout -k 10 120 python bench.py --mode vecnorm --system pmsm --envs 1048576 --steps 512 \
  --warmup 64 > gpurun_out/$out/b_1M.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/$out/prof \
  -o vn -- python3 $GRAFT_REPO_ROOT/bench.py --mode vecnorm --system pmsm --envs 262144 \
  --steps 1024 --warmup 64 > $GRAFT_REPO_ROOT/gpurun_out/$out/prof.log 2>&1
