#!/bin/bash
# Round 3: the split actor / critic f32 policy kernel -- parity, then A/B against the
# one-wave-per-tile kernel (LZ_POL_F32_WAVES=4) at the small-N policy configurations
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03_split
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
  tests/test_gpu_policy_f32.py tests/test_gpu_policy.py > $O/tests.txt 2>&1 || exit 1
b() {  # b <name> bench args...
  local name=$1; shift
  timeout -k 10 300 python bench.py "$@" --no-cpu-baseline --no-extras --no-drift > $O/$name.json 2> $O/$name.log
}
b pmsm_32k_K2048_split --mode policy --system pmsm --envs 32768 --K 2048 --steps 4096 --vecnorm-update rollout || exit 1
(export LZ_POL_F32_WAVES=4; b pmsm_32k_K2048_onewave --mode policy --system pmsm --envs 32768 --K 2048 --steps 4096 --vecnorm-update rollout) || exit 1
b l4_32k_K2048_split --mode policy --system lorenz4 --envs 32768 --K 2048 --steps 4096 --vecnorm-update rollout || exit 1
(export LZ_POL_F32_WAVES=4; b l4_32k_K2048_onewave --mode policy --system lorenz4 --envs 32768 --K 2048 --steps 4096 --vecnorm-update rollout) || exit 1
b pmsm_16k_K16_split --mode policy --system pmsm --envs 16384 --K 16 --steps 512 --vecnorm-update rollout || exit 1
(export LZ_POL_F32_WAVES=4; b pmsm_16k_K16_onewave --mode policy --system pmsm --envs 16384 --K 16 --steps 512 --vecnorm-update rollout) || exit 1
