#!/bin/bash
# Round 3: LORENZ4 f32 rollouts switch to the 256-lane kernel from 256 x CUs envs, and the
# action-free systems' rollout alternates two LDS obs tiles -- rollout parity (LORENZ4 /
# singlecontrol at 256-lane sizes), the divergence diagnostic, then the LORENZ4 lines.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03_l4x
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_cfg5.py -v -m gpu -k "rollout" \
  --timeout 120 --timeout-method thread -p no:cacheprovider > $O/tests.txt 2>&1
rc=$?
timeout -k 10 120 python tools/diag_rollout_steps.py lorenz4 70001 > $O/diag_l4_70001.txt 2>&1 || exit 1
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python bench.py --system lorenz4 --mode rollout --K 2048 --envs 65536 --steps 8192 \
  --no-cpu-baseline --no-extras --no-drift > $O/cfg2_l4_65k_rollout.json 2> $O/cfg2_l4_65k_rollout.log || exit 1
timeout -k 10 300 python bench.py --system lorenz4 --mode rollout --K 2048 --envs 262144 --steps 4096 \
  --no-cpu-baseline --no-extras --no-drift > $O/l4_262k_rollout.json 2> $O/l4_262k_rollout.log || exit 1
