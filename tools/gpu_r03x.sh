#!/bin/bash
# Round 3: LORENZ4 f32 below 256 x CUs envs -- one-wave kernel (0) vs two lanes per env
# (variant 512), two allocations each, K = 2048
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03_l4split
mkdir -p $O
[ -n "$SKIP_SPLIT" ] || AB_VARIANTS=0,512,0,512 AB_ROUNDS=7 timeout -k 10 300 python tools/ab_rollout.py lorenz4 16384 32768 49152 \
  > $O/ab_l4_split.json 2> $O/ab_l4_split.err || exit 1
# and the 256-lane kernel (variant 1<<23) between 32,768 and 65,536
AB_VARIANTS=0,8388608,0,8388608 AB_ROUNDS=7 timeout -k 10 300 python tools/ab_rollout.py lorenz4 40960 49152 57344 \
  > $O/ab_l4_256.json 2> $O/ab_l4_256.err || exit 1
