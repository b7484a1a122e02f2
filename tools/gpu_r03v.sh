#!/bin/bash
# Round 3: where does the 256-lane rollout kernel overtake the one-wave (64-lane) one for
# LORENZ4 / PMSM / HR?  (LORENZ3 float32 switches at 256 x CUs envs, measured in r03b; the
# other systems still switch at 131,072.)  Variant bit 1<<23 = the 256-lane kernel at any
# N; each variant on two allocations (placement noise), K = 2048.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03_xover
mkdir -p $O
V=0,8388608,0,8388608
for s in lorenz4 pmsm hr; do
  AB_VARIANTS=$V AB_ROUNDS=7 timeout -k 10 300 python tools/ab_rollout.py $s 32768 65536 98304 \
    > $O/ab_$s.json 2> $O/ab_$s.err || exit 1
done
