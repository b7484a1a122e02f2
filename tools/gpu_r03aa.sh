#!/bin/bash
# Round 3: PMSM / HR rollouts at and above the 131,072 bound -- 256-lane (0) vs one-wave
# groups (variant bit 1<<24), two allocations each, K = 1024
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03_ow
mkdir -p $O
V=0,16777216,0,16777216
for s in pmsm hr; do
  AB_K=1024 AB_VARIANTS=$V AB_ROUNDS=5 timeout -k 10 300 python tools/ab_rollout.py $s 131072 196608 262144 \
    > $O/ab_$s.json 2> $O/ab_$s.err || exit 1
done
