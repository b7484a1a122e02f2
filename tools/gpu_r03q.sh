#!/bin/bash
# Round 3: small-N rollout kernel choice and done-store policy, each variant on 3
# separate allocations (placement noise) -- split nt / split temporal done / 256-lane nt /
# 256-lane temporal done; 262k: 256-lane nt vs temporal done
set -o pipefail
O=gpurun_out/r03_done
mkdir -p $O
V4=0,262144,8388608,10485760
AB_VARIANTS=$V4,$V4,$V4 AB_ROUNDS=5 timeout -k 10 500 python tools/ab_rollout.py lorenz3 32768 65536 > $O/ab_small_rollout3.json 2> $O/ab_small_rollout3.err || exit 1
AB_VARIANTS=0,2097152,0,2097152,0,2097152 AB_ROUNDS=5 timeout -k 10 400 python tools/ab_rollout.py lorenz3 262144 > $O/ab_rollout_262k_3.json 2> $O/ab_rollout_262k_3.err || exit 1
