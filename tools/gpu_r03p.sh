#!/bin/bash
# Round 3: small-N rollout kernel choice and done-store policy (A/B): split-lane (nt /
# temporal done), one-lane one-wave, 256-lane (nt / temporal done)
set -o pipefail
O=gpurun_out/r03_done
mkdir -p $O
AB_VARIANTS=0,262144,256,8388608,10485760,262144 AB_ROUNDS=9 timeout -k 10 500 python tools/ab_rollout.py lorenz3 32768 65536 131071 > $O/ab_small_rollout.json 2> $O/ab_small_rollout.err || exit 1
AB_VARIANTS=0,2097152,0,2097152 AB_ROUNDS=15 timeout -k 10 300 python tools/ab_rollout.py lorenz3 262144 > $O/ab_rollout_262k_b.json 2> $O/ab_rollout_262k_b.err || exit 1
