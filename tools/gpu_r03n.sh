#!/bin/bash
# Round 3: cfg5 split-lane rollout -- non-temporal vs temporal stores per stream (A/B)
set -o pipefail
O=gpurun_out/r03_rollst
mkdir -p $O
AB_VARIANTS=0,262144,786432,0,262144,786432 AB_ROUNDS=15 timeout -k 10 400 python tools/ab_rollout.py lorenz3 32768 65536 > $O/ab_store_policy2.json 2> $O/ab_store_policy2.err || exit 1
