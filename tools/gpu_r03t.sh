#!/bin/bash
# Round 3: split-lane rollout store policy on top of temporal done bytes: + temporal
# rewards (SV 3), + temporal obs (SV 5), all temporal (SV 7); three allocations each
set -o pipefail
O=gpurun_out/r03_done
mkdir -p $O
V=0,786432,1048576,1835008
AB_VARIANTS=$V,$V,$V AB_ROUNDS=5 timeout -k 10 400 python tools/ab_rollout.py lorenz3 32768 > $O/ab_split_sv.json 2> $O/ab_split_sv.err || exit 1
