#!/bin/bash
# Round 3: temporal vs non-temporal done stores in the PMSM / HR K-step rollouts (256-lane
# kernel, done path), three allocations per variant
set -o pipefail
O=gpurun_out/r03_done
mkdir -p $O
AB_VARIANTS=0,2097152,0,2097152,0,2097152 AB_ROUNDS=5 AB_K=1024 timeout -k 10 400 python tools/ab_rollout.py pmsm 262144 > $O/ab_rollout_pmsm_262k.json 2> $O/ab_rollout_pmsm_262k.err || exit 1
AB_VARIANTS=0,2097152,0,2097152,0,2097152 AB_ROUNDS=5 AB_K=1024 timeout -k 10 400 python tools/ab_rollout.py hr 262144 > $O/ab_rollout_hr_262k.json 2> $O/ab_rollout_hr_262k.err || exit 1
