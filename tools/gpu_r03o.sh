#!/bin/bash
# Round 3: temporal (L2-merged) vs non-temporal done-byte stores -- A/B in every env
# kernel that writes a done byte per env and step
set -o pipefail
O=gpurun_out/r03_done
mkdir -p $O
AB_VARIANTS=0,32,0,32 timeout -k 10 300 python tools/ab_step.py 131072 1048576 4194304 > $O/ab_kstep_l3.json 2> $O/ab_kstep_l3.err || exit 1
AB_VARIANTS=0,32,0,32 AB_SYSTEM=pmsm AB_NOISE=1 timeout -k 10 300 python tools/ab_step.py 262144 > $O/ab_kstep_pmsm.json 2> $O/ab_kstep_pmsm.err || exit 1
AB_VARIANTS=0,4194304,0,4194304 AB_SYSTEM=hr timeout -k 10 300 python tools/ab_step.py 1048576 > $O/ab_multi_hr.json 2> $O/ab_multi_hr.err || exit 1
AB_VARIANTS=0,2097152,0,2097152 AB_ROUNDS=9 timeout -k 10 300 python tools/ab_rollout.py lorenz3 262144 > $O/ab_rollout_262k.json 2> $O/ab_rollout_262k.err || exit 1
AB_VARIANTS=0,262144,0,262144 AB_ROUNDS=9 timeout -k 10 300 python tools/ab_rollout.py lorenz3 32768 131071 > $O/ab_split.json 2> $O/ab_split.err || exit 1
