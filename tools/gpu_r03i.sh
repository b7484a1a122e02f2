#!/bin/bash
# Round 3: k_step_multi tile count vs env count (where one E = 4 generation pays)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03_multi
mkdir -p $O
AB_VARIANTS=16384,49152,16384,49152 AB_SYSTEM=hr timeout -k 10 300 \
  python tools/ab_step.py 524288 786432 917504 1048576 1310720 2097152 > $O/ab_hr_sizes.json 2> $O/ab_hr_sizes.err || exit 1
AB_VARIANTS=16384,49152,16384,49152 AB_SYSTEM=pmsm AB_NOISE=1 timeout -k 10 300 \
  python tools/ab_step.py 524288 786432 917504 1048576 1310720 2097152 > $O/ab_pmsm_sizes.json 2> $O/ab_pmsm_sizes.err || exit 1
