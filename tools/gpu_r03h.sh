#!/bin/bash
# Round 3: multi-tile step kernel (k_step_multi) -- parity vs k_step, then A/B of 1 / 2 / 4
# tiles per workgroup for PMSM (cfg4, noise) and HR float32 over env counts.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03_multi
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
  tests/test_gpu_step_multi.py > $O/tests.txt 2>&1 || exit 1
AB_VARIANTS=16384,32768,49152,16384 AB_SYSTEM=pmsm AB_NOISE=1 timeout -k 10 300 \
  python tools/ab_step.py 65536 131072 262144 1048576 > $O/ab_pmsm.json 2> $O/ab_pmsm.err || exit 1
AB_VARIANTS=16384,32768,49152,16384 AB_SYSTEM=hr timeout -k 10 300 \
  python tools/ab_step.py 131072 262144 1048576 4194304 > $O/ab_hr.json 2> $O/ab_hr.err || exit 1
