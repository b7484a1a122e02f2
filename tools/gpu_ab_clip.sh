#!/bin/bash
# A/B: NaN-propagating maximum/minimum clips (v_maximum3/v_minimum3) vs compare+select,
# cfg5 rollout (LORENZ3 32,768 x 2048) and the HR 1M step; then the parity tests that
# cover every clip (rollouts, steps, goldens).
set -u
export TMPDIR=/tmp
O=gpurun_out/ab_clip
mkdir -p $O
ok() { local s=$1; [ $s -eq 0 ] || [ $s -eq 1 ] || exit $s; }
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread \
  -m gpu tests -q > $O/tests.txt 2>&1; ok $?
timeout -k 10 500 python tools/ab_lib.py ab/lib_before_clip.so default 4 -- --mode rollout --K 2048 --envs 32768 --steps 8192 --no-cpu-baseline > $O/ab_rollout_32k.json 2> $O/ab_rollout_32k.log || exit 1
timeout -k 10 400 python tools/ab_lib.py ab/lib_before_clip.so default 3 -- --system hr --envs 1048576 --steps 2000 --no-cpu-baseline --no-drift --no-extras > $O/ab_hr_1M.json 2> $O/ab_hr_1M.log || exit 1
timeout -k 10 400 python tools/ab_lib.py ab/lib_before_clip.so default 3 -- --system pmsm --envs 262144 --steps 4000 --no-cpu-baseline --no-drift --no-extras > $O/ab_pmsm_262k.json 2> $O/ab_pmsm_262k.log || exit 1
