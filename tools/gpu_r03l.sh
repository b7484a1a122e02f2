#!/bin/bash
# Round 3: HR step with host-derived dt/2, dt/6 and the min/max range check -- full GPU
# suite (KArgs grew), then same-box A/B against the previous build (abso/lib_base.so)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03_hrtrim
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread \
  -p no:cacheprovider > $O/gpu_tests.txt 2>&1 || exit 1
timeout -k 10 400 python tools/ab_lib.py abso/lib_base.so default 4 -- --system hr --envs 1048576 --no-cpu-baseline --no-extras --no-drift > $O/ab_hr_1M.json 2> $O/ab_hr_1M.err || exit 1
timeout -k 10 400 python tools/ab_lib.py abso/lib_base.so default 3 -- --system hr --envs 2097152 --no-cpu-baseline --no-extras --no-drift > $O/ab_hr_2M.json 2> $O/ab_hr_2M.err || exit 1
