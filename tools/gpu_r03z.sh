#!/bin/bash
# Round 3: f32 policy kernels -- split-net kernel == one-wave kernel with grid-stride repeats
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03_pol
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_policy_f32.py -v -m gpu \
  --timeout 120 --timeout-method thread -p no:cacheprovider > $O/tests.txt 2>&1 || exit 1
