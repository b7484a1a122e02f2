#!/bin/bash
# Round 3: LORENZ4 f32 rollouts on the 256-lane kernel from 3/4 x 256 x CUs envs --
# rollout parity (incl. LORENZ4 49,153), then LORENZ4 rollout lines at 49,152 / 57,344.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03_l4y
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_legacy.py -v -m gpu -k "rollout" \
  --timeout 120 --timeout-method thread -p no:cacheprovider > $O/tests.txt 2>&1 || exit 1
for n in 49152 57344; do
  timeout -k 10 300 python bench.py --system lorenz4 --mode rollout --K 2048 --envs $n --steps 8192 \
    --no-cpu-baseline --no-extras --no-drift > $O/l4_${n}_rollout.json 2> $O/l4_${n}_rollout.log || exit 1
done
