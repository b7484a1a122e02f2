#!/bin/bash
# r06 stage E: ragged-group action prefetch -- the rollout parity tests (ragged sizes
# included), then rollout timings at ragged vs whole-group sizes.
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r06e
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_parity.py tests/test_gpu_rollout_pair.py tests/test_gpu_cfg5.py tests/test_gpu_policy_branches.py \
  tests/test_gpu_rk4.py -k "rollout or cfg5 or branch" > $O/tests.txt 2>&1 || { echo TESTS FAILED; grep -E "FAILED|Error" $O/tests.txt | head; tail -30 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
run() {  # name, args...
  local name=$1; shift
  timeout -k 10 120 python bench.py --mode rollout --K 2048 --steps 8192 --no-cpu-baseline --no-drift --no-extras "$@" \
    > $O/$name.json 2> $O/$name.err || { echo "$name FAILED"; tail -20 $O/$name.err; exit 1; }
  python -c "import json;d=json.load(open('$O/$name.json'));print('$name', '%.3e'%d['value'], 'launch_us %.1f'%d['roofline']['avg_launch_us'], d['roofline']['kernel'][:42])"
}
for n in 24576 24608 32768 32800 16384 16416 20480; do run pmsm_$n --system pmsm --envs $n; done
for n in 24576 24608; do run pmsm1_$n --system pmsm --envs $n --variant 268435456; done
for n in 32768 32800; do run hr_$n --system hr --envs $n; done
for n in 32768 32784 16384 16400; do run l3_$n --system lorenz3 --envs $n; done
echo done
