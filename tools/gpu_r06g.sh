#!/bin/bash
# r06 stage G: ragged last groups on the full DMA path (parity + timings), then stage F.
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r06g
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_ragged.py tests/test_gpu_rollout_pair.py tests/test_gpu_parity.py -k "ragged or pair or rollout" \
  > $O/tests.txt 2>&1 || { echo TESTS FAILED; grep -E "FAILED|Error" $O/tests.txt | head; tail -30 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
run() {  # name, args...
  local name=$1; shift
  timeout -k 10 120 python bench.py --mode rollout --K 2048 --steps 8192 --no-cpu-baseline --no-drift --no-extras "$@" \
    > $O/$name.json 2> $O/$name.err || { echo "$name FAILED"; tail -20 $O/$name.err; exit 1; }
  python -c "import json;d=json.load(open('$O/$name.json'));print('$name', '%.3e'%d['value'], 'launch_us %.1f'%d['roofline']['avg_launch_us'])"
}
run l3_16384 --system lorenz3 --envs 16384
run l3_16400 --system lorenz3 --envs 16400
run l3_32768 --system lorenz3 --envs 32768
run l3_32784 --system lorenz3 --envs 32784
run pmsm_24576 --system pmsm --envs 24576
run pmsm_24592 --system pmsm --envs 24592
run pmsm1_24576 --system pmsm --envs 24576 --variant 268435456
run pmsm1_24608 --system pmsm --envs 24608 --variant 268435456
run hr_32768 --system hr --envs 32768
run hr_32784 --system hr --envs 32784
bash tools/gpu_r06f.sh
