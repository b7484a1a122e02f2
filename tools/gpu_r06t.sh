#!/bin/bash
# r06 stage T: HR's noise share of the small-N rollout: HR 32,768 x 2048 with the process
# noise on / off (one-wave k_rollout), and the split-lane kernel off, two rounds.
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r06t
mkdir -p $O
P="--mode rollout --K 2048 --steps 8192 --no-cpu-baseline --no-drift --no-extras --system hr --envs 32768"
for r in 1 2; do
  for nz in 1 0; do
    for v in 0 512; do
      timeout -k 10 200 python bench.py $P --add-noise $nz --variant $v > $O/hr_nz${nz}_v${v}_$r.json 2>> $O/err.txt || { tail $O/err.txt; exit 1; }
      python -c "
import json;d=json.load(open('$O/hr_nz${nz}_v${v}_$r.json'))
print('hr 32768 noise $nz v$v r$r', round(d['roofline']['avg_launch_us'],1))"
    done
  done
done
echo done
