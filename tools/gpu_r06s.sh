#!/bin/bash
# r06 stage S: is HR's small-N rollout helped by two lanes per env at all? One-wave
# k_rollout (variant 0) vs the split-lane kernel (variant 512: both lanes repeat the step),
# HR with noise at 32,768 / 24,576 / 65,536 x 2048, two rounds each.
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r06s
mkdir -p $O
P="--mode rollout --K 2048 --steps 8192 --no-cpu-baseline --no-drift --no-extras --system hr"
for r in 1 2; do
  for n in 32768 24576 65536; do
    for v in 0 512; do
      timeout -k 10 200 python bench.py $P --envs $n --variant $v > $O/hr_${n}_v${v}_$r.json 2>> $O/err.txt || { tail $O/err.txt; exit 1; }
      python -c "
import json;d=json.load(open('$O/hr_${n}_v${v}_$r.json'))
print('hr $n v$v r$r', round(d['roofline']['avg_launch_us'],1), d['roofline'].get('kernel', ''))"
    done
  done
done
echo done
