#!/bin/bash
# r06 stage V: LORENZ3 262,144 step, two tiles (default) vs one (variant 16384), three
# rotated rounds on one box (stage U measured 4.23 us where earlier boxes gave 3.74 - 3.84).
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r06v
mkdir -p $O
Q="--no-cpu-baseline --no-drift --no-extras --system lorenz3"
for r in 1 2 3; do
  for v in 0 16384; do
    for n in 262144 131072; do
      timeout -k 10 200 python bench.py $Q --envs $n --variant $v > $O/l3_${n}_v${v}_r$r.json 2>> $O/err.txt || { tail $O/err.txt; exit 1; }
      python -c "
import json;d=json.load(open('$O/l3_${n}_v${v}_r$r.json'))
print('l3 $n v$v r$r', round(d['roofline']['avg_launch_us'],3), round(d['ms_per_step']*1e3,3))"
    done
  done
done
echo done
