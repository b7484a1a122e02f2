#!/bin/bash
# Round 3: sustained (bench.py) A/B of 1 vs 4 tiles per workgroup at HR 1M and PMSM 1M,
# alternating, 3 rounds each
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03_multi3
mkdir -p $O
for r in 1 2 3; do
  for v in 16384 49152; do
    for sys in hr pmsm; do
      timeout -k 10 200 python bench.py --system $sys --envs 1048576 --variant $v --no-cpu-baseline --no-extras --no-drift > $O/${sys}_v${v}_r$r.json 2> $O/${sys}_v${v}_r$r.log || exit 1
    done
  done
done
