#!/bin/bash
# r06 stage O: the lane-pair kernel's DMA prefetch distance (variant 4096: 15 steps,
# 1024: 3, default 7), PMSM 32,768 x 2048, three interleaved rounds.
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r06o
mkdir -p $O
export PYTHONUNBUFFERED=1
for rep in 1 2 3; do
  for v in 0 4096 1024; do
    name=pmsm32k_v${v}_r$rep
    timeout -k 10 120 python bench.py --system pmsm --mode rollout --envs 32768 --K 2048 --steps 8192 --variant $v \
      --no-cpu-baseline --no-drift --no-extras > $O/$name.json 2> $O/$name.err || { echo FAILED $name; exit 1; }
    python -c "import json;d=json.load(open('$O/$name.json'));print('$name','launch_us %.1f'%d['roofline']['avg_launch_us'], d['roofline']['kernel'][:40])"
  done
done
echo done
