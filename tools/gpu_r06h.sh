#!/bin/bash
# r06 stage H: tiles per workgroup of the step kernel at the per-GPU shards of the strong
# 2 / 4 / 8-GPU headline (524,288 / 262,144 / 131,072 envs) -- variant bits 14-15 force
# 1 / 2 / 4 tiles (0 = the default choice), two interleaved repeats.
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r06h
mkdir -p $O
export PYTHONUNBUFFERED=1
for rep in 1 2; do
  for n in 524288 262144 131072 393216; do
    for v in 0 16384 32768 49152; do
      timeout -k 10 120 python bench.py --envs $n --variant $v --no-cpu-baseline --no-drift --no-extras \
        > $O/l3_${n}_v${v}_r$rep.json 2> $O/l3_${n}_v${v}_r$rep.err || { echo FAILED $n $v; tail -5 $O/l3_${n}_v${v}_r$rep.err; exit 1; }
      python -c "import json;d=json.load(open('$O/l3_${n}_v${v}_r$rep.json'));print($n,$v,'%.3e'%d['value'],'us/step %.3f'%(d['ms_per_step']*1e3),'frac %.3f'%d['roofline']['frac'])"
    done
  done
done
echo done
