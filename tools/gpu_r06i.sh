#!/bin/bash
# r06 stage I: two tiles per workgroup at 262,144 envs for PMSM / HR (LORENZ3 won there in
# stage H), and LORENZ3's neighbours 229,376 / 294,912, two repeats.
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r06i
mkdir -p $O
export PYTHONUNBUFFERED=1
for rep in 1 2; do
  for sn in pmsm:262144 hr:262144 lorenz3:229376 lorenz3:294912 lorenz3:262144; do
    s=${sn%%:*}; n=${sn##*:}
    for v in 0 32768; do
      timeout -k 10 120 python bench.py --system $s --envs $n --variant $v --no-cpu-baseline --no-drift --no-extras \
        > $O/${s}_${n}_v${v}_r$rep.json 2> $O/${s}_${n}_v${v}_r$rep.err || { echo FAILED $s $n $v; tail -5 $O/${s}_${n}_v${v}_r$rep.err; exit 1; }
      python -c "import json;d=json.load(open('$O/${s}_${n}_v${v}_r$rep.json'));print('$s',$n,$v,'%.3e'%d['value'],'us/step %.3f'%(d['ms_per_step']*1e3),'frac %.3f'%d['roofline']['frac'])"
    done
  done
done
echo done
