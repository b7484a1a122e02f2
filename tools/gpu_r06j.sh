#!/bin/bash
# r06 stage J: --head-graph H (the window's first H steps as a graph of their own) at the
# driver's --steps 20 and the default --steps 4000, 1M and 131,072 envs, interleaved.
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r06k
mkdir -p $O
export PYTHONUNBUFFERED=1
for rep in 1 2; do
  for n in 1048576 131072; do
    for st in 20 4000; do
      for h in 0 e2 e4 eager; do
        name=l3_${n}_s${st}_h${h}_r$rep
        timeout -k 10 120 python bench.py --envs $n --steps $st --warmup 5 $(case $h in e*[0-9]) echo --head-eager ${h#e};; eager) echo --launch eager;; *) echo --head-graph $h;; esac) --no-cpu-baseline --no-drift --no-extras \
          > $O/$name.json 2> $O/$name.err || { echo FAILED $name; tail -5 $O/$name.err; exit 1; }
        python -c "import json;d=json.load(open('$O/$name.json'));print('$name','%.3e'%d['value'],'us/step %.3f'%(d['ms_per_step']*1e3),'ev %.3f'%d['roofline']['avg_launch_us'])"
      done
    done
  done
done
echo done
