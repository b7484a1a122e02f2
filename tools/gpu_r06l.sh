#!/bin/bash
# r06 stage L: re-check on the final build, interleaved on one box: the PMSM lane pair
# (default at 32,768) vs one lane (1<<28), LORENZ3 262,144 two tiles (default) vs one (16384).
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r06l
mkdir -p $O
export PYTHONUNBUFFERED=1
for rep in 1 2 3; do
  for v in 0 268435456; do
    name=pmsm32k_v${v}_r$rep
    timeout -k 10 120 python bench.py --system pmsm --mode rollout --envs 32768 --K 2048 --steps 8192 --variant $v \
      --no-cpu-baseline --no-drift --no-extras > $O/$name.json 2> $O/$name.err || { echo FAILED $name; exit 1; }
    python -c "import json;d=json.load(open('$O/$name.json'));print('$name','%.3e'%d['value'],'launch_us %.1f'%d['roofline']['avg_launch_us'])"
  done
  for v in 0 16384; do
    name=l3_262144_v${v}_r$rep
    timeout -k 10 120 python bench.py --envs 262144 --variant $v --no-cpu-baseline --no-drift --no-extras \
      > $O/$name.json 2> $O/$name.err || { echo FAILED $name; exit 1; }
    python -c "import json;d=json.load(open('$O/$name.json'));print('$name','%.3e'%d['value'],'us/step %.3f'%(d['ms_per_step']*1e3))"
  done
done
echo done
# HBM traffic of the two new default kernels (separate FETCH_SIZE / WRITE_SIZE passes)
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $c -d $R/$O/l3_262k_$c -o run --output-format csv -- \
    python3 $R/bench.py --envs 262144 --launch eager --steps 400 --warmup 40 --no-cpu-baseline --no-drift --no-extras \
    > $R/$O/l3_262k_$c.log 2>&1 || { echo PMC FAILED; tail -3 $R/$O/l3_262k_$c.log; exit 1; }
  timeout -s KILL 120 rocprofv3 --pmc $c -d $R/$O/pmsm_pair_$c -o run --output-format csv -- \
    python3 $R/bench.py --system pmsm --mode rollout --envs 32768 --K 2048 --steps 4096 --no-cpu-baseline --no-drift --no-extras \
    > $R/$O/pmsm_pair_$c.log 2>&1 || { echo PMC FAILED; tail -3 $R/$O/pmsm_pair_$c.log; exit 1; }
done
echo pmc done
