#!/bin/bash
# r06 stage D: cfg5's multi-GPU lines rehearsed as 2 gloo ranks sharing the box's one GPU
# (VERDICT r05 #5), the default headline bench (the checked caller-buffer rings, item 1)
# and the driver's --steps 20 line; the pair kernel's lower crossover (24,576 / 28,672).
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r06d
mkdir -p $O
export PYTHONUNBUFFERED=1
run() {  # name, timeout, args...
  local name=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$name.json 2> $O/$name.err || { echo "$name FAILED"; tail -20 $O/$name.err; exit 1; }
  python -c "import json;d=json.load(open('$O/$name.json'));print('$name', '%.3e'%d['value'], d['n_gpus'], d['scaling'], d['config'].get('envs_total'), d['config'].get('envs_per_gpu'))"
}
export LZ_BENCH_BACKEND=gloo
run rollout_l3_gpus2_gloo 300 python bench.py --gpus 2 --mode rollout --envs 65536 --K 2048 --steps 8192
run rollout_pmsm_gpus2_gloo 300 python bench.py --gpus 2 --system pmsm --mode rollout --envs 65536 --K 2048 --steps 8192
run policy_attn_hr_gpus2_gloo 300 python bench.py --gpus 2 --system hr --mode policy --policy attn --envs 65536 --K 2048 --steps 4096
run policy_mlp_pmsm_gpus2_gloo 300 python bench.py --gpus 2 --system pmsm --mode policy --policy mlp --envs 65536 --K 2048 --steps 4096 --vecnorm-update rollout
unset LZ_BENCH_BACKEND
run bench_default 300 python bench.py
run bench_steps20 300 python bench.py --steps 20 --warmup 5
for n in 24576 24608 28672; do
  for v in 0 268435456; do
    run pmsm_${n}_v$v 120 python bench.py --system pmsm --mode rollout --envs $n --K 2048 --steps 8192 --variant $v --no-cpu-baseline --no-drift --no-extras
  done
done
echo done
