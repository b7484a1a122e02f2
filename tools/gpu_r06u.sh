#!/bin/bash
# r06 stage U: every BASELINE config's own line on the final tree (configs[1] LORENZ4
# 65,536 step + its fused rollout, configs[2]'s per-GPU shards 131,072 / 262,144 at
# 8 / 4 GPUs, configs[3] PMSM 262,144 step with noise, configs[4]'s 32,768 x 2048 rollout).
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r06u
mkdir -p $O
Q="--no-cpu-baseline --no-drift --no-extras"
run() {
  local tag=$1; shift
  timeout -k 10 240 python bench.py $Q "$@" > $O/$tag.json 2>> $O/err.txt || { tail $O/err.txt; exit 1; }
  python -c "
import json;d=json.load(open('$O/$tag.json'))
print('$tag', '%.3e' % d['value'], d['unit'], 'ms/step %.5f' % d['ms_per_step'], 'frac', d['roofline']['frac'], d['roofline'].get('kernel','')[:60])"
}
run cfg1_l4_65536_step --system lorenz4 --envs 65536
run cfg1_l4_65536_rollout --system lorenz4 --envs 65536 --mode rollout --K 2048 --steps 8192
run cfg2_l3_131072_step --system lorenz3 --envs 131072
run cfg2_l3_262144_step --system lorenz3 --envs 262144
run cfg3_pmsm_262144_step --system pmsm --envs 262144
run cfg3_pmsm_262144_rollout --system pmsm --envs 262144 --mode rollout --K 2048 --steps 8192
run cfg4_l3_32768_rollout --system lorenz3 --envs 32768 --mode rollout --K 2048 --steps 8192
echo done
