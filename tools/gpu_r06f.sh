#!/bin/bash
# r06 stage F: HIP runtime knobs vs the per-step launch boundary (cfg3's 131,072-env shard,
# cfg2's 65,536, the 1M headline): kernel-argument placement and graph packet capture.
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r06f
mkdir -p $O
export PYTHONUNBUFFERED=1
run() {  # name, envs, env-assignments...
  local name=$1 n=$2; shift 2
  env "$@" timeout -k 10 120 python bench.py --envs $n --no-cpu-baseline --no-drift --no-extras \
    > $O/$name.json 2> $O/$name.err || { echo "$name FAILED"; tail -20 $O/$name.err; exit 1; }
  python -c "import json;d=json.load(open('$O/$name.json'));print('$name', '%.3e'%d['value'], 'us/step %.3f'%(d['ms_per_step']*1e3), 'ev %.3f'%d['roofline']['avg_launch_us'])"
}
for rep in 1 2; do
  for n in 131072 65536 1048576; do
    run base_${n}_$rep $n X=1
    run devkarg1_${n}_$rep $n HIP_FORCE_DEV_KERNARG=1
    run devkarg0_${n}_$rep $n HIP_FORCE_DEV_KERNARG=0
    run gpc0_${n}_$rep $n DEBUG_CLR_GRAPH_PACKET_CAPTURE=0
    run gpc1_${n}_$rep $n DEBUG_CLR_GRAPH_PACKET_CAPTURE=1
  done
done
echo done
