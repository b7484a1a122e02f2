#!/bin/bash
# HBM traffic (rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, separate passes) of the LORENZ4 f32
# 256-lane rollout at 65,536 envs x K = 2048 (cfg2's lorenz_env_transient on the fused path)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/pmc_l4
mkdir -p $O
B="bench.py --system lorenz4 --mode rollout --K 2048 --envs 65536 --steps 4096 --no-cpu-baseline --no-drift --no-extras"
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 180 rocprofv3 --pmc $c -d $O/l4_65k.$c -o run --output-format csv -- python $B > $O/l4_65k.$c.log 2>&1 || exit 1
done
python tools/pmc_generic.py $O/l4_65k.FETCH_SIZE $O/l4_65k.WRITE_SIZE \
  _ZN2lz9k_rolloutINS_5SysL4IfEEfLi256ELi7ELb0ELb1EEEvNS_5KArgsE "k_rollout<lz::SysL4<float>, float, 256, 7, false, true>" \
  65536 4970250240 $O/l4_rollout_65k_pmc_summary.json > $O/summary.txt 2>&1 || exit 1
timeout -k 10 300 python $B > $O/bench_after.json 2> $O/bench_after.log || exit 1
