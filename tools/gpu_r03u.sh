#!/bin/bash
# Round 3: BASELINE configs[1] names lorenz_env_transient (LORENZ4) at 65,536 envs; the
# configs table so far carried LORENZ3 there.  One bench line each for LORENZ4 at
# 65,536: the per-step API and the fused 2048-step rollout; LORENZ3 65,536 rollout beside.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03_cfg2
mkdir -p $O
b() {  # b <name> bench args...
  local name=$1; shift
  timeout -k 10 300 python bench.py "$@" --no-cpu-baseline --no-extras --no-drift > $O/$name.json 2> $O/$name.log
}
b cfg2_l4_65k --system lorenz4 --envs 65536 || exit 1
b cfg2_l4_65k_rollout --system lorenz4 --mode rollout --K 2048 --envs 65536 --steps 8192 || exit 1
b cfg2_l3_65k_rollout --mode rollout --K 2048 --envs 65536 --steps 8192 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/l4_65k.trace -o run --output-format csv -- python bench.py --system lorenz4 --envs 65536 --no-cpu-baseline --no-extras --no-drift > $O/l4_65k.trace.log 2>&1 || exit 1
