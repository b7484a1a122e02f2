#!/bin/bash
# Round 3: one bench line per configuration at HEAD -> gpurun_out/r03_cfg/*.json
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03_cfg
mkdir -p $O
b() {  # b <name> bench args...
  local name=$1; shift
  timeout -k 10 300 python bench.py "$@" --no-cpu-baseline --no-extras --no-drift > $O/$name.json 2> $O/$name.log
}
b cfg2_l3_65k --envs 65536 || exit 1
b cfg3_l3_131k --envs 131072 || exit 1
b cfg4_pmsm_262k --system pmsm --envs 262144 || exit 1
b hr_1M --system hr --envs 1048576 || exit 1
b l4_1M --system lorenz4 --envs 1048576 || exit 1
b l3_4M --envs 4194304 || exit 1
b cfg5_rollout_32k --mode rollout --K 2048 --envs 32768 --steps 8192 || exit 1
b cfg5_rollout_262k --mode rollout --K 2048 --envs 262144 --steps 4096 || exit 1
b vecnorm_pmsm_262k --mode vecnorm --system pmsm --envs 262144 || exit 1
b vecnorm_l3_1M --mode vecnorm --envs 1048576 || exit 1
b policy_f32_pmsm_262k_step --mode policy --system pmsm --envs 262144 --K 16 --steps 512 || exit 1
b policy_f32_pmsm_262k_rollout --mode policy --system pmsm --envs 262144 --K 16 --steps 512 --vecnorm-update rollout || exit 1
b policy_f32_pmsm_32k_K2048 --mode policy --system pmsm --envs 32768 --K 2048 --steps 4096 --vecnorm-update rollout || exit 1
