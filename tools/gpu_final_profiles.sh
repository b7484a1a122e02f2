#!/bin/bash
# Round-2 closing profiles: the fp32 policy rollout and the f1 VecNormalize step at
# their bench configs, kernel-trace stats of the same commands.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/final_prof
mkdir -p $O
timeout -k 10 200 python bench.py --mode policy --system pmsm --envs 262144 --K 16 --steps 4096 --no-extras > $O/policy_f32_pmsm262k.json 2> $O/policy_f32_pmsm262k.err || exit 1
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/policy_trace -o run --output-format csv -- python bench.py --mode policy --system pmsm --envs 262144 --K 16 --steps 2048 --no-extras > $O/policy_trace.log 2>&1 || exit 1
timeout -k 10 200 python bench.py --mode vecnorm --system pmsm --envs 262144 --steps 2048 --warmup 256 > $O/vecnorm_pmsm262k.json 2> $O/vecnorm_pmsm262k.err || exit 1
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/vecnorm_trace -o run --output-format csv -- python bench.py --mode vecnorm --system pmsm --envs 262144 --steps 1024 --warmup 64 > $O/vecnorm_trace.log 2>&1 || exit 1
