#!/bin/bash
# Round 3: HBM traffic (separate rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes) of every
# kernel a bench line names, measured on this build -- each summary records the kernel's
# code hash, which bench.py requires before it reports roofline.traffic -- plus the
# headline's kernel trace.  -> gpurun_out/r03_pmc/*_pmc_summary.json
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03_pmc
mkdir -p $O
pass() {  # pass <name> <counter> bench args...
  local name=$1 c=$2; shift 2
  timeout -k 10 180 rocprofv3 --pmc $c -d $O/$name.$c -o run --output-format csv -- python bench.py "$@" --no-cpu-baseline --no-drift --no-extras > $O/$name.$c.log 2>&1
}
one() {  # one <name> <mangled> <match> <envs> <alg_bytes> bench args...
  local name=$1 mangled=$2 match=$3 envs=$4 alg=$5; shift 5
  pass $name FETCH_SIZE "$@" || return 1
  pass $name WRITE_SIZE "$@" || return 1
  python tools/pmc_generic.py $O/$name.FETCH_SIZE $O/$name.WRITE_SIZE "$mangled" "$match" $envs $alg $O/${name}_pmc_summary.json | tee -a $O/summary.jsonl
}
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/head.trace -o run --output-format csv -- python bench.py --no-cpu-baseline --no-extras > $O/head.trace.log 2>&1 || exit 1
one lz_step_1M _ZN2lz6k_stepINS_5SysL3IfEEfLi0EEEvNS_5KArgsE "k_step<lz::SysL3<float>, float, 0>" 1048576 68157440 \
    --launch eager --steps 400 --warmup 40 || exit 1
one cfg2_l3_65k _ZN2lz6k_stepINS_5SysL3IfEEfLi0EEEvNS_5KArgsE "k_step<lz::SysL3<float>, float, 0>" 65536 4259840 \
    --envs 65536 --steps 2048 --warmup 256 --launch eager || exit 1
one cfg3_l3_131k _ZN2lz6k_stepINS_5SysL3IfEEfLi0EEEvNS_5KArgsE "k_step<lz::SysL3<float>, float, 0>" 131072 8519680 \
    --envs 131072 --steps 2048 --warmup 256 --launch eager || exit 1
one pmsm_262k _ZN2lz6k_stepINS_7SysPMSMEfLi0EEEvNS_5KArgsE "k_step<lz::SysPMSM, float, 0>" 262144 32768000 \
    --system pmsm --envs 262144 --steps 256 --warmup 64 --launch eager || exit 1
one hr_1M _ZN2lz6k_stepINS_5SysHRIfEEfLi0EEEvNS_5KArgsE "k_step<lz::SysHR<float>, float, 0>" 1048576 89128960 \
    --system hr --envs 1048576 --steps 256 --warmup 64 --launch eager || exit 1
one l4_1M _ZN2lz6k_stepINS_5SysL4IfEEfLi0EEEvNS_5KArgsE "k_step<lz::SysL4<float>, float, 0>" 1048576 105906176 \
    --system lorenz4 --envs 1048576 --steps 256 --warmup 64 --launch eager || exit 1
one rollout_32k _ZN2lz15k_rollout_splitINS_5SysL3IfEEfLi2ELi7ELb1EEEvNS_5KArgsE "k_rollout_split<lz::SysL3<float>, float, 2, 7, true>" 32768 2752249856 \
    --mode rollout --K 2048 --envs 32768 --steps 8192 --warmup 2048 || exit 1
one rollout_262k _ZN2lz9k_rolloutINS_5SysL3IfEEfLi256ELi7ELb1EEEvNS_5KArgsE "k_rollout<lz::SysL3<float>, float, 256, 7, true>" 262144 22017998848 \
    --mode rollout --K 2048 --envs 262144 --steps 4096 --warmup 2048 || exit 1
VN="--mode vecnorm --system pmsm --envs 262144 --steps 512 --warmup 64"
pass vn FETCH_SIZE $VN || exit 1
pass vn WRITE_SIZE $VN || exit 1
python tools/pmc_generic.py $O/vn.FETCH_SIZE $O/vn.WRITE_SIZE _ZN2lz9k_step_vnINS_7SysPMSMEfLi24EEEvNS_5KArgsENS_5VArgsE "k_step_vn<lz::SysPMSM, float, 24>" 262144 36962304 $O/step_vn_pmc_summary.json | tee -a $O/summary.jsonl || exit 1
python tools/pmc_generic.py $O/vn.FETCH_SIZE $O/vn.WRITE_SIZE _ZN12_GLOBAL__N_110k_vn_applyIfLi6ELb1EEEvNS_11VnApplyArgsE "k_vn_apply<float, 6, true>" 262144 15204352 $O/vn_apply_pmc_summary.json | tee -a $O/summary.jsonl || exit 1
# the SB3-exact VecNormalize collect after the deeper-batched statistics update
B="python bench.py --mode policy --system pmsm --envs 262144 --K 16 --steps 512"
timeout -k 10 300 $B --vecnorm-update step > $O/bench_vn_step.json 2> $O/bench_vn_step.log || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/vn_step.trace -o run --output-format csv -- $B --vecnorm-update step > $O/vn_step.trace.log 2>&1 || exit 1
