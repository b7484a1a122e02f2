#!/bin/bash
# Round 4: HBM traffic (separate rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes) of every
# step kernel whose machine code changed this round (the step prologue: one kernel-argument
# batch, the tick beside the state loads; k_step_multi's per-system load layout; the RK4
# systems), measured on the final build -- each summary records the kernel's code hash,
# which bench.py requires before it reports roofline.traffic -- plus the headline's
# kernel trace.  -> gpurun_out/r04_pmc_final/*_pmc_summary.json
set -o pipefail
export TMPDIR=/tmp
O=${1:-gpurun_out/r04_pmc_final}
ONLY=${ONLY:-}  # space-separated pass names (e.g. "pmsm_262k vn"): re-measure just those
mkdir -p $O
want() { [ -z "$ONLY" ] || [[ " $ONLY " == *" $1 "* ]]; }
pass() {  # pass <name> <counter> bench args...
  local name=$1 c=$2; shift 2
  timeout -k 10 180 rocprofv3 --pmc $c -d $O/$name.$c -o run --output-format csv -- python bench.py "$@" \
    --no-cpu-baseline --no-drift --no-extras > $O/$name.$c.log 2>&1
}
one() {  # one <name> <mangled> <match> <envs> <alg_bytes> bench args...
  local name=$1 mangled=$2 match=$3 envs=$4 alg=$5; shift 5
  want $name || return 0
  pass $name FETCH_SIZE "$@" || return 1
  pass $name WRITE_SIZE "$@" || return 1
  python tools/pmc_generic.py $O/$name.FETCH_SIZE $O/$name.WRITE_SIZE "$mangled" "$match" $envs $alg \
    $O/${name}_pmc_summary.json | tee -a $O/summary.jsonl
}
want head && { timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/head.trace -o run --output-format csv -- python bench.py \
  --no-cpu-baseline --no-extras > $O/head.trace.log 2>&1 || exit 1; }
E="--launch eager"
one lz_step_1M _ZN2lz12k_step_multiINS_5SysL3IfEEfLi4ELb0EEEvNS_5KArgsE "k_step_multi<lz::SysL3<float>, float, 4" \
  1048576 68157440 $E --steps 400 --warmup 40 || exit 1
one f64_step_1M _ZN2lz6k_stepINS_5SysL3IdEEdLi0EEEvNS_5KArgsE "k_step<lz::SysL3<double>, double, 0>" 1048576 \
  122683392 --dtype float64 $E --steps 400 --warmup 40 || exit 1
one rk4_step_1M _ZN2lz6k_stepINS_8SysL3RK4IfEEfLi0EEEvNS_5KArgsE "k_step<lz::SysL3RK4<float>" 1048576 68157440 \
  --integrator rk4 $E --steps 400 --warmup 40 || exit 1
one cfg2_l3_65k _ZN2lz6k_stepINS_5SysL3IfEEfLi0EEEvNS_5KArgsE "k_step<lz::SysL3<float>, float, 0>" 65536 4259840 \
  --envs 65536 --steps 2048 --warmup 256 $E || exit 1
one cfg3_l3_131k _ZN2lz6k_stepINS_5SysL3IfEEfLi0EEEvNS_5KArgsE "k_step<lz::SysL3<float>, float, 0>" 131072 8519680 \
  --envs 131072 --steps 2048 --warmup 256 $E || exit 1
one pmsm_262k _ZN2lz6k_stepINS_7SysPMSMEfLi0EEEvNS_5KArgsE "k_step<lz::SysPMSM, float, 0>" 262144 32768000 \
  --system pmsm --envs 262144 --steps 256 --warmup 64 $E || exit 1
one l4_1M _ZN2lz6k_stepINS_5SysL4IfEEfLi0EEEvNS_5KArgsE "k_step<lz::SysL4<float>, float, 0>" 1048576 105906176 \
  --system lorenz4 --envs 1048576 --steps 256 --warmup 64 $E || exit 1
one pmsm_multi_1M _ZN2lz12k_step_multiINS_7SysPMSMEfLi4ELb0EEEvNS_5KArgsE "k_step_multi<lz::SysPMSM, float, 4" \
  1048576 131072000 --system pmsm --envs 1048576 --steps 256 --warmup 64 $E || exit 1
one hr_multi_1M _ZN2lz12k_step_multiINS_5SysHRIfEEfLi4ELb0EEEvNS_5KArgsE "k_step_multi<lz::SysHR<float>, float, 4" \
  1048576 89128960 --system hr --envs 1048576 --steps 256 --warmup 64 $E || exit 1
want vn || exit 0
VN="--mode vecnorm --system pmsm --envs 262144 --steps 512 --warmup 64"
pass vn FETCH_SIZE $VN || exit 1
pass vn WRITE_SIZE $VN || exit 1
python tools/pmc_generic.py $O/vn.FETCH_SIZE $O/vn.WRITE_SIZE _ZN2lz9k_step_vnINS_7SysPMSMEfLi24EEEvNS_5KArgsENS_5VArgsE \
  "k_step_vn<lz::SysPMSM, float, 24>" 262144 36962304 $O/step_vn_pmc_summary.json | tee -a $O/summary.jsonl || exit 1
