#!/bin/bash
# Round 3: k_step_multi as the default at the one-generation sizes -- parity, bench lines
# (HR 1M, PMSM 1M, cfg4 PMSM 262k), PMC traffic of the kernels those lines name (and of
# the PMSM kernels whose code moved), kernel trace of the HR 1M line.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03_multi2
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
  tests/test_gpu_step_multi.py > $O/tests.txt 2>&1 || exit 1
b() {  # b <name> bench args...
  local name=$1; shift
  timeout -k 10 300 python bench.py "$@" --no-cpu-baseline --no-extras --no-drift > $O/$name.json 2> $O/$name.log
}
b hr_1M --system hr --envs 1048576 || exit 1
b pmsm_1M --system pmsm --envs 1048576 || exit 1
b cfg4_pmsm_262k --system pmsm --envs 262144 || exit 1
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
one hr_1M _ZN2lz12k_step_multiINS_5SysHRIfEEfLi4EEEvNS_5KArgsE "k_step_multi<lz::SysHR<float>, float, 4>" 1048576 89128960 \
    --system hr --envs 1048576 --steps 256 --warmup 64 --launch eager || exit 1
one pmsm_1M _ZN2lz12k_step_multiINS_7SysPMSMEfLi4EEEvNS_5KArgsE "k_step_multi<lz::SysPMSM, float, 4>" 1048576 131072000 \
    --system pmsm --envs 1048576 --steps 256 --warmup 64 --launch eager || exit 1
one pmsm_262k _ZN2lz6k_stepINS_7SysPMSMEfLi0EEEvNS_5KArgsE "k_step<lz::SysPMSM, float, 0>" 262144 32768000 \
    --system pmsm --envs 262144 --steps 256 --warmup 64 --launch eager || exit 1
VN="--mode vecnorm --system pmsm --envs 262144 --steps 512 --warmup 64"
pass vn FETCH_SIZE $VN || exit 1
pass vn WRITE_SIZE $VN || exit 1
python tools/pmc_generic.py $O/vn.FETCH_SIZE $O/vn.WRITE_SIZE _ZN2lz9k_step_vnINS_7SysPMSMEfLi24EEEvNS_5KArgsENS_5VArgsE "k_step_vn<lz::SysPMSM, float, 24>" 262144 36962304 $O/step_vn_pmc_summary.json | tee -a $O/summary.jsonl || exit 1
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/hr_1M.trace -o run --output-format csv -- python bench.py --system hr --envs 1048576 --no-cpu-baseline --no-extras --no-drift > $O/hr_1M.trace.log 2>&1 || exit 1
