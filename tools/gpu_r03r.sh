#!/bin/bash
# Round 3: rollout with temporal done stores by default + the 256-lane kernel from
# 256 x CUs envs -- full GPU suite, cfg5 bench lines, PMC traffic of the three rollout
# kernels those lines name, kernel trace of the 32k line
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03_roll2
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread \
  -p no:cacheprovider > $O/gpu_tests.txt 2>&1 || exit 1
b() {
  local name=$1; shift
  timeout -k 10 300 python bench.py "$@" --no-cpu-baseline --no-extras --no-drift > $O/$name.json 2> $O/$name.log
}
b cfg5_rollout_32k --mode rollout --K 2048 --envs 32768 --steps 8192 || exit 1
b cfg5_rollout_65k --mode rollout --K 2048 --envs 65536 --steps 8192 || exit 1
b cfg5_rollout_262k --mode rollout --K 2048 --envs 262144 --steps 4096 || exit 1
pass() {
  local name=$1 c=$2; shift 2
  timeout -k 10 180 rocprofv3 --pmc $c -d $O/$name.$c -o run --output-format csv -- python bench.py "$@" --no-cpu-baseline --no-drift --no-extras > $O/$name.$c.log 2>&1
}
one() {
  local name=$1 mangled=$2 match=$3 envs=$4 alg=$5; shift 5
  pass $name FETCH_SIZE "$@" || return 1
  pass $name WRITE_SIZE "$@" || return 1
  python tools/pmc_generic.py $O/$name.FETCH_SIZE $O/$name.WRITE_SIZE "$mangled" "$match" $envs $alg $O/${name}_pmc_summary.json | tee -a $O/summary.jsonl
}
one rollout_32k _ZN2lz15k_rollout_splitINS_5SysL3IfEEfLi2ELi7ELb1ELi1EEEvNS_5KArgsE "k_rollout_split<lz::SysL3<float>, float, 2, 7, true, 1>" 32768 2752249856 \
    --mode rollout --K 2048 --envs 32768 --steps 8192 --warmup 2048 || exit 1
one rollout_65k _ZN2lz9k_rolloutINS_5SysL3IfEEfLi256ELi7ELb1ELb1EEEvNS_5KArgsE "k_rollout<lz::SysL3<float>, float, 256, 7, true, true>" 65536 5504499712 \
    --mode rollout --K 2048 --envs 65536 --steps 8192 --warmup 2048 || exit 1
one rollout_262k _ZN2lz9k_rolloutINS_5SysL3IfEEfLi256ELi7ELb1ELb1EEEvNS_5KArgsE "k_rollout<lz::SysL3<float>, float, 256, 7, true, true>" 262144 22017998848 \
    --mode rollout --K 2048 --envs 262144 --steps 4096 --warmup 2048 || exit 1
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/cfg5_32k.trace -o run --output-format csv -- python bench.py --mode rollout --K 2048 --envs 32768 --steps 8192 --no-cpu-baseline --no-extras --no-drift > $O/cfg5_32k.trace.log 2>&1 || exit 1
