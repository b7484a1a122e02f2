# Round-2 PMC + kernel traces: the small-N per-step configs (cfg2 65,536 envs, cfg3's
# 131,072-env shard) and the rebuilt cfg5 rollout kernels; separate --pmc passes per
# counter; each bench line first, then its kernel trace.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/pmc_r02
mkdir -p $O
pass() {  # pass <name> <counter> bench args...
  local name=$1 c=$2; shift 2
  timeout -k 10 180 rocprofv3 --pmc $c -d $O/$name.$c -o run --output-format csv -- python bench.py "$@" --launch eager --no-cpu-baseline --no-drift --no-extras > $O/$name.$c.log 2>&1
}
one() {  # one <name> <mangled> <match> <envs> <alg_bytes> bench args...
  local name=$1 mangled=$2 match=$3 envs=$4 alg=$5; shift 5
  timeout -k 10 200 python bench.py "$@" --no-cpu-baseline --no-drift --no-extras > $O/${name}_bench.json 2> $O/${name}_bench.err || return 1
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/$name.trace -o run --output-format csv -- python bench.py "$@" --no-cpu-baseline --no-drift --no-extras > $O/$name.trace.log 2>&1 || return 1
  pass $name FETCH_SIZE "$@" || return 1
  pass $name WRITE_SIZE "$@" || return 1
  python tools/pmc_generic.py $O/$name.FETCH_SIZE $O/$name.WRITE_SIZE "$mangled" "$match" $envs $alg $O/${name}_pmc_summary.json | tee -a $O/summary.jsonl
}
one cfg2_l3_65k _ZN2lz6k_stepINS_5SysL3IfEEfLi0EEEvNS_5KArgsE "k_step<lz::SysL3<float>, float, 0>" 65536 4259840 \
    --envs 65536 --steps 2048 --warmup 256 || exit 1
one cfg3_l3_131k _ZN2lz6k_stepINS_5SysL3IfEEfLi0EEEvNS_5KArgsE "k_step<lz::SysL3<float>, float, 0>" 131072 8519680 \
    --envs 131072 --steps 2048 --warmup 256 || exit 1
one rollout_32k _ZN2lz15k_rollout_splitINS_5SysL3IfEEfLi2ELi7ELb1EEEvNS_5KArgsE "k_rollout_split<lz::SysL3<float>, float, 2, 7, true>" 32768 2752249856 \
    --mode rollout --K 2048 --envs 32768 --steps 16384 --warmup 2048 || exit 1
one rollout_262k _ZN2lz9k_rolloutINS_5SysL3IfEEfLi256ELi7ELb1EEEvNS_5KArgsE "k_rollout<lz::SysL3<float>, float, 256, 7, true>" 262144 22017998848 \
    --mode rollout --K 2048 --envs 262144 --steps 8192 --warmup 2048 || exit 1
