# HBM traffic (rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, separate passes) of the config
# kernels other than the headline; summaries -> gpurun_out/pmc_cfg/*_pmc_summary.json
# (copied to profiles/r01/configs/, where bench.py's `traffic` lookup finds them).
set -e
export TMPDIR=/tmp
O=gpurun_out/pmc_cfg
mkdir -p $O
pass() {  # pass <name> <counter> bench args...
  local name=$1 c=$2; shift 2
  timeout -k 10 180 rocprofv3 --pmc $c -d $O/$name.$c -o run --output-format csv -- python bench.py "$@" --no-cpu-baseline --no-drift > $O/$name.$c.log 2>&1
}
one() {  # one <name> <mangled> <match> <envs> <alg_bytes> bench args...
  local name=$1 mangled=$2 match=$3 envs=$4 alg=$5; shift 5
  pass $name FETCH_SIZE "$@"
  pass $name WRITE_SIZE "$@"
  python tools/pmc_generic.py $O/$name.FETCH_SIZE $O/$name.WRITE_SIZE "$mangled" "$match" $envs $alg $O/${name}_pmc_summary.json | tee -a $O/summary.jsonl
}
one pmsm_262k _ZN2lz6k_stepINS_7SysPMSMEfLi0EEEvNS_5KArgsE "k_step<lz::SysPMSM, float, 0>" 262144 32768000 \
    --system pmsm --envs 262144 --steps 256 --warmup 64 --launch eager
one hr_1M _ZN2lz6k_stepINS_5SysHRIfEEfLi0EEEvNS_5KArgsE "k_step<lz::SysHR<float>, float, 0>" 1048576 89128960 \
    --system hr --envs 1048576 --steps 256 --warmup 64 --launch eager
one l4_1M _ZN2lz6k_stepINS_5SysL4IfEEfLi0EEEvNS_5KArgsE "k_step<lz::SysL4<float>, float, 0>" 1048576 105906176 \
    --system lorenz4 --envs 1048576 --steps 256 --warmup 64 --launch eager
one rollout_32k _ZN2lz15k_rollout_splitINS_5SysL3IfEEfLi2ELi7EEEvNS_5KArgsE "k_rollout_split<lz::SysL3<float>, float, 2, 7>" 32768 2752249856 \
    --mode rollout --K 2048 --envs 32768 --steps 4096 --warmup 2048
one rollout_262k _ZN2lz9k_rolloutINS_5SysL3IfEEfLi256ELi7EEEvNS_5KArgsE "k_rollout<lz::SysL3<float>, float, 256, 7>" 262144 22017998848 \
    --mode rollout --K 2048 --envs 262144 --steps 4096 --warmup 2048
