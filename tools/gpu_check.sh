#!/bin/bash
# One GPU-box session: parity tests, smoke, bench variants.  Stops at the first
# crash / timeout (exit codes 124, 134, 137, 139) so nothing else touches the GPU.
set -u
mkdir -p gpurun_out
crashed() { case "$1" in 124|134|137|139) return 0;; esac; return 1; }
run() {  # run <name> <timeout_s> cmd...
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc" | tee -a gpurun_out/summary.txt
  if crashed $rc; then echo "STOP after $name (rc=$rc)" | tee -a gpurun_out/summary.txt; exit $rc; fi
  return 0
}
: > gpurun_out/summary.txt
for step in "$@"; do
  case "$step" in
    tests) run gpu_tests 900 python -m pytest tests -q -m gpu -p no:cacheprovider ;;
    smoke) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) run bench 600 python bench.py ;;
    bench_quick) run bench_quick 300 python bench.py --steps 2000 --warmup 200 --no-cpu-baseline ;;
    sweep)
      for e in 65536 131072 262144 1048576 4194304; do
        run "sweep_graph_$e" 200 python bench.py --envs $e --steps 4000 --warmup 200 --no-cpu-baseline --no-drift
        run "sweep_eager_$e" 200 python bench.py --envs $e --steps 2000 --warmup 200 --no-cpu-baseline --no-drift --launch eager
      done ;;
    prof)
      export TMPDIR=/tmp
      run prof 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python bench.py --steps 2000 --warmup 200 --no-cpu-baseline --no-drift ;;
    ab) run ab_step 600 python tools/ab_step.py 131072 1048576 4194304 ;;
    ab_blk) AB_VARIANTS=0,8,16,24 run ab_blk 600 python tools/ab_step.py 131072 1048576 4194304 ;;
    ab_bar) AB_VARIANTS=0,4 run ab_bar 600 python tools/ab_step.py 65536 131072 1048576 4194304 ;;
    ab_pmsm) AB_SYSTEM=pmsm run ab_pmsm 600 python tools/ab_step.py 262144 1048576 ;;
    counters) run counters 120 rocprofv3 -L ;;
    configs)
      run cfg2_l3_65k 200 python bench.py --envs 65536 --no-cpu-baseline --no-drift
      run cfg3_l3_1M_strong8_shard 200 python bench.py --envs 131072 --no-cpu-baseline --no-drift
      run cfg4_pmsm_262k 300 python bench.py --system pmsm --envs 262144 --steps 4000
      run cfg5_rollout_32k 300 python bench.py --mode rollout --K 2048 --envs 32768 --steps 16384
      run cfg5_rollout_262k 300 python bench.py --mode rollout --K 2048 --envs 262144 --steps 8192
      run l4_1M 200 python bench.py --system lorenz4 --envs 1048576
      run hr_1M 200 python bench.py --system hr --envs 1048576
      run l3_4M 200 python bench.py --envs 4194304 --steps 2000 --no-cpu-baseline --no-drift ;;
    configs2)
      run cfg4_pmsm_262k 300 python bench.py --system pmsm --envs 262144 --steps 4000
      run cfg5_rollout_32k 300 python bench.py --mode rollout --K 2048 --envs 32768 --steps 16384
      run cfg5_rollout_262k 300 python bench.py --mode rollout --K 2048 --envs 262144 --steps 8192 ;;
    policy_tests) run gpu_policy_tests 600 python -m pytest tests/test_gpu_policy.py -q -m gpu -p no:cacheprovider -s ;;
    policy_bench)
      run policy_pmsm_262k_K16 300 python bench.py --mode policy --system pmsm --envs 262144 --K 16 --steps 4096
      run policy_pmsm_32k_K2048 300 python bench.py --mode policy --system pmsm --envs 32768 --K 2048 --steps 8192
      run policy_l3_1M_K16 300 python bench.py --mode policy --system lorenz3 --envs 1048576 --K 16 --steps 1024 ;;
    policy_prof)
      export TMPDIR=/tmp
      run policy_prof 300 rocprofv3 --kernel-trace --stats -d gpurun_out/policy_prof -o run --output-format csv -- python bench.py --mode policy --system pmsm --envs 262144 --K 16 --steps 2048 ;;
    attn_tests) run gpu_attn_tests 600 python -u -m pytest tests/test_gpu_policy_attn.py -v -s -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread ;;
    attn_bench)
      run attn_hr_32k_K2048 300 python bench.py --mode policy --policy attn --system hr --envs 32768 --K 2048 --steps 4096
      run attn_hr_262k_K16 300 python bench.py --mode policy --policy attn --system hr --envs 262144 --K 16 --steps 1024
      run attn_pmsm_262k_K16 300 python bench.py --mode policy --policy attn --system pmsm --envs 262144 --K 16 --steps 1024 ;;
    attn_ln_bench)
      run attn_ln_hr_32k_K2048 300 python bench.py --mode policy --policy attn_ln --system hr --envs 32768 --K 2048 --steps 4096
      run attn_ln_hr_262k_K16 300 python bench.py --mode policy --policy attn_ln --system hr --envs 262144 --K 16 --steps 1024 ;;
    attn_prof)
      export TMPDIR=/tmp
      run attn_prof 300 rocprofv3 --kernel-trace --stats -d gpurun_out/attn_prof -o run --output-format csv -- python bench.py --mode policy --policy attn --system hr --envs 32768 --K 2048 --steps 4096 ;;
    vecnorm_bench)
      run vn_l3_1M 300 python bench.py --mode vecnorm --envs 1048576 --steps 2000 --warmup 200
      run vn_pmsm_262k 300 python bench.py --mode vecnorm --system pmsm --envs 262144 --steps 2000 --warmup 200
      run vn_pmsm_1M 300 python bench.py --mode vecnorm --system pmsm --envs 1048576 --steps 2000 --warmup 200 ;;
    split) run ab_split 600 python tools/ab_split.py 131072 1048576 ;;
    dist2) LZ_BENCH_BACKEND=gloo run dist2 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 500 --warmup 64 --envs 262144 ;;
    pmc)
      export TMPDIR=/tmp
      run pmc_f_calib 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch -o calib --output-format csv -- ./tools/pmc_calib
      run pmc_w_calib 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_write -o calib --output-format csv -- ./tools/pmc_calib
      run pmc_f_step 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch -o step --output-format csv -- python bench.py --steps 256 --warmup 64 --no-cpu-baseline --no-drift --launch eager
      run pmc_w_step 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_write -o step --output-format csv -- python bench.py --steps 256 --warmup 64 --no-cpu-baseline --no-drift --launch eager
      run pmc_summary 60 python tools/pmc_summary.py gpurun_out/pmc_fetch gpurun_out/pmc_write 1048576 gpurun_out/pmc_summary.json ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
