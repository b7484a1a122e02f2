#!/bin/bash
# Round 4 GPU runs.  usage: tools/gpu_r04.sh <stage> [out-dir]
#   new   : the round's new / changed GPU tests (RK4 mode, cfg2 LORENZ4 f32, resident
#           latency in fresh processes, odd-K collect, bench contract)
#   full  : every -m gpu test + smoke()
#   bench : default bench line, the driver's --steps 20, --integrator rk4, and the
#           2-rank self-spawned launcher over gloo on this one GPU (cfg3's strong split)
set -o pipefail
export TMPDIR=/tmp
STAGE=${1:-new}
O=${2:-gpurun_out/r04_$STAGE}
mkdir -p $O
PYT="python -u -m pytest -v --timeout 170 --timeout-method thread -p no:cacheprovider"
BQ="--no-cpu-baseline --no-drift --no-extras"
case $STAGE in
new2)  # the branch table (K = 3), the reference-class attention weights, cfg2 LORENZ4 f32
  timeout -k 10 600 $PYT -m gpu --maxfail=8 tests/test_gpu_policy_branches.py \
    "tests/test_gpu_parity.py::test_l4_f32_vs_oracle_cfg2" \
    "tests/test_gpu_policy_attn_f32.py::test_attn_f32_reference_class_weights_bitexact" \
    > $O/new2_tests.txt 2>&1 || exit 1
  timeout -k 10 120 $PYT -s -m gpu "tests/test_gpu_resident.py::test_resident_does_not_block_torch" \
    > $O/resident_latency.txt 2>&1 || exit 1
  timeout -k 10 1000 $PYT -x -m gpu tests > $O/gpu_tests.txt 2>&1 || exit 1
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('SMOKE OK')" > $O/smoke.txt 2>&1
  ;;
resident)  # the one-round-trip request lines: parity, then latency
  timeout -k 10 600 $PYT -m gpu tests/test_gpu_resident.py "tests/test_gpu_rk4.py::test_rk4_resident_server_vs_oracle" \
    -k "resident or dropin" tests/test_gpu_parity.py > $O/resident_tests.txt 2>&1 || exit 1
  timeout -k 10 300 python tools/single_env_latency.py > $O/single_env_latency.json 2> $O/single_env_latency.err || exit 1
  timeout -k 10 300 python tools/resident_latency.py > $O/resident_latency.json 2> $O/resident_latency.err || exit 1
  ;;
pmc)  # PMC traffic of the RK4 headline kernel (separate FETCH_SIZE / WRITE_SIZE passes)
  K=_ZN2lz6k_stepINS_8SysL3RK4IfEEfLi0EEEvNS_5KArgsE
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 180 rocprofv3 --pmc $c -d $O/rk4_$c -o run --output-format csv -- python bench.py \
      --integrator rk4 --launch eager --steps 400 --warmup 40 $BQ > $O/rk4_$c.log 2>&1 || exit 1
  done
  python tools/pmc_generic.py $O/rk4_FETCH_SIZE $O/rk4_WRITE_SIZE $K "k_step<lz::SysL3RK4<float>" 1048576 68157440 \
    $O/rk4_step_1M_pmc_summary.json || exit 1
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/rk4_trace -o run --output-format csv -- python bench.py \
    --integrator rk4 $BQ > $O/rk4_trace.log 2>&1 || exit 1
  ;;
cfg3)  # cfg3's per-GPU shard (131,072) and cfg2 (65,536): where a step's time goes
  for n in 65536 131072; do
    timeout -k 10 200 python bench.py --envs $n $BQ > $O/bench_$n.json 2> $O/bench_$n.err || exit 1
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace_$n -o run --output-format csv \
      -- python bench.py --envs $n $BQ > $O/trace_$n.log 2>&1 || exit 1
  done
  AB_VARIANTS=0,2,16,8,24,3,0 timeout -k 10 300 python tools/ab_step.py 65536 131072 > $O/ab_step_variants.json || exit 1
  for n in 131072 65536; do  # state planes nt / write-through, streamed outputs write-through, both
    timeout -k 10 600 python tools/ab_libs.py 3 default ablib/libgym_lorenz_amd_state_nt.so \
      ablib/libgym_lorenz_amd_state_wt.so ablib/libgym_lorenz_amd_out_wt.so ablib/libgym_lorenz_amd_all_wt.so \
      -- --envs $n $BQ > $O/ab_stores_$n.json 2> $O/ab_stores_$n.err || exit 1
  done
  timeout -k 10 120 tools/launch_floor > $O/launch_floor.txt 2>&1
  ;;
tick)  # the tick as a vector load + one kernel-argument round trip (vs HEAD's k_step)
  timeout -k 10 600 $PYT -m gpu --maxfail=4 tests/test_gpu_parity.py tests/test_gpu_vecnorm_step.py \
    "tests/test_gpu_rk4.py::test_l3_rk4_step_vs_oracle" > $O/tick_tests.txt 2>&1 || exit 1
  for n in 131072 65536 1048576; do
    timeout -k 10 600 python tools/ab_libs.py 3 default ablib/libgym_lorenz_amd_base.so \
      ablib/libgym_lorenz_amd_statent.so -- --envs $n $BQ > $O/ab_tick_$n.json 2> $O/ab_tick_$n.err || exit 1
  done
  for r in 1 2; do
    for nv in 65536:0 65536:3 65536:2 131072:0 131072:16 131072:3; do
      timeout -k 10 200 python bench.py --envs ${nv%%:*} --variant ${nv##*:} $BQ \
        > $O/var_${nv%%:*}_${nv##*:}_$r.json 2>> $O/var.err || exit 1
    done
  done
  timeout -k 10 300 python tools/single_env_latency.py > $O/single_env_latency.json 2> $O/single_env_latency.err || exit 1
  ;;
kargs)  # one kernel-argument batch in k_step; straight-line multi-tile loads (vs HEAD = tick)
  timeout -k 10 600 $PYT -m gpu --maxfail=4 tests/test_gpu_step_multi.py tests/test_gpu_parity.py \
    tests/test_gpu_noise.py "tests/test_gpu_rk4.py::test_l3_rk4_step_vs_oracle" tests/test_gpu_resident.py \
    > $O/kargs_tests.txt 2>&1 || exit 1
  timeout -k 10 300 python tools/single_env_latency.py > $O/single_env_latency.json 2> $O/single_env_latency.err || exit 1
  for cfg in "--envs 131072" "--envs 65536" "--system pmsm --envs 1048576" "--system hr --envs 1048576" \
             "--envs 1048576" "--system pmsm --envs 262144"; do
    tag=$(echo $cfg | tr -d ' -')
    timeout -k 10 600 python tools/ab_libs.py 3 default ablib/libgym_lorenz_amd_tick.so \
      -- $cfg $BQ > $O/ab_$tag.json 2> $O/ab_$tag.err || exit 1
  done
  ;;
rt)  # the resident round trip taken apart; the per-system multi-tile load layouts
  timeout -k 10 120 tools/rt_probe 20000 > $O/rt_probe.txt 2>&1 || exit 1
  timeout -k 10 600 $PYT -m gpu --maxfail=4 tests/test_gpu_step_multi.py > $O/multi_tests.txt 2>&1 || exit 1
  for cfg in "--system pmsm --envs 1048576" "--system hr --envs 1048576"; do
    tag=$(echo $cfg | tr -d ' -')
    timeout -k 10 600 python tools/ab_libs.py 3 default ablib/libgym_lorenz_amd_tick.so \
      -- $cfg $BQ > $O/ab_$tag.json 2> $O/ab_$tag.err || exit 1
  done
  ;;
noise)  # how much of the PMSM / HR env rollout at cfg5's 32,768 envs is the process noise
  for sys in pmsm hr; do for nz in 1 0; do for n in 32768 65536; do
    timeout -k 10 200 python bench.py --system $sys --mode rollout --K 2048 --envs $n --steps 4096 --warmup 2048 \
      --add-noise $nz $BQ > $O/${sys}_${n}_noise$nz.json 2>> $O/noise.err || exit 1
  done; done; done
  ;;
np)  # the noise-producer wave of the one-wave PMSM / HR rollout: parity, then A/B
  timeout -k 10 600 $PYT -m gpu --maxfail=3 "tests/test_gpu_parity.py::test_rollout_noise_producer_equals_steps" \
    "tests/test_gpu_parity.py::test_rollout_equals_steps" tests/test_gpu_cfg5.py tests/test_gpu_noise.py \
    "tests/test_gpu_policy_branches.py::test_env_rollout_branch_reported" > $O/np_tests.txt 2>&1 || exit 1
  for r in 1 2; do for sys in pmsm hr; do for n in 32768 65536; do for v in 0 33554432; do
    timeout -k 10 200 python bench.py --system $sys --mode rollout --K 2048 --envs $n --steps 4096 --warmup 2048 \
      --add-noise 1 --variant $v $BQ > $O/${sys}_${n}_v${v}_$r.json 2>> $O/np.err || exit 1
  done; done; done; done
  ;;
l3multi)  # LORENZ3 f32 multi-tile step (E = 2 / 4, straight-line loads) vs k_step
  timeout -k 10 600 $PYT -m gpu --maxfail=3 tests/test_gpu_step_multi.py > $O/l3multi_tests.txt 2>&1 || exit 1
  for r in 1 2; do for n in 1048576 131072 2097152 4194304; do for v in 0 32768 49152; do
    timeout -k 10 200 python bench.py --envs $n --variant $v $BQ > $O/l3_${n}_v${v}_$r.json 2>> $O/l3multi.err || exit 1
  done; done; done
  ;;
f64ab)  # the fp64 extra line's k_step across the round's step-prologue changes
  timeout -k 10 600 python tools/ab_libs.py 3 default ablib/libgym_lorenz_amd_tick.so ablib/libgym_lorenz_amd_base.so \
    -- --dtype float64 $BQ > $O/ab_f64_1M.json 2> $O/ab_f64_1M.err || exit 1
  ;;
f64b)  # float64 back on round 3's step prologue (vs the float32 one), then the bench line
  timeout -k 10 600 python tools/ab_libs.py 3 default ablib/libgym_lorenz_amd_f64new.so ablib/libgym_lorenz_amd_base.so \
    -- --dtype float64 $BQ > $O/ab_f64_1M.json 2> $O/ab_f64_1M.err || exit 1
  timeout -k 10 600 $PYT -m gpu --maxfail=3 tests/test_gpu_parity.py tests/test_gpu_step_multi.py \
    > $O/f64b_tests.txt 2>&1 || exit 1
  timeout -k 10 400 python bench.py > $O/bench_default.json 2> $O/bench_default.err || exit 1
  ;;
l3window)  # LORENZ3 multi-tile: temporal done stores at 1M; the window edges (k_step forced = 16384)
  for r in 1 2; do
    for nv in 1048576:0 1048576:4194304 917504:0 917504:16384 786432:0 786432:49152 851968:0 851968:16384; do
      timeout -k 10 200 python bench.py --envs ${nv%%:*} --variant ${nv##*:} $BQ \
        > $O/w_${nv%%:*}_${nv##*:}_$r.json 2>> $O/w.err || exit 1
    done
  done
  ;;
phwindow)  # PMSM / HR multi-tile window edges: E = 4 (49152) vs k_step (16384)
  for r in 1 2; do for sys in pmsm hr; do for n in 786432 851968 917504; do for v in 16384 49152; do
    timeout -k 10 200 python bench.py --system $sys --envs $n --variant $v --steps 1000 --warmup 100 $BQ \
      > $O/w_${sys}_${n}_${v}_$r.json 2>> $O/w.err || exit 1
  done; done; done; done
  ;;
hrflat)  # HR's flag planes read without a branch: parity, then A/B vs HEAD's kernels
  timeout -k 10 900 $PYT -m gpu --maxfail=3 tests/test_gpu_step_multi.py tests/test_gpu_parity.py \
    tests/test_gpu_noise.py tests/test_gpu_wrappers.py tests/test_gpu_policy_attn_f32.py tests/test_gpu_resident.py \
    > $O/hrflat_tests.txt 2>&1 || exit 1
  for cfg in "--system hr --envs 1048576" "--system hr --envs 2097152" "--system hr --envs 262144" \
             "--system hr --mode rollout --K 2048 --envs 32768 --steps 4096 --warmup 2048"; do
    tag=$(echo $cfg | tr -d ' -')
    timeout -k 10 600 python tools/ab_libs.py 3 default ablib/libgym_lorenz_amd_head.so \
      -- $cfg $BQ > $O/ab_$tag.json 2> $O/ab_$tag.err || exit 1
  done
  ;;
pmc_hr)  # HR's multi-tile step after the branch-free flag-plane loads
  K=_ZN2lz12k_step_multiINS_5SysHRIfEEfLi4ELb0EEEvNS_5KArgsE
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 180 rocprofv3 --pmc $c -d $O/hr_$c -o run --output-format csv -- python bench.py \
      --system hr --envs 1048576 --launch eager --steps 256 --warmup 64 $BQ > $O/hr_$c.log 2>&1 || exit 1
  done
  python tools/pmc_generic.py $O/hr_FETCH_SIZE $O/hr_WRITE_SIZE $K "k_step_multi<lz::SysHR<float>, float, 4" 1048576 \
    89128960 $O/hr_multi_1M_pmc_summary.json || exit 1
  ;;
nobias)  # what PMSM's per-step Adam bias-table load costs (A/B lib gives WRONG results)
  for cfg in "--system pmsm --mode rollout --K 2048 --envs 32768 --steps 4096 --warmup 2048" \
             "--system pmsm --envs 262144" "--system pmsm --envs 1048576"; do
    tag=$(echo $cfg | tr -d ' -')
    timeout -k 10 600 python tools/ab_libs.py 3 default ablib/libgym_lorenz_amd_nobias.so \
      -- $cfg $BQ > $O/ab_$tag.json 2> $O/ab_$tag.err || exit 1
  done
  ;;
bias)  # PMSM fused rollout: the Adam bias pair carried by the action DMA ring (vs HEAD)
  timeout -k 10 900 $PYT -m gpu --maxfail=4 tests/test_gpu_parity.py tests/test_gpu_cfg5.py tests/test_gpu_noise.py \
    tests/test_gpu_step_multi.py tests/test_gpu_policy_branches.py > $O/bias_tests.txt 2>&1 || exit 1
  for cfg in "--system pmsm --mode rollout --K 2048 --envs 32768 --steps 4096 --warmup 2048" \
             "--system pmsm --mode rollout --K 2048 --envs 262144 --steps 4096 --warmup 2048"; do
    tag=$(echo $cfg | tr -d ' -')
    timeout -k 10 600 python tools/ab_libs.py 3 default ablib/libgym_lorenz_amd_head.so \
      -- $cfg $BQ > $O/ab_$tag.json 2> $O/ab_$tag.err || exit 1
  done
  ;;
div)  # PMSM: the Adam bias correction through the tabulated reciprocals (vs HEAD's divisions)
  timeout -k 10 900 $PYT -m gpu --maxfail=4 tests/test_gpu_parity.py tests/test_gpu_cfg5.py tests/test_gpu_noise.py \
    tests/test_gpu_step_multi.py tests/test_gpu_policy_branches.py tests/test_gpu_vecnorm_step.py \
    > $O/div_tests.txt 2>&1 || exit 1
  for cfg in "--system pmsm --mode rollout --K 2048 --envs 32768 --steps 4096 --warmup 2048" \
             "--system pmsm --envs 262144" "--system pmsm --envs 1048576" \
             "--mode vecnorm --system pmsm --envs 262144 --steps 512 --warmup 64"; do
    tag=$(echo $cfg | tr -d ' -')
    timeout -k 10 600 python tools/ab_libs.py 3 default ablib/libgym_lorenz_amd_head.so \
      -- $cfg $BQ > $O/ab_$tag.json 2> $O/ab_$tag.err || exit 1
  done
  ;;
fast)  # PMSM: the bias pair for the wave's first lane without a branch (waterfall only on mixed k)
  timeout -k 10 900 $PYT -m gpu --maxfail=4 tests/test_gpu_pmsm_adam_mixed.py tests/test_gpu_parity.py \
    tests/test_gpu_cfg5.py tests/test_gpu_noise.py tests/test_gpu_step_multi.py tests/test_gpu_policy_branches.py \
    tests/test_gpu_vecnorm_step.py tests/test_gpu_state_index.py > $O/fast_tests.txt 2>&1 || exit 1
  for cfg in "--system pmsm --mode rollout --K 2048 --envs 32768 --steps 4096 --warmup 2048" \
             "--system pmsm --envs 262144" "--system pmsm --envs 1048576" \
             "--mode vecnorm --system pmsm --envs 262144 --steps 512 --warmup 64"; do
    tag=$(echo $cfg | tr -d ' -')
    timeout -k 10 600 python tools/ab_libs.py 3 default ablib/libgym_lorenz_amd_head.so \
      -- $cfg $BQ > $O/ab_$tag.json 2> $O/ab_$tag.err || exit 1
  done
  ;;
fast2)  # PMSM: the bias pair loaded at the top of step() through a constant-space pointer (vs HEAD)
  timeout -k 10 900 $PYT -m gpu --maxfail=4 tests/test_gpu_pmsm_adam_mixed.py tests/test_gpu_parity.py \
    tests/test_gpu_cfg5.py tests/test_gpu_noise.py tests/test_gpu_step_multi.py tests/test_gpu_policy_branches.py \
    tests/test_gpu_vecnorm_step.py tests/test_gpu_state_index.py > $O/fast2_tests.txt 2>&1 || exit 1
  for cfg in "--system pmsm --mode rollout --K 2048 --envs 32768 --steps 4096 --warmup 2048" \
             "--system pmsm --mode rollout --K 2048 --envs 262144 --steps 4096 --warmup 2048" \
             "--system pmsm --envs 262144" "--system pmsm --envs 1048576" \
             "--mode vecnorm --system pmsm --envs 262144 --steps 512 --warmup 64"; do
    tag=$(echo $cfg | tr -d ' -')
    timeout -k 10 600 python tools/ab_libs.py 3 default ablib/libgym_lorenz_amd_fast1.so \
      -- $cfg $BQ > $O/ab_$tag.json 2> $O/ab_$tag.err || exit 1
  done
  ;;
scalartick)  # the scalar tick load (with the one-batch kernel arguments) vs the vector one
  for cfg in "--dtype float64" "--envs 131072" "--integrator rk4" "--envs 2097152"; do
    tag=$(echo $cfg | tr -d ' -')
    timeout -k 10 600 python tools/ab_libs.py 3 default ablib/libgym_lorenz_amd_scalartick.so ablib/libgym_lorenz_amd_base.so \
      -- $cfg $BQ > $O/ab_$tag.json 2> $O/ab_$tag.err || exit 1
  done
  ;;
new)
  timeout -k 10 1100 $PYT -m gpu --maxfail=8 tests/test_gpu_rk4.py tests/test_gpu_vecnorm_step.py \
    tests/test_gpu_resident.py tests/test_bench_contract.py tests/test_gpu_policy_branches.py \
    "tests/test_gpu_parity.py::test_l4_f32_vs_oracle_cfg2" \
    "tests/test_gpu_policy_attn_f32.py::test_attn_f32_reference_class_weights_bitexact" \
    > $O/new_tests.txt 2>&1
  ;;
full)
  timeout -k 10 1000 $PYT -x -m gpu tests > $O/gpu_tests.txt 2>&1 || exit 1
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('SMOKE OK')" > $O/smoke.txt 2>&1
  ;;
bench)
  timeout -k 10 400 python bench.py > $O/bench_default.json 2> $O/bench_default.err || exit 1
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 > $O/bench_steps20.json 2> $O/bench_steps20.err || exit 1
  timeout -k 10 200 python bench.py --integrator rk4 --no-cpu-baseline > $O/bench_rk4.json 2> $O/bench_rk4.err || exit 1
  LZ_BENCH_BACKEND=gloo timeout -k 10 300 python bench.py --gpus 2 > $O/bench_gpus2_gloo.json 2> $O/bench_gpus2_gloo.err
  ;;
esac
