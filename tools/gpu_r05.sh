#!/bin/bash
# Round 5 GPU runs.  usage: tools/gpu_r05.sh <stage> [out-dir]
#   new   : the round's new / changed GPU tests (default step launches at their selecting
#           sizes, step-after-close, step_multi injected-noise cases, resident server)
#   full  : every -m gpu test + smoke()
#   bench : default bench line, the driver's --steps 20, and the 2-rank self-spawned
#           launcher over gloo on this one GPU (cfg3's strong split + gather accounting)
set -o pipefail
export TMPDIR=/tmp
STAGE=${1:-new}
O=${2:-gpurun_out/r05_$STAGE}
mkdir -p $O
PYT="python -u -m pytest -v --timeout 170 --timeout-method thread -p no:cacheprovider"
BQ="--no-cpu-baseline --no-drift --no-extras"
case $STAGE in
new)
  timeout -k 10 900 $PYT -m gpu --maxfail=8 tests/test_gpu_default_launch.py tests/test_gpu_step_multi.py \
    tests/test_gpu_resident.py tests/test_gpu_policy_branches.py > $O/new_tests.txt 2>&1 || exit 1
  LZ_BENCH_BACKEND=gloo timeout -k 10 300 python bench.py --gpus 2 > $O/bench_gpus2_gloo.json 2> $O/bench_gpus2_gloo.err
  ;;
ic)  # the headline state's reuse distance: bench.py as is (warm) vs a 2 x 192 MiB copy after every step (cold)
  for r in 1 2; do for m in 0 192; do
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/f${m}_$r -o run --output-format csv \
      -- python bench.py --ic-flush-mib $m --steps 2000 --warmup 100 $BQ > $O/f${m}_$r.json 2> $O/f${m}_$r.err || exit 1
  done; done
  ;;
diag)  # graph replays of lz_step: eager, k_step graph, then the default (k_step_multi) graph
  timeout -k 10 200 python bench.py --launch eager $BQ > $O/eager.json 2> $O/eager.err || exit 1
  timeout -k 10 200 python bench.py --variant 16384 $BQ > $O/kstep_graph.json 2> $O/kstep_graph.err || exit 1
  timeout -k 10 200 python bench.py $BQ > $O/default.json 2> $O/default.err || exit 1
  ;;
i8)  # the default bench path first, then the i8x4 attention policies: parity, then A/B vs fp32
  timeout -k 10 200 python bench.py $BQ > $O/default.json 2> $O/default.err || exit 1
  timeout -k 10 900 $PYT -m gpu --maxfail=6 tests/test_gpu_policy_i8x4.py > $O/i8_tests.txt 2>&1 || exit 1
  PB="--mode policy --system hr --envs 32768 --K 2048 --steps 4096 $BQ"
  for r in 1 2; do for pr in fp32 i8x4; do for po in attn attn_ln; do
    timeout -k 10 300 python bench.py $PB --policy $po --precision $pr > $O/${po}_${pr}_$r.json 2>> $O/bench.err || exit 1
  done; done; done
  ;;
pmc_i8)  # SQ issue / co-execution counters of the attention rollout: fp32 vs i8x4
  for pr in fp32 i8x4; do
    bash tools/policy_pmc.sh r05_attn_$pr --policy attn --precision $pr --system hr --envs 32768 --K 2048 --steps 4096 $BQ || exit 1
  done
  ;;
r2)  # i8x4 after the shared feature digits + pipelined layer 2: parity, A/B, counters; IC read-only flush
  timeout -k 10 900 $PYT -m gpu --maxfail=6 tests/test_gpu_policy_i8x4.py > $O/i8_tests.txt 2>&1 || exit 1
  PB="--mode policy --system hr --envs 32768 --K 2048 --steps 4096 $BQ"
  for r in 1 2; do for pr in fp32 i8x4; do for po in attn attn_ln; do
    timeout -k 10 300 python bench.py $PB --policy $po --precision $pr > $O/${po}_${pr}_$r.json 2>> $O/bench.err || exit 1
  done; done; done
  for r in 1 2; do
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/read192_$r -o run --output-format csv \
      -- python bench.py --ic-flush-mib 192 --ic-flush-kind read --steps 2000 --warmup 100 $BQ > $O/read192_$r.json 2> $O/read192_$r.err || exit 1
  done
  bash tools/policy_pmc.sh r05_attn_i8x4 --policy attn --precision i8x4 --system hr --envs 32768 --K 2048 --steps 4096 $BQ || exit 1
  bash tools/policy_pmc.sh r05_attn_fp32 --policy attn --precision fp32 --system hr --envs 32768 --K 2048 --steps 4096 $BQ || exit 1
  ;;
r3)  # IC read-only flush; SQ counters of the attention rollout (fp32 vs i8x4)
  for r in 1 2; do
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/read192_$r -o run --output-format csv \
      -- python bench.py --ic-flush-mib 192 --ic-flush-kind read --steps 2000 --warmup 100 $BQ > $O/read192_$r.json 2> $O/read192_$r.err || exit 1
  done
  bash tools/policy_pmc.sh r05_attn_i8x4 --policy attn --precision i8x4 --system hr --envs 32768 --K 2048 --steps 4096 $BQ || exit 1
  bash tools/policy_pmc.sh r05_attn_fp32 --policy attn --precision fp32 --system hr --envs 32768 --K 2048 --steps 4096 $BQ || exit 1
  ;;
r4)  # i8x4 with post_attention_fc on the int8 MFMA: parity, A/B vs fp32 and vs the r2 build; IC read flush; counters
  timeout -k 10 900 $PYT -m gpu --maxfail=6 tests/test_gpu_policy_i8x4.py > $O/i8_tests.txt 2>&1 || exit 1
  PB="--mode policy --system hr --envs 32768 --K 2048 --steps 4096 $BQ"
  for r in 1 2; do for pr in fp32 i8x4; do for po in attn attn_ln; do
    timeout -k 10 300 python bench.py $PB --policy $po --precision $pr > $O/${po}_${pr}_$r.json 2>> $O/bench.err || exit 1
  done; done; done
  timeout -k 10 900 python tools/ab_libs.py 2 default ablib/libgym_lorenz_amd_i8nopipe.so -- $PB --policy attn \
    --precision i8x4 > $O/ab_i8_nopipe.json 2> $O/ab_i8_nopipe.err || exit 1
  for r in 1 2; do
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/read192_$r -o run --output-format csv \
      -- python bench.py --ic-flush-mib 192 --ic-flush-kind read --steps 2000 --warmup 100 $BQ > $O/read192_$r.json 2> $O/read192_$r.err || exit 1
  done
  bash tools/policy_pmc.sh r05_attn_i8x4 --policy attn --precision i8x4 --system hr --envs 32768 --K 2048 --steps 4096 $BQ || exit 1
  bash tools/policy_pmc.sh r05_attn_fp32 --policy attn --precision fp32 --system hr --envs 32768 --K 2048 --steps 4096 $BQ || exit 1
  ;;
mlp)  # i8x4 MlpPolicy: parity, then fp32 vs i8x4 at cfg5's 32,768 envs (split kernel) and at 1M (8 / 4 waves)
  timeout -k 10 900 $PYT -m gpu --maxfail=5 tests/test_gpu_policy_mlp_i8x4.py tests/test_gpu_policy_f32.py \
    "tests/test_gpu_policy_i8x4.py::test_i8x4_flag_refused_elsewhere" > $O/mlp_tests.txt 2>&1 || exit 1
  PB="--mode policy --system pmsm --vecnorm-update rollout $BQ"
  for r in 1 2; do for p in fp32 i8x4; do
    timeout -k 10 200 python bench.py $PB --envs 32768 --K 2048 --steps 4096 --precision $p > $O/mlp32k_${p}_$r.json 2>> $O/bench.err || exit 1
    timeout -k 10 200 python bench.py $PB --envs 1048576 --K 64 --steps 256 --precision $p > $O/mlp1m_${p}_$r.json 2>> $O/bench.err || exit 1
    LZ_POL_F32_WAVES=4 timeout -k 10 200 python bench.py $PB --envs 1048576 --K 64 --steps 256 --precision $p > $O/mlp1m_w4_${p}_$r.json 2>> $O/bench.err || exit 1
  done; done
  ;;
ab2)  # two-pass MLP i8x4 tail + NaN at the attention heads (default) vs the r05a build
  timeout -k 10 900 $PYT -m gpu --maxfail=5 tests/test_gpu_policy_mlp_i8x4.py tests/test_gpu_policy_i8x4.py \
    > $O/tests.txt 2>&1 || exit 1
  PB="--mode policy --system pmsm --vecnorm-update rollout --precision i8x4 $BQ"
  timeout -k 10 900 python tools/ab_libs.py 2 default ablib/libgym_lorenz_amd_r05a.so -- $PB --envs 32768 --K 2048 \
    --steps 4096 > $O/mlp32k.json 2> $O/mlp32k.err || exit 1
  timeout -k 10 900 python tools/ab_libs.py 2 default ablib/libgym_lorenz_amd_r05a.so -- $PB --envs 1048576 --K 64 \
    --steps 256 > $O/mlp1m.json 2> $O/mlp1m.err || exit 1
  timeout -k 10 900 python tools/ab_libs.py 2 default ablib/libgym_lorenz_amd_r05a.so -- --mode policy --system hr \
    --envs 32768 --K 2048 --steps 4096 --policy attn --precision i8x4 $BQ > $O/attn.json 2> $O/attn.err || exit 1
  ;;
ab3)  # MLP i8x4 tail with hi / lo accumulated directly (two accumulators, shift between passes) vs r05a
  timeout -k 10 900 $PYT -m gpu --maxfail=5 tests/test_gpu_policy_mlp_i8x4.py tests/test_gpu_policy_f32.py \
    > $O/tests.txt 2>&1 || exit 1
  PB="--mode policy --system pmsm --vecnorm-update rollout --precision i8x4 $BQ"
  timeout -k 10 900 python tools/ab_libs.py 2 default ablib/libgym_lorenz_amd_r05a.so -- $PB --envs 32768 --K 2048 \
    --steps 4096 > $O/mlp32k.json 2> $O/mlp32k.err || exit 1
  timeout -k 10 900 python tools/ab_libs.py 2 default ablib/libgym_lorenz_amd_r05a.so -- $PB --envs 1048576 --K 64 \
    --steps 256 > $O/mlp1m.json 2> $O/mlp1m.err || exit 1
  timeout -k 10 900 python tools/ab_libs.py 2 default ablib/libgym_lorenz_amd_r05a.so -- --mode policy --system hr \
    --envs 32768 --K 2048 --steps 4096 --vecnorm-update rollout --precision i8x4 $BQ > $O/mlp_hr32k.json 2> $O/mlp_hr32k.err || exit 1
  ;;
ab4)  # lz_policy.o built with MachineLICM sinking (fewer spills) vs the r05b build, every policy path
  timeout -k 10 1000 $PYT -m gpu --maxfail=5 tests/test_gpu_policy*.py > $O/tests.txt 2>&1 || exit 1
  AB="timeout -k 10 600 python tools/ab_libs.py 1 default ablib/libgym_lorenz_amd_r05b.so --"
  P="--mode policy $BQ"
  $AB $P --system pmsm --envs 32768 --K 2048 --steps 4096 --vecnorm-update rollout > $O/mlp_f32_32k.json 2>> $O/ab.err || exit 1
  $AB $P --system pmsm --envs 1048576 --K 64 --steps 256 --vecnorm-update rollout > $O/mlp_f32_1m.json 2>> $O/ab.err || exit 1
  $AB $P --system pmsm --envs 32768 --K 2048 --steps 4096 --vecnorm-update rollout --precision i8x4 > $O/mlp_i8_32k.json 2>> $O/ab.err || exit 1
  $AB $P --system pmsm --envs 1048576 --K 64 --steps 256 --vecnorm-update rollout --precision i8x4 > $O/mlp_i8_1m.json 2>> $O/ab.err || exit 1
  $AB $P --system pmsm --envs 262144 --K 16 --steps 512 > $O/mlp_f32_vnstep_262k.json 2>> $O/ab.err || exit 1
  $AB $P --system hr --envs 32768 --K 2048 --steps 4096 --policy attn > $O/attn_f32_hr.json 2>> $O/ab.err || exit 1
  $AB $P --system hr --envs 32768 --K 2048 --steps 4096 --policy attn --precision i8x4 > $O/attn_i8_hr.json 2>> $O/ab.err || exit 1
  $AB $P --system hr --envs 32768 --K 2048 --steps 4096 --policy attn_ln > $O/attn_ln_f32_hr.json 2>> $O/ab.err || exit 1
  $AB $P --system pmsm --envs 32768 --K 2048 --steps 4096 --precision bf16 > $O/mlp_bf16_32k.json 2>> $O/ab.err || exit 1
  ;;
ab5)  # tanh_tab: clamp into a constant-1 segment (11 VALU) + 4-wide batched coefficient reads in the attention nets, vs r05c
  timeout -k 10 1000 $PYT -m gpu --maxfail=5 tests/test_gpu_policy*.py > $O/tests.txt 2>&1 || exit 1
  AB="timeout -k 10 600 python tools/ab_libs.py 2 default ablib/libgym_lorenz_amd_r05c.so --"
  P="--mode policy $BQ --envs 32768 --K 2048 --steps 4096"
  $AB $P --system hr --policy attn > $O/attn_f32_hr.json 2>> $O/ab.err || exit 1
  $AB $P --system hr --policy attn --precision i8x4 > $O/attn_i8_hr.json 2>> $O/ab.err || exit 1
  $AB $P --system hr --policy attn_ln > $O/attn_ln_f32_hr.json 2>> $O/ab.err || exit 1
  $AB $P --system hr --policy attn_ln --precision i8x4 > $O/attn_ln_i8_hr.json 2>> $O/ab.err || exit 1
  $AB $P --system pmsm --vecnorm-update rollout > $O/mlp_f32_32k.json 2>> $O/ab.err || exit 1
  $AB $P --system pmsm --vecnorm-update rollout --precision i8x4 > $O/mlp_i8_32k.json 2>> $O/ab.err || exit 1
  ;;
ab6)  # MLP i8x4 recombine as fma(t, packed float row scale, bias) vs r05d
  timeout -k 10 900 $PYT -m gpu --maxfail=5 tests/test_gpu_policy_mlp_i8x4.py tests/test_gpu_policy_f32.py > $O/tests.txt 2>&1 || exit 1
  AB="timeout -k 10 600 python tools/ab_libs.py 2 default ablib/libgym_lorenz_amd_r05d.so --"
  P="--mode policy $BQ --vecnorm-update rollout --precision i8x4"
  $AB $P --system pmsm --envs 32768 --K 2048 --steps 4096 > $O/mlp_i8_32k.json 2>> $O/ab.err || exit 1
  $AB $P --system pmsm --envs 1048576 --K 64 --steps 256 > $O/mlp_i8_1m.json 2>> $O/ab.err || exit 1
  $AB $P --system hr --envs 32768 --K 2048 --steps 4096 > $O/mlp_i8_hr32k.json 2>> $O/ab.err || exit 1
  ;;
ab7)  # MLP i8x4 tail software-pipelined (tile t + 1's MFMA passes around tile t's VALU work) vs r05d
  timeout -k 10 900 $PYT -m gpu --maxfail=5 tests/test_gpu_policy_mlp_i8x4.py > $O/tests.txt 2>&1 || exit 1
  AB="timeout -k 10 600 python tools/ab_libs.py 2 default ablib/libgym_lorenz_amd_r05d.so --"
  P="--mode policy $BQ --vecnorm-update rollout --precision i8x4"
  $AB $P --system pmsm --envs 32768 --K 2048 --steps 4096 > $O/mlp_i8_32k.json 2>> $O/ab.err || exit 1
  $AB $P --system pmsm --envs 1048576 --K 64 --steps 256 > $O/mlp_i8_1m.json 2>> $O/ab.err || exit 1
  $AB $P --system hr --envs 32768 --K 2048 --steps 4096 > $O/mlp_i8_hr32k.json 2>> $O/ab.err || exit 1
  LZ_POL_F32_WAVES=4 $AB $P --system pmsm --envs 1048576 --K 64 --steps 256 > $O/mlp_i8_1m_w4.json 2>> $O/ab.err || exit 1
  ;;
ab8)  # attention i8x4 layer 1 software-pipelined (tile t + 1's MFMAs before tile t's VALU) vs r05d
  timeout -k 10 900 $PYT -m gpu --maxfail=5 tests/test_gpu_policy_i8x4.py tests/test_gpu_policy_mlp_i8x4.py > $O/tests.txt 2>&1 || exit 1
  AB="timeout -k 10 600 python tools/ab_libs.py 2 default ablib/libgym_lorenz_amd_r05d.so --"
  P="--mode policy $BQ --envs 32768 --K 2048 --steps 4096 --precision i8x4"
  $AB $P --system hr --policy attn > $O/attn_i8_hr.json 2>> $O/ab.err || exit 1
  $AB $P --system hr --policy attn_ln > $O/attn_ln_i8_hr.json 2>> $O/ab.err || exit 1
  $AB $P --system pmsm --vecnorm-update rollout > $O/mlp_i8_32k.json 2>> $O/ab.err || exit 1
  ;;
final)  # the closing run on the final tree: every GPU test, smoke, the bench lines and the headline's rocprof summary
  timeout -k 10 1000 $PYT -x -m gpu tests > $O/gpu_tests.txt 2>&1 || exit 1
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('SMOKE OK')" > $O/smoke.txt 2>&1 || exit 1
  timeout -k 10 400 python bench.py > $O/bench_default.json 2> $O/bench_default.err || exit 1
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 > $O/bench_steps20.json 2> $O/bench_steps20.err || exit 1
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv \
    -- python bench.py --no-cpu-baseline --no-drift > $O/bench_prof.json 2> $O/bench_prof.err || exit 1
  ;;
ab9)  # attention i8x4 row shifts as per-value ds_read_i16 (no VALU unpack) vs r05d
  timeout -k 10 900 $PYT -m gpu --maxfail=5 tests/test_gpu_policy_i8x4.py > $O/tests.txt 2>&1 || exit 1
  AB="timeout -k 10 600 python tools/ab_libs.py 2 default ablib/libgym_lorenz_amd_r05d.so --"
  P="--mode policy $BQ --envs 32768 --K 2048 --steps 4096 --precision i8x4 --system hr"
  $AB $P --policy attn > $O/attn_i8_hr.json 2>> $O/ab.err || exit 1
  $AB $P --policy attn_ln > $O/attn_ln_i8_hr.json 2>> $O/ab.err || exit 1
  ;;
pmc_mlp)  # counters of the MlpPolicy rollout, float32 vs i8x4 (PMSM 32,768 x 2048)
  bash tools/policy_pmc.sh r05_mlp_i8x4 --system pmsm --envs 32768 --K 2048 --steps 4096 --vecnorm-update rollout --precision i8x4 $BQ || exit 1
  bash tools/policy_pmc.sh r05_mlp_fp32 --system pmsm --envs 32768 --K 2048 --steps 4096 --vecnorm-update rollout --precision fp32 $BQ || exit 1
  ;;
dist)  # the driver's N > 1 launch path on this 1-GPU box: torchrun + RCCL at world size 1, and the
       # refusal of more nccl ranks than GPUs (must exit non-zero, not share the card)
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
    --master-port 29517 bench.py --gpus 1 --steps 400 --warmup 40 > $O/torchrun_n1.json 2> $O/torchrun_n1.err || exit 1
  if timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29518 bench.py --gpus 2 --steps 400 --warmup 40 > $O/torchrun_n2.json 2> $O/torchrun_n2.err; then
    echo "UNEXPECTED: 2 nccl ranks on 1 GPU ran" > $O/refusal.txt; exit 1
  else
    echo "refused as intended (exit $?)" > $O/refusal.txt
  fi
  ;;
ab10)  # attention softmax: NaN-propagating v_maximum for the max, no NaN select in exp_att, vs r05e
  timeout -k 10 900 $PYT -m gpu --maxfail=5 tests/test_gpu_policy_attn_f32.py tests/test_gpu_policy_i8x4.py \
    tests/test_gpu_policy_branches.py tests/test_gpu_policy_edges.py > $O/tests.txt 2>&1 || exit 1
  AB="timeout -k 10 600 python tools/ab_libs.py 2 default ablib/libgym_lorenz_amd_r05e.so --"
  P="--mode policy $BQ --envs 32768 --K 2048 --steps 4096 --system hr"
  $AB $P --policy attn > $O/attn_f32_hr.json 2>> $O/ab.err || exit 1
  $AB $P --policy attn --precision i8x4 > $O/attn_i8_hr.json 2>> $O/ab.err || exit 1
  $AB $P --policy attn_ln > $O/attn_ln_f32_hr.json 2>> $O/ab.err || exit 1
  $AB $P --policy attn_ln --precision i8x4 > $O/attn_ln_i8_hr.json 2>> $O/ab.err || exit 1
  ;;
table)  # the DESIGN §6.3 table at HEAD (every row one r05 file)
  R="timeout -k 10 300 python bench.py $BQ"
  $R --envs 65536 > $O/cfg3_step_65536.json 2>> $O/table.err || exit 1
  $R --envs 131072 > $O/cfg3_step_131072.json 2>> $O/table.err || exit 1
  $R --mode rollout --K 2048 --envs 32768 --steps 8192 > $O/cfg5_rollout_l3.json 2>> $O/table.err || exit 1
  $R --mode rollout --system hr --K 2048 --envs 32768 --steps 4096 --warmup 2048 > $O/cfg5_rollout_hr.json 2>> $O/table.err || exit 1
  $R --mode vecnorm --system pmsm --envs 262144 --steps 512 > $O/vecnorm_pmsm262k.json 2>> $O/table.err || exit 1
  $R --mode policy --system pmsm --envs 262144 --K 16 --steps 512 > $O/mlp_f32_vnstep_pmsm262k.json 2>> $O/table.err || exit 1
  $R --mode policy --system pmsm --envs 32768 --K 2048 --steps 4096 --precision bf16 > $O/mlp_bf16_pmsm32k.json 2>> $O/table.err || exit 1
  $R --mode policy --system hr --envs 32768 --K 2048 --steps 4096 --policy attn --precision bf16 > $O/attn_bf16_hr32k.json 2>> $O/table.err || exit 1
  $R --mode policy --system hr --envs 32768 --K 2048 --steps 4096 --policy attn_ln --precision bf16 > $O/attn_ln_bf16_hr32k.json 2>> $O/table.err || exit 1
  timeout -k 10 300 python tools/frame_stack_bench.py > $O/frame_stack_hr1m.json 2>> $O/table.err || exit 1
  timeout -k 10 300 python tools/resident_latency.py > $O/resident_latency.json 2>> $O/table.err || exit 1
  ;;
zpmc)  # counters of the rejected kZN noise pipelining (variant 1<<26) vs the default, PMSM 32,768 x 2048
  for v in 0 67108864; do
    B="python bench.py --system pmsm --mode rollout --K 2048 --envs 32768 --steps 4096 --warmup 2048 --add-noise 1 --variant $v $BQ"
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/v${v}_prof -o run --output-format csv -- $B > $O/v${v}_prof.log 2>&1 || exit 1
    timeout -k 10 200 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_BUSY_CYCLES \
      -d $O/v${v}_pmc1 -o p1 --output-format csv -- $B > $O/v${v}_pmc1.log 2>&1 || exit 1
    timeout -k 10 200 rocprofv3 --pmc SQ_INSTS_VALU_TRANS_F SQ_ACTIVE_INST_VMEM SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INST_LEVEL_VMEM GRBM_GUI_ACTIVE \
      -d $O/v${v}_pmc2 -o p2 --output-format csv -- $B > $O/v${v}_pmc2.log 2>&1 || exit 1
  done
  ;;
zn)  # software-pipelined noise draws in the PMSM / HR rollouts (variant 1<<26): parity, then A/B
  timeout -k 10 600 $PYT -m gpu --maxfail=3 "tests/test_gpu_parity.py::test_rollout_noise_producer_equals_steps" \
    > $O/zn_tests.txt 2>&1 || exit 1
  for r in 1 2 3; do for sys in pmsm hr; do for n in 32768 4097 65536; do for v in 0 67108864; do
    timeout -k 10 200 python bench.py --system $sys --mode rollout --K 2048 --envs $n --steps 4096 --warmup 2048 \
      --add-noise 1 --variant $v $BQ > $O/${sys}_${n}_v${v}_$r.json 2>> $O/zn.err || exit 1
  done; done; done; done
  ;;
full)
  timeout -k 10 1000 $PYT -x -m gpu tests > $O/gpu_tests.txt 2>&1 || exit 1
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('SMOKE OK')" > $O/smoke.txt 2>&1
  ;;
bench)
  timeout -k 10 400 python bench.py > $O/bench_default.json 2> $O/bench_default.err || exit 1
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 > $O/bench_steps20.json 2> $O/bench_steps20.err || exit 1
  ;;
bench_all)
  timeout -k 10 400 python bench.py > $O/bench_default.json 2> $O/bench_default.err || exit 1
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 > $O/bench_steps20.json 2> $O/bench_steps20.err || exit 1
  LZ_BENCH_BACKEND=gloo timeout -k 10 300 python bench.py --gpus 2 > $O/bench_gpus2_gloo.json 2> $O/bench_gpus2_gloo.err
  ;;
esac
