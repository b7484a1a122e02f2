#!/bin/bash
# Round-2 PMC for the fused VecNormalize step (PMSM 262,144 envs): HBM bytes per launch
# of k_step_vn and k_vn_apply from separate FETCH_SIZE / WRITE_SIZE passes.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/pmc_vn
mkdir -p $O
ARGS="--mode vecnorm --system pmsm --envs 262144 --steps 512 --warmup 64 --no-cpu-baseline --no-drift --no-extras"
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 180 rocprofv3 --pmc $c -d $O/vn.$c -o run --output-format csv -- python bench.py $ARGS > $O/vn.$c.log 2>&1 || exit 1
done
python tools/pmc_generic.py $O/vn.FETCH_SIZE $O/vn.WRITE_SIZE _ZN2lz9k_step_vnINS_7SysPMSMEfLi24EEEvNS_5KArgsENS_5VArgsE "k_step_vn<lz::SysPMSM, float, 24>" 262144 36962304 $O/step_vn_pmc_summary.json || exit 1
python tools/pmc_generic.py $O/vn.FETCH_SIZE $O/vn.WRITE_SIZE _ZN12_GLOBAL__N_110k_vn_applyIfLi6ELb1EEEvNS_11VnApplyArgsE "k_vn_apply<float, 6, true>" 262144 15204352 $O/vn_apply_pmc_summary.json || exit 1
timeout -k 10 200 python bench.py $ARGS > $O/bench_line.json 2> $O/bench_line.err || exit 1
