#!/bin/bash
# PMC passes on the fused action-driven rollout (k_rollout), cfg5: LORENZ3, 32,768 envs,
# K=2048.  Counter-only runs, one pass per counter set.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
B="python bench.py --mode rollout --K 2048 --envs 32768 --steps 8192 --no-cpu-baseline --no-drift"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/roll_prof -o run --output-format csv -- $B > gpurun_out/roll_prof.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD -d gpurun_out/roll_pmc1 -o p1 --output-format csv -- $B > gpurun_out/roll_pmc1.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_INSTS_SALU GRBM_GUI_ACTIVE SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_INST_LEVEL_VMEM -d gpurun_out/roll_pmc2 -o p2 --output-format csv -- $B > gpurun_out/roll_pmc2.log 2>&1 || exit 1
