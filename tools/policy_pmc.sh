#!/bin/bash
# PMC passes on the fused policy rollout (k_rollout_policy).  Counter-only runs (no
# trace domains besides the kernel trace), one pass per counter set.
#   bash tools/policy_pmc.sh [tag] [bench.py args...]   (default: PMSM 262,144 envs, K=16)
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-policy}
shift || true
ARGS=${*:-"--system pmsm --envs 262144 --K 16 --steps 512"}
B="python bench.py --mode policy $ARGS"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_prof -o run --output-format csv -- $B > gpurun_out/${TAG}_prof.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA -d gpurun_out/${TAG}_pmc1 -o p1 --output-format csv -- $B > gpurun_out/${TAG}_pmc1.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU_TRANS_F SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES SQ_VALU_MFMA_COEXEC_CYCLES SQ_INSTS_SALU GRBM_GUI_ACTIVE -d gpurun_out/${TAG}_pmc2 -o p2 --output-format csv -- $B > gpurun_out/${TAG}_pmc2.log 2>&1 || exit 1
