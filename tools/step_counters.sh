#!/bin/bash
# Round-3 re-measurement of the two per-step kernels BASELINE names that are not
# launch-bound (VERDICT r02 "next" 6): cfg4 (PMSM 262,144 envs, process noise, alpha 0.5)
# and HR RK4 at 1,048,576 envs.  Per config: the bench line, a kernel trace with --stats,
# FETCH_SIZE and WRITE_SIZE in separate passes, and two SQ passes (issue / wait split,
# instruction mix).  Counter-only runs: no trace domain besides the kernel trace.
#   bash tools/step_counters.sh            -> gpurun_out/r03_step/
set -u
export TMPDIR=/tmp
O=gpurun_out/r03_step
mkdir -p $O
run() {  # run <tag> <bench args...>
  local tag=$1; shift
  local B="python bench.py $* --no-cpu-baseline --no-drift --no-extras"
  timeout -k 10 240 $B > $O/$tag.bench.json 2> $O/$tag.bench.log || return 1
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/$tag.trace -o run --output-format csv -- $B > $O/$tag.trace.log 2>&1 || return 1
  timeout -k 10 240 rocprofv3 --pmc FETCH_SIZE -d $O/$tag.FETCH_SIZE -o run --output-format csv -- $B > $O/$tag.fetch.log 2>&1 || return 1
  timeout -k 10 240 rocprofv3 --pmc WRITE_SIZE -d $O/$tag.WRITE_SIZE -o run --output-format csv -- $B > $O/$tag.write.log 2>&1 || return 1
  timeout -k 10 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_BUSY_CYCLES -d $O/$tag.sq1 -o run --output-format csv -- $B > $O/$tag.sq1.log 2>&1 || return 1
  timeout -k 10 240 rocprofv3 --pmc SQ_INSTS_VALU_TRANS_F SQ_INSTS_LDS SQ_WAVES GRBM_GUI_ACTIVE -d $O/$tag.sq2 -o run --output-format csv -- $B > $O/$tag.sq2.log 2>&1 || return 1
}
run cfg4_pmsm_262k --system pmsm --envs 262144 --steps 512 --warmup 64 --launch eager || exit 1
run hr_1M --system hr --envs 1048576 --steps 256 --warmup 64 --launch eager || exit 1
