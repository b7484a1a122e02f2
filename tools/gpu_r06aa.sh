#!/bin/bash
# r06 stage AA: SQ counters of the PMSM rollout at 65,536 (one wave per SIMD) and 262,144
# envs (four per SIMD, configs[3] as a rollout) -- what bounds the 262,144 launch.
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r06aa
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for n in 65536 262144; do
  timeout -s KILL 150 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY \
    -d $GRAFT_REPO_ROOT/$O/pmsm_$n -o pmc --output-format csv -- \
    python3 $GRAFT_REPO_ROOT/bench.py --system pmsm --mode rollout --envs $n --K 2048 --steps 4096 \
    --no-cpu-baseline --no-drift --no-extras > $GRAFT_REPO_ROOT/$O/pmsm_$n.json 2> $GRAFT_REPO_ROOT/$O/pmsm_$n.err \
    || { echo PMC FAILED; tail -5 $GRAFT_REPO_ROOT/$O/pmsm_$n.err; exit 1; }
  echo $n ok
done
echo done
