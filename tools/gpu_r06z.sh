#!/bin/bash
# r06 stage Z: HBM traffic (rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, separate passes) of
# the BASELINE config lines that had none: LORENZ4 65,536 step and rollout, LORENZ3
# 262,144 step (one tile), PMSM 262,144 rollout, LORENZ3 / HR 32,768 rollouts.
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r06z
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
Q="--no-cpu-baseline --no-drift --no-extras"
run() {
  local tag=$1; shift
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 150 rocprofv3 --pmc $c -d $R/$O/${tag}_$c -o run --output-format csv -- \
      python3 $R/bench.py $Q "$@" > $R/$O/${tag}_$c.log 2>&1 || { echo PMC FAILED $tag $c; tail -3 $R/$O/${tag}_$c.log; exit 1; }
  done
  echo $tag ok
}
run l4_65536_step --system lorenz4 --envs 65536 --steps 2000 --warmup 100
run l4_65536_rollout --system lorenz4 --envs 65536 --mode rollout --K 2048 --steps 4096
run l3_262144_step --system lorenz3 --envs 262144 --steps 2000 --warmup 100
run pmsm_262144_rollout --system pmsm --envs 262144 --mode rollout --K 2048 --steps 4096
run l3_32768_rollout --system lorenz3 --envs 32768 --mode rollout --K 2048 --steps 4096
run hr_32768_rollout --system hr --envs 32768 --mode rollout --K 2048 --steps 4096
echo done
