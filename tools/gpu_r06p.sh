#!/bin/bash
# r06 stage P: HBM traffic of the final build's lane-pair PMSM rollout (32,768 x 2048).
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r06p
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $c -d $R/$O/pmsm_pair_$c -o run --output-format csv -- \
    python3 $R/bench.py --system pmsm --mode rollout --envs 32768 --K 2048 --steps 4096 --no-cpu-baseline --no-drift --no-extras \
    > $R/$O/pmsm_pair_$c.log 2>&1 || { echo PMC FAILED; tail -3 $R/$O/pmsm_pair_$c.log; exit 1; }
done
echo done
