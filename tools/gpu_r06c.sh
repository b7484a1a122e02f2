#!/bin/bash
# r06 stage C: the whole GPU suite on the current tree; the pair kernel's crossover
# (16,384 / 32,768 / 49,152 envs, default vs forced / disabled); SQ counters of both PMSM
# rollout kernels at 32,768 x 2048 (one --pmc pass each).
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r06c
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests \
  > $O/gpu_tests.txt 2>&1 || { echo TESTS FAILED; grep -E "FAILED|Error" $O/gpu_tests.txt | head; tail -30 $O/gpu_tests.txt; exit 1; }
tail -3 $O/gpu_tests.txt
for rep in 1 2; do
  for n in 16384 32768 49152; do
    for v in 0 134217728 268435456; do
      timeout -k 10 120 python bench.py --system pmsm --mode rollout --envs $n --K 2048 --steps 8192 --variant $v \
        --no-cpu-baseline --no-drift --no-extras > $O/pmsm_${n}_v${v}_r${rep}.json 2> $O/pmsm_${n}_v${v}_r${rep}.err \
        || { echo BENCH FAILED $n $v; tail -5 $O/pmsm_${n}_v${v}_r${rep}.err; exit 1; }
      python -c "import json;d=json.load(open('$O/pmsm_${n}_v${v}_r${rep}.json'));print($n,$v,'%.3e'%d['value'],'launch_us %.1f'%d['roofline']['avg_launch_us'],d['roofline']['kernel'][:40])"
    done
  done
done
cd /tmp && export TMPDIR=/tmp
for v in 268435456 0; do
  timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY \
    -d $GRAFT_REPO_ROOT/$O/pmc_v$v -o pmc --output-format csv -- \
    python3 $GRAFT_REPO_ROOT/bench.py --system pmsm --mode rollout --envs 32768 --K 2048 --steps 4096 --variant $v \
    --no-cpu-baseline --no-drift --no-extras > $GRAFT_REPO_ROOT/$O/pmc_v$v.json 2> $GRAFT_REPO_ROOT/$O/pmc_v$v.err \
    || { echo PMC FAILED; tail -5 $GRAFT_REPO_ROOT/$O/pmc_v$v.err; exit 1; }
done
echo done
