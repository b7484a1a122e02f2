#!/bin/bash
# r06 stage B: the lane-pair PMSM rollout -- parity tests, then an interleaved A/B of the
# default one-wave / 256-lane kernel vs the pair kernel (variant 1<<27), K = 2048, noise on,
# at 32,768 (cfg5's per-GPU shard) .. 262,144 envs; kernel stats of both at 32,768.
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r06b
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread \
  tests/test_gpu_rollout_pair.py > $O/tests.txt 2>&1 || { echo TESTS FAILED; tail -40 $O/tests.txt; exit 1; }
tail -3 $O/tests.txt
for rep in 1 2 3; do
  for n in 32768 65536 131072 262144; do
    for v in 0 134217728; do
      timeout -k 10 120 python bench.py --system pmsm --mode rollout --envs $n --K 2048 --steps 8192 --variant $v \
        --no-cpu-baseline --no-drift --no-extras > $O/pmsm_${n}_v${v}_r${rep}.json 2> $O/pmsm_${n}_v${v}_r${rep}.err \
        || { echo BENCH FAILED $n $v; tail -5 $O/pmsm_${n}_v${v}_r${rep}.err; exit 1; }
      python -c "import json;d=json.load(open('$O/pmsm_${n}_v${v}_r${rep}.json'));print($n,$v,'%.3e'%d['value'],'launch_us %.1f'%d['roofline']['avg_launch_us'])"
    done
  done
done
cd /tmp && export TMPDIR=/tmp
for v in 0 134217728; do
  timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof_v$v -o prof --output-format csv -- \
    python3 $GRAFT_REPO_ROOT/bench.py --system pmsm --mode rollout --envs 32768 --K 2048 --steps 8192 --variant $v \
    --no-cpu-baseline --no-drift --no-extras > $GRAFT_REPO_ROOT/$O/prof_v$v.json 2> $GRAFT_REPO_ROOT/$O/prof_v$v.err \
    || { echo PROF FAILED; tail -5 $GRAFT_REPO_ROOT/$O/prof_v$v.err; exit 1; }
done
echo done
