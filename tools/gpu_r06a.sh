#!/bin/bash
# r06 stage A: new GPU tests (stream split, blob tag), the --streams A/B at cfg2 / cfg3's
# per-GPU shards (bench.py, 3 interleaved repeats), a kernel trace of the S = 4 run.
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r06a
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
  tests/test_gpu_streams.py tests/test_gpu_blob_tag.py > $O/tests.txt 2>&1 || { echo TESTS FAILED; tail -30 $O/tests.txt; exit 1; }
tail -3 $O/tests.txt
for rep in 1 2 3; do
  for n in 131072 65536; do
    for S in 1 2 4; do
      timeout -k 10 120 python bench.py --envs $n --streams $S --no-cpu-baseline --no-drift --no-extras \
        > $O/bench_${n}_s${S}_r${rep}.json 2> $O/bench_${n}_s${S}_r${rep}.err || { echo BENCH FAILED $n $S; tail -5 $O/bench_${n}_s${S}_r${rep}.err; exit 1; }
      python -c "import json;d=json.load(open('$O/bench_${n}_s${S}_r${rep}.json'));print($n,$S,'%.3e'%d['value'],'us/step %.3f'%(d['ms_per_step']*1e3),'ev %.3f'%d['roofline']['avg_launch_us'],'med %.3f'%d['timing']['window_ms_median'])"
    done
  done
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 180 rocprofv3 --kernel-trace -d $GRAFT_REPO_ROOT/$O/trace_s4 -o trace -- \
  python3 $GRAFT_REPO_ROOT/bench.py --envs 131072 --streams 4 --steps 256 --warmup 64 --no-cpu-baseline --no-drift --no-extras \
  > $GRAFT_REPO_ROOT/$O/trace_s4.json 2> $GRAFT_REPO_ROOT/$O/trace_s4.err || { echo TRACE FAILED; tail -5 $GRAFT_REPO_ROOT/$O/trace_s4.err; exit 1; }
echo done
