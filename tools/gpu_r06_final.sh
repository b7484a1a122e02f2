#!/bin/bash
# r06 closing run on the final tree: every GPU test, smoke, the default bench line, the
# driver's --steps 20 line, the headline's rocprof kernel-trace summary, the driver-style
# torchrun launch at world size 1, and cfg5 / cfg4 lines.
set -o pipefail
cd "$(dirname "$0")/.."
O=${O:-gpurun_out/r06_final2}
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 1000 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests \
  > $O/gpu_tests.txt 2>&1 || { echo TESTS FAILED; grep -E "FAILED|Error" $O/gpu_tests.txt | head; tail -20 $O/gpu_tests.txt; exit 1; }
tail -1 $O/gpu_tests.txt
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('SMOKE OK')" > $O/smoke.txt 2>&1 || { echo SMOKE FAILED; tail $O/smoke.txt; exit 1; }
tail -1 $O/smoke.txt
timeout -k 10 400 python bench.py > $O/bench_default.json 2> $O/bench_default.err || { echo BENCH FAILED; tail $O/bench_default.err; exit 1; }
timeout -k 10 200 python bench.py --steps 20 --warmup 5 > $O/bench_steps20.json 2> $O/bench_steps20.err || exit 1
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
  --master-port 29517 bench.py --gpus 1 --steps 400 --warmup 40 > $O/torchrun_n1.json 2> $O/torchrun_n1.err || exit 1
for m in "rollout --envs 32768 --K 2048 --system lorenz3" "rollout --envs 32768 --K 2048 --system pmsm" \
         "rollout --envs 32768 --K 2048 --system hr" "step --envs 262144 --system pmsm" "step --envs 262144 --system lorenz3"; do
  name=$(echo $m | tr ' ' '_' | tr -d '-')
  timeout -k 10 200 python bench.py --mode $m --no-cpu-baseline --no-drift --no-extras > $O/$name.json 2> $O/$name.err || { echo FAILED $m; exit 1; }
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof -o run --output-format csv \
  -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --no-drift > $GRAFT_REPO_ROOT/$O/bench_prof.json 2> $GRAFT_REPO_ROOT/$O/bench_prof.err || exit 1
echo done
