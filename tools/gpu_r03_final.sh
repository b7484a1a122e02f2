#!/bin/bash
# Round 3 closing validation at HEAD: every -m gpu test, smoke(), the default bench line
# (with CPU baseline, fp32 drift and the fp64 extra line), the driver's short setting,
# and a kernel-trace profile of the default bench command.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03_final
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread \
  -p no:cacheprovider > $O/gpu_tests.txt 2>&1 || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('SMOKE OK')" > $O/smoke.txt 2>&1 || exit 1
timeout -k 10 400 python bench.py > $O/bench_default.json 2> $O/bench_default.err || exit 1
timeout -k 10 200 python bench.py --steps 20 --warmup 5 > $O/bench_steps20.json 2> $O/bench_steps20.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/default.trace -o run --output-format csv -- python bench.py --no-cpu-baseline --no-extras > $O/default.trace.log 2>&1 || exit 1
