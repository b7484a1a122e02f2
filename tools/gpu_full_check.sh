#!/bin/bash
# Round-end style validation on one GPU box: every -m gpu test, smoke(), the default
# bench line, and a kernel-trace profile of the default bench.
set -o pipefail
out=gpurun_out/full
mkdir -p $out
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread \
  -p no:cacheprovider > $out/gpu_tests.txt 2>&1 || exit $?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('SMOKE OK')" > $out/smoke.txt 2>&1 || exit $?
timeout -k 10 400 python bench.py > $out/bench.json 2> $out/bench.err || exit $?
