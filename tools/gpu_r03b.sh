#!/bin/bash
# Round 3: the whole -m gpu suite at HEAD (multi-handle resident server, indexed state,
# cfg4 device-noise tails, cfg3 shard geometry, f32 attention, SB3-exact VecNormalize),
# the drop-in latency table and the default bench line.  A test FAILURE (pytest exit 1)
# lets the next step run; anything else (timeout, abort, fault) ends the script.
set -u
export TMPDIR=/tmp
O=gpurun_out/r03b
mkdir -p $O
ok() { local s=$1; [ $s -eq 0 ] || [ $s -eq 1 ] || exit $s; }
timeout -k 10 1000 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests \
  -s > $O/tests_gpu.txt 2>&1; ok $?
timeout -k 10 240 python -u tools/single_env_latency.py > $O/single_env_latency.json 2> $O/single_env_latency.log || exit 1
timeout -k 10 300 python bench.py > $O/bench_default.json 2> $O/bench_default.log || exit 1
